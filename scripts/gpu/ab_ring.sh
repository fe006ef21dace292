#!/bin/bash
# fp32 LDS-DMA ring forward kernels: numerics (pinned variants), then bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_ring
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q -s --timeout 300 --timeout-method thread -k "ring or conv_fp32" > gpurun_out/ab_ring/tests.log 2>&1 || { grep -E "ring fwd|Error|error|assert" gpurun_out/ab_ring/tests.log | tail -30; exit 1; }
grep -E "ring fwd" gpurun_out/ab_ring/tests.log | sort -t'e' -k1 | tail -40
tail -1 gpurun_out/ab_ring/tests.log
bash scripts/gpu/ab_env.sh "CER_FP32_RING=0 CER_FP32_RING=1"
