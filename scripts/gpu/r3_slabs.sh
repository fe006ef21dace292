#!/bin/bash
# atomic BN-statistics slabs: numerics tiers, then a same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3slabs
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py tests/test_graph_gpu.py tests/test_conv_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3slabs/tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r3slabs/tests.log | head -20; tail -5 gpurun_out/r3slabs/tests.log; exit 1; }
tail -1 gpurun_out/r3slabs/tests.log
bash scripts/gpu/ab.sh slabs "CER_BN_ATOMIC_SLABS=0 CER_BN_ATOMIC_SLABS=8" "1 8" 2
