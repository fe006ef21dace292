#!/bin/bash
# fused depthwise + BN statistics: size threshold sweep on MobileNetV2
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwstats_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3s11_tests.log 2>&1 || { tail -30 gpurun_out/r3s11_tests.log; exit 1; }
tail -1 gpurun_out/r3s11_tests.log
AB_ARGS="--model mobilenetv2" bash scripts/gpu/ab.sh dwmin \
  "CER_DW_STATS=0 CER_DW_STATS_MIN=0 CER_DW_STATS_MIN=4194304 CER_DW_STATS_MIN=16777216" "8 1" 2
