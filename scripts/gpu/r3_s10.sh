#!/bin/bash
# depthwise fwd + BN statistics: numerics tests, then MobileNetV2 A/B
# (CER_DW_STATS=0: the BN's own statistics pass) at 8 and 1 configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwstats_gpu.py tests/test_conv_gpu.py tests/test_fp32_gpu.py \
  tests/test_kernels_gpu.py -k "dwstats or dwconv or mobilenet or stats_matches" -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_ARGS="--model mobilenetv2" bash scripts/gpu/ab.sh dwstats "CER_DW_STATS=0 CER_DW_STATS=1" "8 1" 2
