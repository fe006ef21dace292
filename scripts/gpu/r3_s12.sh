#!/bin/bash
# standalone-BN link (MobileNetV2 depthwise BN -> projection dgrad epilogue):
# numerics tests, MobileNetV2 model tests, then MobileNetV2 rates
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwstats_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py \
  -k "dwconv or bn_link or mobilenet or graph" -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_ARGS="--model mobilenetv2" bash scripts/gpu/ab.sh bnlink "CER_NONE=0" "8 1" 2
