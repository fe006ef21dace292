#!/bin/bash
# stem / pointwise BN links into the depthwise dgrads (MobileNetV1/V2):
# model-family GPU tests, then MobileNetV2 / V1 rates
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s15
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwstats_gpu.py tests/test_kernels_gpu.py tests/test_graph_gpu.py \
  tests/test_fp32_gpu.py -k "dwconv or bn_link or mobilenet or graph" -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_ARGS="--model mobilenetv2" bash scripts/gpu/ab.sh stemlink "CER_NONE=0" "8 1" 2 || exit $?
AB_ARGS="--model mobilenetv1" bash scripts/gpu/ab.sh mbv1 "CER_DW_BNLINK=0 CER_DW_BNLINK=1" "8" 2
