#!/bin/bash
# depthwise dgrad BN link (expansion BN partials in the depthwise dgrad):
# numerics tests, then MobileNetV2 A/B (CER_DW_BNLINK=0: the BN's own pass)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s13
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwstats_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py \
  -k "dwconv or bn_link or mobilenet or graph" -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_ARGS="--model mobilenetv2" bash scripts/gpu/ab.sh dwlink "CER_DW_BNLINK=0 CER_DW_BNLINK=1" "8 1" 2
