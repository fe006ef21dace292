#!/bin/bash
# round 4 debug: depthwise fused-vs-plain forward difference (dwb twin),
# the lanes test with its noise floor printed, the depthwise tests on the twin
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4dbg
mkdir -p $O
PYTHONPATH=. CER_HIP_LIB=libcerebro_hip_dwb.so timeout -k 10 120 python -u scripts/dev/dw_diff.py > $O/dw_diff.log 2>&1 || { tail -20 $O/dw_diff.log; exit 1; }
cat $O/dw_diff.log
timeout -k 10 400 python -u -m pytest tests/test_lanes_gpu.py -x -q -s --timeout 380 --timeout-method thread > $O/lanes.log 2>&1
rc=$?
grep -E "group|passed|failed|Error" $O/lanes.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CER_HIP_LIB=libcerebro_hip_dwb.so timeout -k 10 600 python -u -m pytest tests/test_dwstats_gpu.py tests/test_conv_gpu.py -k "dw" -q \
  --timeout 120 --timeout-method thread > $O/dwtests.log 2>&1
grep -E "FAILED|passed|failed" $O/dwtests.log | head -30
