#!/bin/bash
# round 4: numerics of the wave-specialised kernels, then a same-box A/B of
# the driver-shape bench (8 configs and 1) with them off / wgrad only / all
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4ws
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -k "wave_specialised or wgrad_batch" \
  -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" $O/tests.log | head -20; exit $rc; fi
for V in "CER_FP32_WS=0,CER_WGB_WS=0" "CER_FP32_WS=0,CER_WGB_WS=1" "CER_FP32_WS=1,CER_WGB_WS=1"; do
  for C in 8 1; do
    F="$O/b_${V//[,=]/_}_c$C"
    env ${V//,/ } CER_TUNE_LOG=$F.tune.json timeout -k 10 300 python -u bench.py --configs $C \
      > $F.json 2> $F.err || { tail -5 $F.err; exit 1; }
    echo "$V c$C $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
  done
done
