#!/bin/bash
# pre-split fp32 weight image (Arena.wsplit): numerics, then bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_ws
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/ab_ws/tests.log 2>&1 || { tail -40 gpurun_out/ab_ws/tests.log; exit 1; }
grep -E "presplit|passed|trajectory" gpurun_out/ab_ws/tests.log | tail -8
for R in 1 2; do
  for S in 0 1; do
    for C in 8 1; do
      CER_W_SPLIT=$S timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/ab_ws/b_s${S}_c${C}_$R.json 2>/dev/null || exit $?
      echo "wsplit=$S c$C $(python3 -c "import json;d=json.load(open('gpurun_out/ab_ws/b_s${S}_c${C}_$R.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
