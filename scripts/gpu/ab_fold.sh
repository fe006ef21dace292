#!/bin/bash
# BN apply folded into the consumer conv (fp32): numerics, then bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_fold
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/ab_fold/tests.log 2>&1 || { tail -40 gpurun_out/ab_fold/tests.log; exit 1; }
grep -E "bn fold|passed|trajectory" gpurun_out/ab_fold/tests.log | tail -6
for R in 1 2; do
  for F in 0 1; do
    for C in 8 1; do
      CER_BN_FOLD_APPLY=$F timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/ab_fold/b_f${F}_c${C}_$R.json 2>/dev/null || exit $?
      echo "fold=$F c$C $(python3 -c "import json;d=json.load(open('gpurun_out/ab_fold/b_f${F}_c${C}_$R.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
