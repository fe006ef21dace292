#!/bin/bash
# ring wgrad + step-glue changes: ring numerics, the full GPU tier, then
# 8- / 1-config bench with the ring off / on (same box)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-wgring}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_wgring_gpu.py > $O/ring_tests.log 2>&1
RC=$?
grep -E "passed|failed|Error|ring [0-9]" $O/ring_tests.log | tail -12
[ $RC -ne 0 ] && exit $RC
bash scripts/gpu/gpu_tier.sh $1
TRC=$?
if [ $TRC -ne 0 ] && [ $TRC -ne 1 ]; then exit $TRC; fi
for R in 0 2 0 2; do
  for C in 8 1; do
    CER_WGB_RING=$R timeout -k 10 300 python -u bench.py --configs $C > $O/c${C}_r$R.json 2> $O/c${C}_r$R.err || exit $?
    echo "ring=$R configs=$C: $(python3 -c "import json;d=json.load(open('$O/c${C}_r$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
exit $TRC
