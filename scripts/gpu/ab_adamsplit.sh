#!/bin/bash
# Adam split across streams with the side wgrad batch: numerics + A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/adamsplit
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/adamsplit/tests.log 2>&1 || { tail -40 gpurun_out/adamsplit/tests.log; exit 1; }
grep -E "split at|passed|failed" gpurun_out/adamsplit/tests.log | tail -3
for R in 1 2; do
for S in 1 0; do
  for C in 8 4; do
    CER_ADAM_SPLIT=$S timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/adamsplit/b${C}_s${S}_$R.json 2> gpurun_out/adamsplit/b${C}_s${S}_$R.err || exit $?
    echo "cfg=$C adam_split=$S: $(python -c "import json;d=json.load(open('gpurun_out/adamsplit/b${C}_s${S}_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
