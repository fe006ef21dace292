#!/bin/bash
# adaptive side-stream wgrad split (packs >= CER_WGB_SIDE_MIN_G configs): k = 1/frac side batches
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sidefrac
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sidefrac/tests.log 2>&1 || { tail -40 gpurun_out/sidefrac/tests.log; exit 1; }
tail -1 gpurun_out/sidefrac/tests.log
for R in 1 2; do
for CFG in "0.5 96" "0.4 96" "0.6 96" "0.5 128" "0 96"; do
  set -- $CFG
  for C in 8 4; do
    CER_WGB_SIDE_FRAC=$1 CER_WGB_SPLIT_GRID=$2 timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/sidefrac/b${C}_f$1_g$2_$R.json 2> gpurun_out/sidefrac/b${C}_f$1_g$2_$R.err || exit $?
    echo "cfg=$C frac=$1 grid=$2: $(python -c "import json;d=json.load(open('gpurun_out/sidefrac/b${C}_f$1_g$2_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
CER_WGB_SIDE_MIN_G=1 timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/sidefrac/b1_on_$R.json 2> gpurun_out/sidefrac/b1_on_$R.err || exit $?
echo "cfg=1 frac=0.5 (forced): $(python -c "import json;d=json.load(open('gpurun_out/sidefrac/b1_on_$R.json'));print(d['value'],d['ms_per_step'])")"
timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/sidefrac/b1_off_$R.json 2> gpurun_out/sidefrac/b1_off_$R.err || exit $?
echo "cfg=1 default (off below 4): $(python -c "import json;d=json.load(open('gpurun_out/sidefrac/b1_off_$R.json'));print(d['value'],d['ms_per_step'])")"
done
