#!/bin/bash
# side-stream wgrad chunks with a persistent capped grid (CER_WGB_CHUNK x CER_WGB_GRID)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chunk2
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_fp32_gpu.py -k "graph_replays or wgrad_batch" -x -q --timeout 120 --timeout-method thread > gpurun_out/chunk2/tests.log 2>&1 || { tail -40 gpurun_out/chunk2/tests.log; exit 1; }
tail -1 gpurun_out/chunk2/tests.log
for R in 1 2; do
for CFG in "0 0" "8 32" "8 64" "16 64" "8 128" "27 96"; do
  set -- $CFG
  for C in 1 8; do
    CER_WGB_CHUNK=$1 CER_WGB_GRID=$2 timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/chunk2/b${C}_c$1_g$2_$R.json 2> gpurun_out/chunk2/b${C}_c$1_g$2_$R.err || exit $?
    echo "cfg=$C chunk=$1 grid=$2: $(python -c "import json;d=json.load(open('gpurun_out/chunk2/b${C}_c$1_g$2_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
