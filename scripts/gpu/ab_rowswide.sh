#!/bin/bash
# per-pack wgrad batch rows (CER_WGB_ROWS_WIDE for packs >= 4 configs) A/B + tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rowswide
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_fp32_gpu.py -k "graph or wgrad_batch or trajectory" -x -q --timeout 200 --timeout-method thread > gpurun_out/rowswide/tests.log 2>&1 || { tail -40 gpurun_out/rowswide/tests.log; exit 1; }
tail -1 gpurun_out/rowswide/tests.log
for R in 1 2; do
for W in 2048 1024; do
  for C in 8 4 1; do
    CER_WGB_ROWS_WIDE=$W timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/rowswide/b${C}_w${W}_$R.json 2> gpurun_out/rowswide/b${C}_w${W}_$R.err || exit $?
    echo "cfg=$C rows_wide=$W: $(python -c "import json;d=json.load(open('gpurun_out/rowswide/b${C}_w${W}_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
