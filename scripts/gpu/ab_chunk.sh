#!/bin/bash
# batched wgrads launched in chunks on the side stream (CER_WGB_CHUNK): graph test + bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chunk
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/chunk/tests.log 2>&1 || { tail -40 gpurun_out/chunk/tests.log; exit 1; }
tail -1 gpurun_out/chunk/tests.log
for R in 1 2; do
for C in 0 8 16 27; do
  CER_WGB_CHUNK=$C timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/chunk/b1_c${C}_r$R.json 2> gpurun_out/chunk/b1_c${C}_r$R.err || exit $?
  echo "1cfg chunk=$C: $(tail -1 gpurun_out/chunk/b1_c${C}_r$R.json | cut -c1-150)"
  CER_WGB_CHUNK=$C timeout -k 10 300 python -u bench.py > gpurun_out/chunk/b8_c${C}_r$R.json 2> gpurun_out/chunk/b8_c${C}_r$R.err || exit $?
  echo "8cfg chunk=$C: $(tail -1 gpurun_out/chunk/b8_c${C}_r$R.json | cut -c1-150)"
done
done
