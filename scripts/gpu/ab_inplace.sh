#!/bin/bash
# strided-1x1 dgrad accumulating into the GradJoin addend in place: tests + bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/inplace
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_fp32_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/inplace/tests.log 2>&1 || { tail -40 gpurun_out/inplace/tests.log; exit 1; }
tail -1 gpurun_out/inplace/tests.log
for R in 1 2; do
  for C in 8 1; do
    timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/inplace/b${C}_$R.json 2> gpurun_out/inplace/b${C}_$R.err || exit $?
    echo "cfg=$C: $(python -c "import json;d=json.load(open('gpurun_out/inplace/b${C}_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
