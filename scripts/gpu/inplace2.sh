#!/bin/bash
# in-place strided dgrad incl. BN-linked calls: tests, bench, HBM traffic
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/inplace2
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_fp32_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/inplace2/tests.log 2>&1 || { tail -40 gpurun_out/inplace2/tests.log; exit 1; }
tail -1 gpurun_out/inplace2/tests.log
for R in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/inplace2/b8_$R.json 2> gpurun_out/inplace2/b8_$R.err || exit $?
  echo "cfg=8: $(python -c "import json;d=json.load(open('gpurun_out/inplace2/b8_$R.json'));print(d['value'],d['ms_per_step'])")"
done
bash scripts/gpu/hbm_pmc.sh 8 > gpurun_out/inplace2/hbm.log 2>&1 || { tail -20 gpurun_out/inplace2/hbm.log; exit 1; }
echo hbm-done
