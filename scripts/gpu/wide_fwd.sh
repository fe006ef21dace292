#!/bin/bash
# wide (32x32x16) fp32 conv kernels: numerics, per-shape sweep, 8/1-config bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wide
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/wide/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/wide/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q -k "wide" --timeout 120 --timeout-method thread > gpurun_out/wide/tests.log 2>&1 || { tail -40 gpurun_out/wide/tests.log; exit 1; }
tail -2 gpurun_out/wide/tests.log
timeout -k 10 400 python -u -m cerebro_ds_kpgi_amd.tools.bench_conv --sweep --dtype fp32 --iters 10 --json gpurun_out/wide/sweep_c8.json > gpurun_out/wide/sweep_c8.txt 2>&1 || exit $?
grep SWEEP_TOTAL gpurun_out/wide/sweep_c8.txt
timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.bench_conv --sweep --dtype fp32 --iters 10 --G 1 --json gpurun_out/wide/sweep_c1.json > gpurun_out/wide/sweep_c1.txt 2>&1 || exit $?
grep SWEEP_TOTAL gpurun_out/wide/sweep_c1.txt
for R in 1 2; do
for CFG in "1 1" "0 1" "1 13"; do
  set -- $CFG
  CER_FP32_WIDE=$1 CER_WGB_VARIANT=$2 timeout -k 10 300 python -u bench.py > gpurun_out/wide/b8_w$1_g$2_r$R.json 2> gpurun_out/wide/b8_w$1_g$2_r$R.err || exit $?
  echo "8cfg wide=$1 wgb=$2: $(tail -1 gpurun_out/wide/b8_w$1_g$2_r$R.json | cut -c1-160)"
  CER_FP32_WIDE=$1 CER_WGB_VARIANT=$2 timeout -k 10 300 python -u bench.py --configs 1 > gpurun_out/wide/b1_w$1_g$2_r$R.json 2> gpurun_out/wide/b1_w$1_g$2_r$R.err || exit $?
  echo "1cfg wide=$1 wgb=$2: $(tail -1 gpurun_out/wide/b1_w$1_g$2_r$R.json | cut -c1-160)"
done
done
