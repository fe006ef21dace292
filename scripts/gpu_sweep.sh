#!/bin/bash
# Conv numerics under every pinned variant + per-shape variant sweep.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-sweep}
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -x -q -k "conv_matches or variant" > gpurun_out/pytest_conv_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_conv_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^E|FAILED|Error" gpurun_out/pytest_conv_$TAG.log | head -30; exit 1; fi
timeout -k 10 600 python -m cerebro_ds_kpgi_amd.tools.bench_conv --G 8 --B 32 --sweep --json gpurun_out/sweep_$TAG.json > gpurun_out/sweep_$TAG.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/sweep_$TAG.log; exit 1; }
echo sweep ok
