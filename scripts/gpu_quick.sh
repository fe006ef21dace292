#!/bin/bash
# Conv numerics + conv microbench + headline bench (no profiler).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -x -q > gpurun_out/pytest_conv_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_conv_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^E|FAILED" gpurun_out/pytest_conv_$TAG.log | head -20; exit 1; fi
timeout -k 10 300 python -m cerebro_ds_kpgi_amd.tools.bench_conv --G 8 --B 32 --json gpurun_out/conv_$TAG.json > gpurun_out/conv_$TAG.log 2>&1 || { echo "conv bench failed"; tail -20 gpurun_out/conv_$TAG.log; exit 1; }
tail -1 gpurun_out/conv_$TAG.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --steps_per_round 10 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
