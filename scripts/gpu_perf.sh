#!/bin/bash
# Kernel numerics + conv microbench + headline bench + rocprof (one GPU box).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-perf}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^E|FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20; exit 1; fi
timeout -k 10 300 python -m cerebro_ds_kpgi_amd.tools.bench_conv --G 8 --B 32 --json gpurun_out/conv_$TAG.json > gpurun_out/conv_$TAG.log 2>&1 || { echo "conv bench failed"; tail -20 gpurun_out/conv_$TAG.log; exit 1; }
tail -1 gpurun_out/conv_$TAG.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --steps_per_round 10 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?"
