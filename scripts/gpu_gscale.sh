#!/bin/bash
# Per-GPU throughput at the packing of N = 8/K GPUs (K configs on one GPU).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-gs}
for K in 1 2 4; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --steps_per_round 10 --configs $K > gpurun_out/bench_${TAG}_c$K.log 2>&1 || { echo "bench K=$K failed"; tail -20 gpurun_out/bench_${TAG}_c$K.log; exit 1; }
  tail -1 gpurun_out/bench_${TAG}_c$K.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c1 -o prof -- python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 --configs 1 > gpurun_out/prof_${TAG}_c1.log 2>&1
echo "rocprof rc=$?"
