#!/bin/bash
# GPU tests, headline bench, 1-config bench (the per-GPU work at N=8), and a
# rocprofv3 kernel-trace of the 1-config step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-s3}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^E|FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20; exit 1; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 300 python bench.py --configs 1 > gpurun_out/bench_${TAG}_c1.log 2>&1 || { echo "bench c1 failed"; tail -30 gpurun_out/bench_${TAG}_c1.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c1.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c1 -o prof -- python3 bench.py --configs 1 --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/prof_${TAG}_c1.log 2>&1
echo "rocprof rc=$?"
