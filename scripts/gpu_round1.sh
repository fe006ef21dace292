#!/bin/bash
# First GPU pass: gpu tests, bench (torch oracle vs partial HIP), rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest gpu"; date
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu.log
echo "== bench torch"; date
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --steps_per_round 10 --backend torch > gpurun_out/bench_torch.log 2>&1 || { echo "bench torch failed"; tail -30 gpurun_out/bench_torch.log; exit 1; }
tail -1 gpurun_out/bench_torch.log
echo "== bench hip"; date
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --steps_per_round 10 > gpurun_out/bench_hip.log 2>&1 || { echo "bench hip failed"; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -1 gpurun_out/bench_hip.log
echo "== rocprof"; date
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof -- python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/prof1.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof1 -name "*stats*" | head
