#!/bin/bash
# GPU pass: kernel numerics, then bench (HIP kernels / torch oracle), then rocprof.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -x -v > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -45
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed (rc=$rc), stopping"; exit 1; fi
echo "== bench hip"; date
timeout -k 10 500 python bench.py --steps 30 --warmup 10 --steps_per_round 10 > gpurun_out/bench_hip.log 2>&1 || { echo "bench hip failed"; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -1 gpurun_out/bench_hip.log
echo "== bench torch"; date
timeout -k 10 500 python bench.py --steps 30 --warmup 10 --steps_per_round 10 --backend torch > gpurun_out/bench_torch.log 2>&1 || { echo "bench torch failed"; tail -30 gpurun_out/bench_torch.log; exit 1; }
tail -1 gpurun_out/bench_torch.log
echo "== rocprof"; date
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o prof -- python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/prof4.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof4 -name "*stats*"
