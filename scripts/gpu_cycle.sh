#!/bin/bash
# One measurement cycle: GPU tests -> headline bench (8 cfg) -> 1-config bench -> rocprof of both.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-cyc}
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ]; then grep -E "^E|FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head -30; exit 1; fi
fi
for C in 8 1; do
  timeout -k 10 300 python bench.py --configs $C > gpurun_out/bench_${TAG}_c$C.log 2>&1 || { echo "bench c$C failed"; tail -30 gpurun_out/bench_${TAG}_c$C.log; exit 1; }
  echo "configs=$C $(tail -1 gpurun_out/bench_${TAG}_c$C.log | cut -c1-190)"
done
for C in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c$C -o prof -- python3 bench.py --configs $C --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/prof_${TAG}_c$C.log 2>&1 || { echo "rocprof c$C failed"; exit 1; }
done
echo done
