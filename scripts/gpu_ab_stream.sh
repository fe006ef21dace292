#!/bin/bash
# GPU tests, then headline and 1-config bench with / without the wgrad side stream.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^E|FAILED" gpurun_out/pytest_gpu_$TAG.log | head -20; exit 1; fi
for S in 1 0; do
  for C in 8 1; do
    CER_WGRAD_STREAM=$S timeout -k 10 300 python bench.py --configs $C > gpurun_out/bench_${TAG}_s${S}_c${C}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_s${S}_c${C}.log; exit 1; }
    echo "stream=$S configs=$C $(tail -1 gpurun_out/bench_${TAG}_s${S}_c${C}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
