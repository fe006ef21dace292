#!/bin/bash
# GPU tests, then bench (8 cfg, 1 cfg) with an env knob on / off:  gpu_ab_env.sh TAG VAR
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}; VAR=${2:-CER_BN_COOP}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ]; then grep -E "^E|FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head -30; exit 1; fi
fi
for V in 1 0; do
  for C in 8 1; do
    env $VAR=$V timeout -k 10 300 python bench.py --configs $C > gpurun_out/bench_${TAG}_v${V}_c${C}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_v${V}_c${C}.log; exit 1; }
    echo "$VAR=$V configs=$C $(tail -1 gpurun_out/bench_${TAG}_v${V}_c${C}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
