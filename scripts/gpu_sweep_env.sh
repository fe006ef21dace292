#!/bin/bash
# GPU tests (unless SKIP_TESTS=1), then bench.py under a list of env settings:
#   gpu_sweep_env.sh TAG "CONFIGS" "ENV1" "ENV2" ...   (ENV = space-separated VAR=VAL list)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; CONFIGS=$2; shift 2
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ]; then grep -E "^E|FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head -30; exit 1; fi
fi
i=0
for E in "$@"; do
  for C in $CONFIGS; do
    f=gpurun_out/bench_${TAG}_${i}_c${C}.log
    env $E timeout -k 10 300 python bench.py --configs $C > $f 2>&1 || { echo "bench failed: $E c$C"; tail -20 $f; exit 1; }
    echo "[$E] configs=$C $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
  i=$((i+1))
done
