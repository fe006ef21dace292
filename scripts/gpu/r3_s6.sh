#!/bin/bash
# residual-join bit masks: bitwise test, full GPU tier, A/B at 1 / 8 configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s6
timeout -k 10 300 python -u -m pytest tests/test_bitmask_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3s6/bitmask.log 2>&1 || { tail -30 gpurun_out/r3s6/bitmask.log; exit 1; }
tail -1 gpurun_out/r3s6/bitmask.log
bash scripts/gpu/gpu_tier.sh r3s6 || exit $?
bash scripts/gpu/ab.sh bitmask "CER_BN_BITMASK=0 CER_BN_BITMASK=1" "1 8" 2
