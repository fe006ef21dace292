#!/bin/bash
# baselines on the GPU: tests, then 1-epoch MA / DDP / task-parallel / MOP at N = 1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3base
timeout -k 10 900 python -u -m pytest tests/test_baselines_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r3base/tests.log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|Error|segments" gpurun_out/r3base/tests.log | tail -12
exit $rc
