#!/bin/bash
# grouped conv numerics + resnext101 under a graph, then the DA at-scale run
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3grp
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  -k "grouped or resnext" > gpurun_out/r3grp/tests.log 2>&1
rc=$?
grep -E "grouped \(|PASSED|FAILED|passed|failed|Error" gpurun_out/r3grp/tests.log | tail -16
exit $rc
