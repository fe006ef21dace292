#!/bin/bash
# round 4: concurrent pack groups (lanes) + pack-aware order on the 48-config
# hetero drill-down: the lanes numerics test, then the CTQ / UDAF jobs with
# lanes (default 4) and with --lanes 1 (pack order only)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4sec
timeout -k 10 400 python -u -m pytest tests/test_lanes_gpu.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r4sec/lanes_test.log 2>&1
rc=$?
tail -3 gpurun_out/r4sec/lanes_test.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" gpurun_out/r4sec/lanes_test.log | head -20; exit $rc; fi
timeout -k 10 120 python3 -u scripts/dev/lanes_overlap.py > gpurun_out/r4sec/lanes_overlap.json 2>&1 || exit 1
cat gpurun_out/r4sec/lanes_overlap.json
bash scripts/gpu/secondary.sh hetero_jobs lanes || exit 1
bash scripts/gpu/secondary.sh hetero_jobs packserial --lanes 1 || exit 1
