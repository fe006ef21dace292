#!/bin/bash
# shortcut-branch stream: GPU tests + A/B; BN apply microbench; baseline makespans
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s3
timeout -k 10 600 python -u -m pytest tests/test_branch_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r3s3/branch_tests.log 2>&1 || { tail -30 gpurun_out/r3s3/branch_tests.log; exit 1; }
grep -E "passed|failed|rel diff" gpurun_out/r3s3/branch_tests.log | tail -5
bash scripts/gpu/ab.sh branch "CER_SC_BRANCH=0 CER_SC_BRANCH=1" "1 2 8" 2 || exit 1
for S in "1568 256 1" "1568 512 1" "392 1024 1" "25088 64 1" "25088 256 1" "1568 256 8" "25088 256 8"; do
  set -- $S
  timeout -k 10 120 python -m cerebro_ds_kpgi_amd.tools.bn_one --rows $1 --C $2 --G $3 \
    >> gpurun_out/r3s3/bn_one.jsonl 2> gpurun_out/r3s3/bn_one.err || { tail gpurun_out/r3s3/bn_one.err; exit 1; }
done
cat gpurun_out/r3s3/bn_one.jsonl
bash scripts/gpu/r3_baseline_makespan.sh
