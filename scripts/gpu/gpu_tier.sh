#!/bin/bash
# full GPU test tier (the driver's round-end command shape), log per run
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-tier}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_$TAG.log | tail -3
grep -E "FAILED|^E " gpurun_out/gpu_$TAG.log | head -20
exit $rc
