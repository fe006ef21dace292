#!/bin/bash
# fp32 numerics tests + rocprofv3 kernel stats of the fp32 headline step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-fp32}
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/fp32_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/fp32_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o prof -- python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?"
tail -1 gpurun_out/prof_$TAG.log
