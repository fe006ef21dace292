#!/bin/bash
# fp32 bring-up: numerics tests, smoke, short bench (exit early on a crash)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/fp32_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 5 > gpurun_out/bench_fp32.log 2>&1 || exit $?
tail -2 gpurun_out/bench_fp32.log
