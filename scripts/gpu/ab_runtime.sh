#!/bin/bash
# GPU tier + 1-GPU bench on the async runtime and an A/B against lock-step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/gpu/gpu_tier.sh "${1:-r2async}" || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench_async.json 2> gpurun_out/bench_async.err || exit $?
cat gpurun_out/bench_async.json
CER_RUNTIME=lockstep timeout -k 10 300 python -u bench.py > gpurun_out/bench_lockstep.json 2> gpurun_out/bench_lockstep.err || exit $?
cat gpurun_out/bench_lockstep.json
