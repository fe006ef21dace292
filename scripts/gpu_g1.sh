#!/bin/bash
# Per-GPU work at N=8 (one config) with / without the conv-fused BN finalize.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-g1}
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --steps_per_round 10 --configs 1 > gpurun_out/bench_${TAG}_a.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_a.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_a.log
CER_BN_FUSED_FINALIZE=1 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --steps_per_round 10 --configs 1 > gpurun_out/bench_${TAG}_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_b.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_b.log
CER_BN_FUSED_FINALIZE=1 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --steps_per_round 10 > gpurun_out/bench_${TAG}_c.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_c.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}_c.log
