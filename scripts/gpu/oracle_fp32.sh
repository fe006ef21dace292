#!/bin/bash
# the same fp32 headline step on the PyTorch-ROCm / MIOpen oracle backend (eager) for comparison
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/oracle
timeout -k 10 600 python -u bench.py --backend torch --steps 20 --warmup 5 > gpurun_out/oracle/c8.json 2> gpurun_out/oracle/c8.err || exit $?
cat gpurun_out/oracle/c8.json | cut -c1-220
timeout -k 10 600 python -u bench.py --backend torch --configs 1 --steps 20 --warmup 5 > gpurun_out/oracle/c1.json 2> gpurun_out/oracle/c1.err || exit $?
cat gpurun_out/oracle/c1.json | cut -c1-220
