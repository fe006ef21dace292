#!/bin/bash
# per-kernel HBM bytes (FETCH_SIZE / WRITE_SIZE, one counter group per pass)
# of the fp32 headline step: hbm_pmc.sh [configs]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
C=${1:-8}
mkdir -p gpurun_out/hbm_c$C
for CTR in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d gpurun_out/hbm_c$C/$CTR -o p -- \
    python3 bench.py --steps 4 --warmup 3 --steps_per_round 4 --configs $C --no_graphs \
    > gpurun_out/hbm_c$C/$CTR.log 2>&1 || { tail -20 gpurun_out/hbm_c$C/$CTR.log; exit 1; }
done
find gpurun_out/hbm_c$C -name "*.csv" | xargs ls -la
