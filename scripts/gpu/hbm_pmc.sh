#!/bin/bash
# per-kernel HBM bytes (FETCH_SIZE / WRITE_SIZE, one counter group per pass)
# of the fp32 headline step: hbm_pmc.sh [configs]
# (BENCH_ARGS="--model vgg16" HBM_TAG=_vgg for another model)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
C=${1:-8}
D=gpurun_out/hbm_c$C$HBM_TAG
mkdir -p $D
for CTR in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $D/$CTR -o p -- \
    python3 bench.py --steps 4 --warmup 3 --steps_per_round 4 --configs $C $BENCH_ARGS --no_graphs \
    > $D/$CTR.log 2>&1 || { tail -20 $D/$CTR.log; exit 1; }
done
find $D -name "*.csv" | xargs ls -la
