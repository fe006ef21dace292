#!/bin/bash
# Round 6: bisect the round-5 headline drift, the lanes
# default on criteo16, and the per-shape fp32 conv table of the HEAD build
# (baseline for the GM_GEMM / HL-weight kernel work).  Output under
# gpurun_out/r6b/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6b
mkdir -p "$OUT"
bash scripts/gpu/ab_trees.sh bisect \
  "abtree/r4 abtree/34bea3c abtree/a876166 abtree/ee648c5 abtree/d42ec09 abtree/fe2d148 ." \
  2 headline || exit 1
for R in 1 2; do
  for L in 1 4; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --workload criteo16 \
      --lanes $L > "$OUT/criteo_l${L}_$R.json" 2> "$OUT/criteo_l${L}_$R.err" || exit 1
    echo "criteo16 lanes $L r$R $(python3 -c "import json;d=json.load(open('$OUT/criteo_l${L}_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
for G in 8 1; do
  timeout -k 10 600 python -u -m cerebro_ds_kpgi_amd.tools.bench_conv --dtype fp32 --G $G \
    --no_miopen --iters 20 --json "$OUT/conv_g$G.json" > "$OUT/conv_g$G.log" 2>&1 || exit 1
  tail -1 "$OUT/conv_g$G.log"
done
