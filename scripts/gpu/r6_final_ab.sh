#!/bin/bash
# Round 6 end: whole-build A/B of the round-4 end build (abtree/r4 =
# `git archive 75bda2a`, built in place) against this tree on the headline,
# the one-config headline and criteo16 (2 alternating rounds), then the N = 2
# rehearsal of the multi-rank path with telemetry (gloo on one GPU).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/ab_trees.sh r4r6 "abtree/r4 ." 2 "headline c1 criteo16" || exit 1
OUT=$PWD/gpurun_out/r6final_n2
mkdir -p "$OUT/logs"
timeout -k 10 300 env CER_DIST_BACKEND=gloo CER_ALLOW_DEVICE_WRAP=1 python -u -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 \
  --steps 10 --warmup 0 --steps_per_round 5 --logs_root "$OUT/logs" > "$OUT/n2.log" 2>&1 || { tail -20 "$OUT/n2.log"; exit 1; }
grep '^{' "$OUT/n2.log" | tail -1
ls "$OUT/logs" "$OUT/logs/sys_logs"
