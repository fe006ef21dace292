#!/bin/bash
# Round 6: N = 4 rehearsal on one GPU (gloo data plane, 4 ranks x 2 configs:
# the HL weight image is on at G = 2, so hops must refresh it).  Checks that
# every job's loss after the hop is finite and in the range of the ones
# before it.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6n4
rm -rf "$OUT"; mkdir -p "$OUT/logs"
timeout -k 10 600 env CER_DIST_BACKEND=gloo CER_ALLOW_DEVICE_WRAP=1 python -u -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 \
  --steps 10 --warmup 0 --steps_per_round 5 --logs_root "$OUT/logs" > "$OUT/n4.log" 2>&1 || { tail -30 "$OUT/n4.log"; exit 1; }
grep '^{' "$OUT/n4.log" | tail -1
python3 - "$OUT/logs/metrics.jsonl" <<'PY' || exit 1
import json, math, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
jobs = [r for r in recs if r.get("kind") == "job"]
hops = [r for r in recs if r.get("kind") == "hop"]
print("jobs", len(jobs), "hops", len(hops))
for r in jobs:
    print(r["epoch"], r["subepoch"], r["rank"], r["cfg"][:34], round(r["loss"], 3), r.get("hop_ms"))
assert hops and all(math.isfinite(r["loss"]) and r["loss"] < 20 for r in jobs)
PY
