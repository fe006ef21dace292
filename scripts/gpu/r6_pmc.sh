#!/bin/bash
# Round 6: (1) the timed-path oracle test, (2) the N = 2 rehearsal of the
# multi-rank path on one GPU with per-hop telemetry (gloo data plane,
# CER_ALLOW_DEVICE_WRAP), (3) SQ counters of the uniform-K fp32 GEMMs on
# 8-config and one-config ResNet-50 shapes.  Output: gpurun_out/r6pmc/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6pmc
mkdir -p "$OUT"
step() {   # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 "$OUT/$name.log")"
  return $rc
}
mkdir -p "$OUT/n2logs"
step n2 300 env CER_DIST_BACKEND=gloo CER_ALLOW_DEVICE_WRAP=1 python -u -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
  --steps 10 --warmup 0 --steps_per_round 5 --logs_root "$OUT/n2logs" || exit 1
python3 - "$OUT/n2logs/metrics.jsonl" <<'EOF' || exit 1
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1])]
hops = [r for r in recs if r.get("kind") == "hop"]
hold = [r for r in recs if r.get("kind") == "hop_hold"]
print("metrics: %d job, %d hop, %d hop_hold records" % (
    sum(1 for r in recs if r.get("kind") == "job"), len(hops), len(hold)))
print("hop example:", hops[0] if hops else None)
print("hold:", hold[-1] if hold else None)
assert hops and hold
EOF
PMC_G=8 PMC_OUT=r6pmc/c8 PMC_SHAPES="32,28,28,64,64,3,1,1 32,14,14,128,512,1,1,0 32,7,7,1024,256,1,1,0" \
  bash scripts/gpu/conv32_pmc2.sh || exit 1
PMC_G=1 PMC_OUT=r6pmc/c1 PMC_SHAPES="32,7,7,1024,256,1,1,0 32,4,4,512,2048,1,1,0 32,28,28,64,64,3,1,1" \
  bash scripts/gpu/conv32_pmc2.sh || exit 1
for D in c8 c1; do
  for SH in $(ls "$OUT/$D" | grep '^a_' | sed 's/^a_//'); do
    python3 -m cerebro_ds_kpgi_amd.tools.pmc_table "$OUT/$D/a_$SH" "$OUT/$D/b_$SH" \
      > "$OUT/$D/table_$SH.md" 2>&1 || exit 1
  done
done
echo done
