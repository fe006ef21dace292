#!/bin/bash
# multi-rank rehearsal on one GPU (2 ranks, gloo data plane) with the final
# build; SQ counters of the one-config step (BN apply fwd vs bwd in context)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/rehearse_n2.sh
O=gpurun_out/r3s8
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d $O/pmc -o p -- python3 bench.py --configs 1 --steps 3 --warmup 1 --steps_per_round 4 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
tail -1 $O/pmc.log
python3 - <<'PY' > $O/pmc_bn.md
import csv, glob, collections
rows = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/r3s8/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        e = rows[int(r["Dispatch_Id"])]
        e["name"] = r["Kernel_Name"].split("(")[0]
        e["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
ids = sorted(rows)
last = ids[-300:]                      # the last step's dispatches (and a bit)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for k in last:
    e = rows[k]
    a = agg[e["name"]]
    a["n"] += 1
    for c in ("dur", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        a[c] += e.get(c, 0.0)
print("| kernel | n | dur us | waves | cyc/wave | wait | issue-stall | active |")
print("|---|---:|---:|---:|---:|---:|---:|---:|")
for n, a in sorted(agg.items(), key=lambda kv: -kv[1]["dur"])[:20]:
    wc = max(a["SQ_WAVE_CYCLES"], 1.0)
    print("| %s | %d | %.1f | %.0f | %.0f | %.2f | %.2f | %.2f |" % (
        n[:60], a["n"], a["dur"] / a["n"], a["SQ_WAVES"] / a["n"], wc / max(a["SQ_WAVES"], 1),
        a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc, a["SQ_ACTIVE_INST_ANY"] / wc))
PY
cat $O/pmc_bn.md
find $O/pmc -name "*.csv" -size +20M -delete
