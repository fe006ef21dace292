#!/bin/bash
# one- and eight-config step timelines (rocprofv3 kernel trace ->
# tools.prof_timeline), lagged-Adam grid A/B, then the baselines on the GPU:
# tests + 1-epoch makespans at N = 1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3tl
mkdir -p $O
for C in 1 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c$C -o prof -- python3 bench.py --configs $C \
    --steps 20 --warmup 10 --steps_per_round 10 > $O/c$C.log 2>&1 || { tail -20 $O/c$C.log; exit 1; }
  tail -1 $O/c$C.log
  python3 -m cerebro_ds_kpgi_amd.tools.prof_timeline $O/c$C > $O/c${C}_timeline.md 2> $O/tl.err || { tail $O/tl.err; exit 1; }
  python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/c$C --last-steps 10 > $O/c$C.md 2>> $O/tl.err || exit 1
  find $O/c$C -name "*.db" -delete
  tail -28 $O/c${C}_timeline.md
done
bash scripts/gpu/ab.sh laggrid "CER_LAG=0 CER_LAG=1,CER_LAG_GRID=16 CER_LAG=1,CER_LAG_GRID=64" "1 8" 2 || exit 1
bash scripts/gpu/r3_baselines.sh || exit 1
bash scripts/gpu/r3_baseline_makespan.sh
