#!/bin/bash
# one-config step timeline (rocprofv3 kernel trace -> tools.prof_timeline),
# then the baselines on the GPU: tests + 1-epoch makespans at N = 1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3tl
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c1 -o prof -- python3 bench.py --configs 1 \
  --steps 20 --warmup 10 --steps_per_round 10 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
tail -1 $O/c1.log
python3 -m cerebro_ds_kpgi_amd.tools.prof_timeline $O/c1 > $O/c1_timeline.md 2> $O/tl.err || { tail $O/tl.err; exit 1; }
python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/c1 --last-steps 10 > $O/c1.md 2>> $O/tl.err || exit 1
find $O/c1 -name "*.db" -delete
tail -32 $O/c1_timeline.md
bash scripts/gpu/r3_baselines.sh || exit 1
bash scripts/gpu/r3_baseline_makespan.sh
