#!/bin/bash
# quick state check: 1- and 8-config bench plus the 1-config step timeline
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-base}
mkdir -p $O
for C in 1 8; do
  timeout -k 10 300 python -u bench.py --configs $C > $O/c$C.json 2> $O/c$C.err || exit $?
  echo "configs=$C: $(python3 -c "import json;d=json.load(open('$O/c$C.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o prof -- python3 bench.py --configs 1 \
  --steps 20 --warmup 10 --steps_per_round 10 > $O/prof_c1.log 2>&1 || { tail -20 $O/prof_c1.log; exit 1; }
python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/prof_c1 --last-steps 10 > $O/prof_c1.md 2> $O/sum.err || exit 1
python3 -m cerebro_ds_kpgi_amd.tools.prof_timeline $O/prof_c1 > $O/timeline_c1.md 2>> $O/sum.err || exit 1
find $O/prof_c1 -name "*.db" -delete
tail -30 $O/timeline_c1.md
