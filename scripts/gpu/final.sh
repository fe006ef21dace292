#!/bin/bash
# end of round: GPU tier, smoke, driver-shape bench, per-GPU work at
# N = 1/2/4/8 (configs 8/4/2/1), steady-state kernel summaries and step
# timelines at 1 and 8 configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
bash scripts/gpu/gpu_tier.sh final
TIER_RC=$?
# a test failure is reported, the measurements still run (a GPU fault /
# timeout of the tier stops here)
if [ $TIER_RC -ne 0 ] && [ $TIER_RC -ne 1 ]; then exit $TIER_RC; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit $?
cat $O/driver.json
for C in 8 4 2 1; do
  timeout -k 10 300 python -u bench.py --configs $C > $O/c$C.json 2> $O/c$C.err || exit $?
  echo "configs=$C: $(python3 -c "import json;d=json.load(open('$O/c$C.json'));print(d['value'],d['ms_per_step'])")"
done
for C in 1 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c$C -o prof -- python3 bench.py --configs $C \
    --steps 20 --warmup 10 --steps_per_round 10 > $O/prof_c$C.log 2>&1 || { tail -20 $O/prof_c$C.log; exit 1; }
  python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/prof_c$C --last-steps 10 > $O/prof_c$C.md 2> $O/sum.err || exit 1
  python3 -m cerebro_ds_kpgi_amd.tools.prof_timeline $O/prof_c$C > $O/timeline_c$C.md 2>> $O/sum.err || exit 1
  find $O/prof_c$C -name "*.db" -delete
  head -22 $O/prof_c$C.md
done
exit $TIER_RC
