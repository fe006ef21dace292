#!/bin/bash
# rocprof kernel summaries + one-step timelines of bench.py --configs C under
# environment variants: prof_ab.sh TAG C "VAR1=a" "VAR1=b" ...
# (BENCH_ARGS="--model vgg16" etc. is passed to every bench.py)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; C=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
i=0
for V in "$@"; do
  i=$((i+1))
  env $V timeout -k 10 300 python -u bench.py --configs $C $BENCH_ARGS > $O/b$i.json 2> $O/b$i.err || exit $?
  echo "[$V] $(python3 -c "import json;d=json.load(open('$O/b$i.json'));print(d['value'],d['ms_per_step'])")"
  env $V timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p$i -o prof -- python3 bench.py --configs $C $BENCH_ARGS \
    --steps 20 --warmup 10 --steps_per_round 10 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/p$i --last-steps 10 > $O/p$i.md 2> $O/sum.err || exit 1
  python3 -m cerebro_ds_kpgi_amd.tools.prof_timeline $O/p$i > $O/t$i.md 2>> $O/sum.err || exit 1
  find $O/p$i -name "*.db" -delete
  grep "step wall" $O/t$i.md
done
