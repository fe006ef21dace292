#!/bin/bash
# same-box A/B of runtime knobs on the fp32 headline step: ab_env.sh "NAME=V1 NAME=V2 ..." [configs...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_env
VARIANTS=${1:-"CER_NONE=0"}
CFGS=${2:-"8 1"}
for R in 1 2; do
  for V in $VARIANTS; do
    for C in $CFGS; do
      env $V timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/ab_env/b_${V}_c${C}_$R.json 2>gpurun_out/ab_env/b_${V}_c${C}_$R.err || exit $?
      echo "$V c$C $(python3 -c "import json;d=json.load(open('gpurun_out/ab_env/b_${V}_c${C}_$R.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
