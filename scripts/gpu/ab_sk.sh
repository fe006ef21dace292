#!/bin/bash
# split-K block target / max splits (CER_SK_TARGET, CER_SK_MAX) A/B, 1- and 8-config steps
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sk
for R in 1 2; do
for CFG in "384 8" "768 16" "1024 16" "512 12"; do
  set -- $CFG
  for C in 1 8; do
    CER_SK_TARGET=$1 CER_SK_MAX=$2 timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/sk/b${C}_t$1_m$2_r$R.json 2> gpurun_out/sk/b${C}_t$1_m$2_r$R.err || exit $?
    echo "cfg=$C target=$1 max=$2: $(python -c "import json;d=json.load(open('gpurun_out/sk/b${C}_t$1_m$2_r$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
