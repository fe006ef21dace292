#!/bin/bash
# side-stream wgrad chunks x capped grid around the 8-config optimum; 4-config check
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chunk3
for R in 1 2; do
for CFG in "0 0" "27 96" "27 128" "27 64" "20 96" "36 96" "27 0"; do
  set -- $CFG
  for C in 8 4; do
    CER_WGB_CHUNK=$1 CER_WGB_GRID=$2 timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/chunk3/b${C}_c$1_g$2_$R.json 2> gpurun_out/chunk3/b${C}_c$1_g$2_$R.err || exit $?
    echo "cfg=$C chunk=$1 grid=$2: $(python -c "import json;d=json.load(open('gpurun_out/chunk3/b${C}_c$1_g$2_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
