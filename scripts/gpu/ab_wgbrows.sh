#!/bin/bash
# wgrad batch rows per split x side-batch grid, 8 / 4 configs
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wgbrows
for R in 1 2; do
for CFG in "1024 96" "2048 96" "3072 96" "4096 96"; do
  set -- $CFG
  for C in 8 4 1; do
    CER_WGB_ROWS=$1 CER_WGB_SPLIT_GRID=$2 timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/wgbrows/b${C}_r$1_g$2_$R.json 2> gpurun_out/wgbrows/b${C}_r$1_g$2_$R.err || exit $?
    echo "cfg=$C rows=$1 grid=$2: $(python -c "import json;d=json.load(open('gpurun_out/wgbrows/b${C}_r$1_g$2_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
