#!/bin/bash
# side-batch fraction x grid with 2048-row wgrad splits (8 configs)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/frac2
for R in 1 2; do
for CFG in "0.5 96" "0.4 96" "0.6 96" "0.5 128" "0.5 80" "0.6 128"; do
  set -- $CFG
  CER_WGB_SIDE_FRAC=$1 CER_WGB_SPLIT_GRID=$2 timeout -k 10 300 python -u bench.py > gpurun_out/frac2/b8_f$1_g$2_$R.json 2> gpurun_out/frac2/b8_f$1_g$2_$R.err || exit $?
  echo "cfg=8 frac=$1 grid=$2: $(python -c "import json;d=json.load(open('gpurun_out/frac2/b8_f$1_g$2_$R.json'));print(d['value'],d['ms_per_step'])")"
done
done
