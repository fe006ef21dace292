#!/bin/bash
# two-config packs (per-GPU work at N = 4): side split / wide rows thresholds
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/g2
for R in 1 2; do
for CFG in "4 1024" "2 2048" "2 1024" "4 2048"; do
  set -- $CFG
  if [ "$1" = "2" ]; then MG=2; else MG=4; fi
  CER_WGB_SIDE_MIN_G=$MG CER_WGB_ROWS=$2 CER_WGB_ROWS_WIDE=$2 timeout -k 10 300 python -u bench.py --configs 2 > gpurun_out/g2/b2_m$1_r$2_$R.json 2> gpurun_out/g2/b2_m$1_r$2_$R.err || exit $?
  echo "cfg=2 min_g=$1 rows=$2: $(python -c "import json;d=json.load(open('gpurun_out/g2/b2_m$1_r$2_$R.json'));print(d['value'],d['ms_per_step'])")"
done
done
