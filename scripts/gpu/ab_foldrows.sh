#!/bin/bash
# BN folded-apply rows per block (CER_BN_FOLD_ROWS) and fold threshold (CER_BN_FOLD) A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/foldrows
for R in 1 2; do
for CFG in "16 64" "32 64" "24 64" "16 32" "32 128"; do
  set -- $CFG
  for C in 8 1; do
    CER_BN_FOLD_ROWS=$1 CER_BN_FOLD=$2 timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/foldrows/b${C}_r$1_f$2_$R.json 2> gpurun_out/foldrows/b${C}_r$1_f$2_$R.err || exit $?
    echo "cfg=$C rows=$1 fold=$2: $(python -c "import json;d=json.load(open('gpurun_out/foldrows/b${C}_r$1_f$2_$R.json'));print(d['value'],d['ms_per_step'])")"
  done
done
done
