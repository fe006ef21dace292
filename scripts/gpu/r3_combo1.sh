#!/bin/bash
# wgrad batch isolation + G=8 PMC passes + DA ETL at scale, one box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/wgb
for G in 8 1; do
  timeout -k 10 300 python3 -u -m cerebro_ds_kpgi_amd.tools.wgrad_batch_bench --G $G --rows 0,512,2048 \
    > gpurun_out/wgb/g$G.jsonl 2> gpurun_out/wgb/g$G.err || { tail -5 gpurun_out/wgb/g$G.err; exit 1; }
  cat gpurun_out/wgb/g$G.jsonl
done
bash scripts/gpu/r3_pmc_c8.sh || exit 1
bash scripts/gpu/r3_da_etl.sh
