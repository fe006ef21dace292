#!/bin/bash
# final build: bf16 diag metric + per-kernel HBM traffic of the fp32 8-config step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final_extra
timeout -k 10 300 python -u bench.py --dtype bf16 > gpurun_out/final_extra/bf16.json 2> gpurun_out/final_extra/bf16.err || exit $?
cut -c1-200 gpurun_out/final_extra/bf16.json
bash scripts/gpu/hbm_pmc.sh 8 > gpurun_out/final_extra/hbm.log 2>&1 || { tail -20 gpurun_out/final_extra/hbm.log; exit 1; }
echo hbm-done
