#!/bin/bash
# PMC counters for single conv shapes (kernel-trace + counters only).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pmc}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
for SH in 32,7,7,256,256,3,1,1 32,28,28,64,256,1,1,0; do
  N=$(echo $SH | tr ',' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_${TAG}_sq_$N -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --shape $SH --iters 5 > gpurun_out/pmc_${TAG}_sq_$N.log 2>&1 || { echo "pmc sq failed $SH"; tail -5 gpurun_out/pmc_${TAG}_sq_$N.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_${TAG}_tcc_$N -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --shape $SH --iters 5 > gpurun_out/pmc_${TAG}_tcc_$N.log 2>&1 || { echo "pmc tcc failed $SH"; tail -5 gpurun_out/pmc_${TAG}_tcc_$N.log; exit 1; }
done
echo done
