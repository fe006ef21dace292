#!/bin/bash
# one-config (G = 1) fp32 conv shapes of the N = 8 per-GPU step: SQ counters
# (where a K step's ~1 us goes), every autotune candidate dispatched
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_c1
export TMPDIR=/tmp
for SH in 32,28,28,64,64,3,1,1 32,4,4,512,512,3,1,1 32,14,14,512,128,1,1,0; do
  T=$(echo $SH | tr ',' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU \
    --output-format csv -d gpurun_out/pmc_c1/a_$T -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --G 1 --shape $SH --iters 5 > gpurun_out/pmc_c1/a_$T.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
    --output-format csv -d gpurun_out/pmc_c1/b_$T -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --G 1 --shape $SH --iters 5 > gpurun_out/pmc_c1/b_$T.log 2>&1 || exit $?
  tail -1 gpurun_out/pmc_c1/a_$T.log
done
echo done
