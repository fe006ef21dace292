#!/bin/bash
# fp32 conv per-shape throughput (vs MIOpen fp32) + PMC passes on three shapes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c32
export TMPDIR=/tmp
timeout -k 10 300 python -u -m cerebro_ds_kpgi_amd.tools.bench_conv --dtype fp32 --iters 10 \
  --json gpurun_out/c32/bench_conv_fp32.json > gpurun_out/c32/bench_conv_fp32.txt 2>&1 || exit $?
tail -3 gpurun_out/c32/bench_conv_fp32.txt
for SH in 32,14,14,128,128,3,1,1 32,28,28,64,256,1,1,0 32,7,7,1024,256,1,1,0; do
  T=$(echo $SH | tr ',' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU \
    --output-format csv -d gpurun_out/c32/pmc_$T -o p1 -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --shape $SH --iters 5 > gpurun_out/c32/pmc_$T.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/c32/pmc2_$T -o p2 -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --shape $SH --iters 5 > gpurun_out/c32/pmc2_$T.log 2>&1 || exit $?
done
echo done
