#!/bin/bash
# fp32 conv kernels: SQ counters (issue / wait / MFMA busy / LDS) on three ResNet-50 shapes
#   PMC_G=1 PMC_SHAPES="..." PMC_OUT=pmc_c1 bash scripts/gpu/conv32_pmc2.sh   (one-config packs)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${PMC_OUT:-pmc2}
mkdir -p $O
export TMPDIR=/tmp
for SH in ${PMC_SHAPES:-32,14,14,128,128,3,1,1 32,28,28,64,256,1,1,0 32,7,7,1024,256,1,1,0}; do
  T=$(echo $SH | tr ',' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    --output-format csv -d $O/a_$T -o p -- python3 scripts/dev/conv_one.py --dtype fp32 --shape $SH --G ${PMC_G:-8} --iters 5 > $O/a_$T.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU \
    --output-format csv -d $O/b_$T -o p -- python3 scripts/dev/conv_one.py --dtype fp32 --shape $SH --G ${PMC_G:-8} --iters 5 > $O/b_$T.log 2>&1 || exit $?
  tail -1 $O/a_$T.log
done
echo done
