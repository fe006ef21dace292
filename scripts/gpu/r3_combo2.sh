#!/bin/bash
# what the fp32 conv kernels spend: timing-only builds without the hi/lo
# split VALU / with one MFMA pass (wrong numerics, conv_one only); DA ETL
# re-measure after the loader fixes; batched-wgrad knobs at 1-2 configs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/split_cost
mkdir -p $O
for LIB in libcerebro_hip.so libcerebro_hip_nosplit.so libcerebro_hip_onepass.so; do
  for SH in 32,7,7,256,256,3,1,1 32,28,28,64,64,3,1,1 32,14,14,512,128,1,1,0 32,28,28,256,64,1,1,0; do
    for G in 8 1; do
      CER_HIP_LIB=$LIB timeout -k 10 120 python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --G $G --shape $SH --iters 20 \
        >> $O/$LIB.txt 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    done
  done
  echo "== $LIB"; cat $O/$LIB.txt
done
DA_ONLY_FULL=1 bash scripts/gpu/r3_da_etl.sh || exit 1
bash scripts/gpu/ab.sh wgbknob "CER_NONE=0 CER_WGB_ROWS=2048 CER_WGB_ROWS=2048,CER_WGB_VARIANT=2" "1 2" 2
