#!/bin/bash
# 8-config (G = 8) fp32 conv shapes of the headline step: SQ counters per
# autotune candidate (fwd / dgrad / unbatched wgrad), three counter passes,
# plus the gfx950 counter list (pass C: MFMA busy + LDS bank conflicts)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_c8
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list-avail rc=$?"
grep -o "SQ_VALU_MFMA_BUSY_CYCLES\|SQ_LDS_BANK_CONFLICT\|SQ_BUSY_CU_CYCLES\|SQ_INST_CYCLES_VMEM\|SQ_LDS_IDX_ACTIVE" $O/avail.txt | sort -u > $O/have.txt || true
cat $O/have.txt
C3=$(tr '\n' ' ' < $O/have.txt)
for SH in 32,7,7,256,256,3,1,1 32,28,28,64,64,3,1,1 32,14,14,512,128,1,1,0; do
  T=$(echo $SH | tr ',' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU \
    --output-format csv -d $O/a_$T -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --G 8 --shape $SH --iters 5 > $O/a_$T.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
    --output-format csv -d $O/b_$T -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --G 8 --shape $SH --iters 5 > $O/b_$T.log 2>&1 || exit $?
  if [ -n "$C3" ]; then
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES $C3 \
      --output-format csv -d $O/c_$T -o p -- python3 -m cerebro_ds_kpgi_amd.tools.conv_one --dtype fp32 --G 8 --shape $SH --iters 5 > $O/c_$T.log 2>&1 || exit $?
  fi
  tail -1 $O/a_$T.log
done
echo done
