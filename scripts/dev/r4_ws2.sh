#!/bin/bash
# round 4: why the wave-specialised kernels lose.  The batched wgrad flush
# with the 128x128 kernel off / on (G = 8 and 1), its kernel summary, two SQ
# counter passes over both kernels, and the bench's per-variant autotune times
# (fwd / dgrad WS twins against the winner of every conv problem)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4ws2
mkdir -p $O
W="scripts/dev/wgrad_batch_bench.py --variants 1 --ws 0,1"
for G in 8 1; do
  timeout -k 10 200 python3 -u $W --G $G > $O/wgb_g$G.log 2>&1 || { tail -5 $O/wgb_g$G.log; exit 1; }
  cat $O/wgb_g$G.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $W --G 8 --reps 3 \
  > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $O/pmc_a -o p -- python3 $W --G 8 --reps 1 > $O/pmc_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_SALU \
  --output-format csv -d $O/pmc_b -o p -- python3 $W --G 8 --reps 1 > $O/pmc_b.log 2>&1 || exit 1
for C in 8 1; do
  CER_TUNE_LOG=$O/tune_c$C.json timeout -k 10 300 python3 -u bench.py --configs $C \
    > $O/b_c$C.json 2> $O/b_c$C.err || { tail -5 $O/b_c$C.err; exit 1; }
  cat $O/b_c$C.json | cut -c1-200
done
echo done
