#!/bin/bash
# round 4: where the BN folded apply's time goes.  (1) bn_one per layer
# shape with the committed library and the one-round-trip fold twin
# (libcerebro_hip_bnf.so, bn.hip of bd1acdc), at 8 / 4 / 2 slabs;
# (2) the step with CER_BN_ATOMIC_SLABS 8 / 4 / 2 (same box)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4bnfold
mkdir -p $O
for L in libcerebro_hip.so libcerebro_hip_bnf.so; do
  for S in 8 4 2; do
    for SH in "25088 64 1" "25088 256 1" "1568 1024 1" "512 2048 1" "512 512 1" "25088 64 8" "6272 512 8" "1568 1024 8"; do
      set -- $SH
      CER_HIP_LIB=$L timeout -k 10 120 python3 -u scripts/dev/bn_one.py --rows $1 --C $2 --G $3 --nslab $S --iters 100 \
        > $O/one.tmp 2>> $O/one.err || { tail -5 $O/one.err; exit 1; }
      sed "s/^{/{\"lib\": \"$L\", \"nslab\": $S, /" $O/one.tmp >> $O/one.jsonl
    done
  done
  echo "$L done"
done
bash scripts/gpu/ab.sh slabs "CER_BN_ATOMIC_SLABS=8 CER_BN_ATOMIC_SLABS=4 CER_BN_ATOMIC_SLABS=2" "8 1" 2
