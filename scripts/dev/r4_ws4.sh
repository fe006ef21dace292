#!/bin/bash
# round 4: what bounds the wave-specialised wgrad -- the isolated batched
# wgrad flush, WS off / on, on the normal build and on two timing-only twins
# (wrong numerics): no hi/lo split VALU (the loaders' work), and one MFMA per
# fragment pair instead of three (the consumers' work)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4ws4
mkdir -p $O
W="scripts/dev/wgrad_batch_bench.py --variants 1 --ws 0,1 --G 8"
for L in "" nosplit onepass; do
  N=${L:-base}
  if [ -n "$L" ]; then export CER_HIP_LIB=libcerebro_hip_$L.so; else unset CER_HIP_LIB; fi
  timeout -k 10 200 python3 -u $W > $O/wgb_$N.log 2>&1 || { tail -5 $O/wgb_$N.log; exit 1; }
  echo "$N"; grep '"G"' $O/wgb_$N.log
done
