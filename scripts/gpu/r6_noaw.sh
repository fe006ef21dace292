#!/bin/bash
# Round 6: upper bound of an A-direct fp32 GEMM (A fragments straight from
# global, no A tile in LDS): the timing-only twin libcerebro_hip_noaw.so
# (CER_TIMING_NOAW: the A operand's LDS stores dropped, its loads kept; wrong
# numerics) against the default build, kernel summaries of the bench step at
# 8 and 1 configs.  Then the BN apply kernels (first row chunk loaded before
# the partial fold) against the HEAD build (abtree/base), per launch.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/prof_ab.sh r6noaw/c8 8 "CER_NONE=0" "CER_HIP_LIB=libcerebro_hip_noaw.so" || exit 1
bash scripts/gpu/prof_ab.sh r6noaw/c1 1 "CER_NONE=0" "CER_HIP_LIB=libcerebro_hip_noaw.so" || exit 1
O=$PWD/gpurun_out/r6noaw/bn
mkdir -p "$O"
for R in 1 2; do
  for T in abtree/base .; do
    TAG=${T//[\/.]/_}
    for SH in "25088 64 1" "25088 256 1" "1568 1024 1" "512 2048 1" "512 512 1" "6272 512 8" "1568 1024 8"; do
      set -- $SH
      (cd "$T" && timeout -k 10 120 python -u scripts/dev/bn_one.py --rows $1 --C $2 --G $3 --iters 200 --nslab 2) \
        >> "$O/${TAG}_$R.jsonl" 2>> "$O/err.log" || exit 1
    done
    echo "bn $T r$R done"
  done
done
