#!/bin/bash
# round 4: BN fold over slab pairs (one round trip per pair) as a twin
# (libcerebro_hip_pair.so): BN / fp32 numerics on the twin, bn_one per shape,
# then the step A/B against the committed library
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4pair
mkdir -p $O
CER_HIP_LIB=libcerebro_hip_pair.so timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py tests/test_kernels_gpu.py \
  tests/test_dwstats_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" $O/tests.log | head -20; exit $rc; fi
for L in libcerebro_hip.so libcerebro_hip_pair.so; do
  for SH in "25088 256 1" "1568 1024 1" "512 2048 1" "25088 64 8" "6272 512 8"; do
    set -- $SH
    CER_HIP_LIB=$L timeout -k 10 120 python3 -u scripts/dev/bn_one.py --rows $1 --C $2 --G $3 --nslab 2 --iters 100 \
      > $O/one.tmp 2>> $O/one.err || { tail -5 $O/one.err; exit 1; }
    sed "s/^{/{\"lib\": \"$L\", /" $O/one.tmp >> $O/one.jsonl
  done
done
bash scripts/gpu/ab.sh pair "CER_HIP_LIB=libcerebro_hip.so CER_HIP_LIB=libcerebro_hip_pair.so" "8 1" 3
