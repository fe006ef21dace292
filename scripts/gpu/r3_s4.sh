#!/bin/bash
# BN forward apply: early-load restructure (twins bnf0 = old order, bnf2 =
# timing-only without statistic writes) by microbench + step A/B; fp32 / HL /
# branch tests on the default build; then the secondary published workloads
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s4
mkdir -p $O
for LIB in libcerebro_hip.so libcerebro_hip_bnf0.so libcerebro_hip_bnf2.so; do
  for S in "1568 256 1" "392 1024 1" "25088 64 1" "1568 256 8"; do
    set -- $S
    CER_HIP_LIB=$LIB timeout -k 10 120 python -m cerebro_ds_kpgi_amd.tools.bn_one --rows $1 --C $2 --G $3 \
      > $O/tmp.jsonl 2> $O/bn_one.err || { tail $O/bn_one.err; exit 1; }
    sed "s/^/$LIB /" $O/tmp.jsonl | grep -E '"fwd"|bwd_zmask' >> $O/bn_one.txt
  done
done
cat $O/bn_one.txt
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py tests/test_hl_gpu.py tests/test_branch_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu/ab.sh bnf "CER_HIP_LIB=libcerebro_hip_bnf0.so CER_HIP_LIB=libcerebro_hip.so" "1 8" 2 || exit 1
bash scripts/gpu/r3_secondary.sh
