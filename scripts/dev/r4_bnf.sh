#!/bin/bash
# round 4: the fp64-slab BN fold in one round trip + per-channel loads hoisted above it (bn.hip),
# and the wgrad batch item lookup without a dependent kernarg-load chain (conv.hip wgb_item)
# as an A/B twin: numerics of every fp32 conv / BN-link
# path on the twin, then the bench with the twin and without, same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4bnf
mkdir -p $O
CER_HIP_LIB=libcerebro_hip_bnf.so timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py tests/test_hl_gpu.py tests/test_kernels_gpu.py \
  -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" $O/tests.log | head -20; exit $rc; fi
for R in 1 2; do
  for L in base bnf; do
    for C in 8 1; do
      if [ $L = bnf ]; then export CER_HIP_LIB=libcerebro_hip_bnf.so; else unset CER_HIP_LIB; fi
      F=$O/b_${L}_c${C}_r$R
      timeout -k 10 300 python3 -u bench.py --configs $C > $F.json 2> $F.err || { tail -5 $F.err; exit 1; }
      echo "$L c$C r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
