#!/bin/bash
# round 4: every pending kernel change in one twin (libcerebro_hip_dwb.so =
# the BN fold in one round trip, the wgrad batch item lookup, the gavg row
# batch, the branch-free depthwise bodies): the GPU numerics of the touched
# paths + the lanes test on the twin, then A/B benches against the committed
# library (base) on the same box
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4ver
mkdir -p $O
CER_HIP_LIB=libcerebro_hip_dwb.so timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py tests/test_hl_gpu.py \
  tests/test_kernels_gpu.py tests/test_dwstats_gpu.py tests/test_lanes_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" $O/tests.log | head -20; exit $rc; fi
CER_HIP_LIB=libcerebro_hip_dwb.so timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -k "dw" -x -q \
  --timeout 120 --timeout-method thread > $O/tests_conv.log 2>&1
rc=$?
tail -3 $O/tests_conv.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" $O/tests_conv.log | head -20; exit $rc; fi
for R in 1 2; do
  for L in base dwb; do
    for A in "--configs 8" "--configs 1" "--model mobilenetv2" "--model mobilenetv2 --batch 128 --configs 8"; do
      T=$(echo "$A" | tr -d ' -')
      F=$O/b_${L}_${T}_r$R
      if [ $L = base ]; then unset CER_HIP_LIB; else export CER_HIP_LIB=libcerebro_hip_$L.so; fi
      timeout -k 10 300 python3 -u bench.py $A > $F.json 2> $F.err || { tail -5 $F.err; exit 1; }
      echo "$L $T r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
unset CER_HIP_LIB
CER_HIP_LIB=libcerebro_hip_dwb.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -- python3 bench.py \
  --model mobilenetv2 --steps 20 --warmup 10 --steps_per_round 10 > $O/prof.log 2>&1 || exit 1
python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/prof --last-steps 10 > $O/prof_mbv2.md 2> $O/sum.err || exit 1
find $O/prof -name "*.db" -delete
head -45 $O/prof_mbv2.md
