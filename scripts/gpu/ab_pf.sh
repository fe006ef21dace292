#!/bin/bash
# A/B: fp32 conv K loop with two register sets (default lib) vs one (pf1 twin)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_pf
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pf/tests.log 2>&1 || { tail -30 gpurun_out/ab_pf/tests.log; exit 1; }
tail -2 gpurun_out/ab_pf/tests.log
for V in pf1 pf2 pf1 pf2; do
  LIB=libcerebro_hip.so; [ $V = pf1 ] && LIB=libcerebro_hip_pf1.so
  for C in 8 1; do
    CER_HIP_LIB=$LIB timeout -k 10 300 python -u bench.py --configs $C > gpurun_out/ab_pf/bench_${V}_c$C.json 2>/dev/null || exit $?
    echo "$V c$C $(python3 -c "import json;d=json.load(open('gpurun_out/ab_pf/bench_${V}_c$C.json'));print(d['value'],d['ms_per_step'])")"
  done
done
for V in pf1 pf2; do
  LIB=libcerebro_hip.so; [ $V = pf1 ] && LIB=libcerebro_hip_pf1.so
  CER_HIP_LIB=$LIB timeout -k 10 400 python -u -m cerebro_ds_kpgi_amd.tools.bench_conv --dtype fp32 --iters 10 \
    --json gpurun_out/ab_pf/conv_$V.json > gpurun_out/ab_pf/conv_$V.txt 2>&1 || exit $?
  tail -4 gpurun_out/ab_pf/conv_$V.txt
done
