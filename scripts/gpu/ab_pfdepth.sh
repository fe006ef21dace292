#!/bin/bash
# fp32 K-loop register-ring depth (CER_FP32_PF* twins): numerics on the default
# and deepest twin, then bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_pfd
for L in libcerebro_hip.so libcerebro_hip_pf34.so; do
  CER_HIP_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread -k "conv or linear or trajectory" > gpurun_out/ab_pfd/tests_$L.log 2>&1 || { tail -30 gpurun_out/ab_pfd/tests_$L.log; exit 1; }
  tail -1 gpurun_out/ab_pfd/tests_$L.log
done
bash scripts/gpu/ab_env.sh "CER_HIP_LIB=libcerebro_hip.so CER_HIP_LIB=libcerebro_hip_pf24.so CER_HIP_LIB=libcerebro_hip_pf33.so CER_HIP_LIB=libcerebro_hip_pf34.so"
