#!/bin/bash
# Round 6: prefetch depth / occupancy of the 128x128 fp32 tiles.
#   wgpf2: the weight-gradient body (wgrad_batch32 / igemm_wgrad32) takes two
#          register sets at 128x128 (200 VGPRs, still 2 workgroups per CU)
#   occ1:  every 128x128 fp32 kernel compiled for 1 workgroup per CU with two
#          register sets (no spills; half the waves)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh occ "CER_NONE=0 CER_HIP_LIB=libcerebro_hip_wgpf2.so CER_HIP_LIB=libcerebro_hip_occ1.so" \
  "8 1" 2 "tests/test_uk_gpu.py"
