#!/bin/bash
# Round 6: register prefetch depth of the small (64x64) fp32 tiles (3 / 4
# sets at 3 waves per SIMD vs 2 sets at 4) and the 128x128 weight-gradient
# body's second set, 3 alternating rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh pf "CER_NONE=0 CER_HIP_LIB=libcerebro_hip_pf4s.so CER_HIP_LIB=libcerebro_hip_wgpf2.so" \
  "1 8" 3 "tests/test_uk_gpu.py"
