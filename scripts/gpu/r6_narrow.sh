#!/bin/bash
# Round 6: 64x128 tiles for the <= 64-output-channel batched wgrad items
# (CER_WGB_NARROW=2) against 64x64 (1, default); fp64 tests first
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh narrow "CER_WGB_NARROW=1 CER_WGB_NARROW=2" "8 1" 3 \
  "tests/test_fp32_gpu.py -k wgrad_batch"
