#!/bin/bash
# Round 6: a second side-stream wgrad batch (CER_WGB_SIDE_FRAC2): the first
# one ends ~0.7 ms before backward does, the tail batch then runs serially
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh side2 "CER_NONE=0 CER_WGB_SIDE_FRAC2=0.7 CER_WGB_SIDE_FRAC2=0.8 CER_WGB_SIDE_FRAC2=0.9" "8 4" 3 \
  "tests/test_graph_gpu.py"
