#!/bin/bash
# Round 6: side-stream wgrad share / grid after the lean epilogues shortened
# the dgrad chain (8 configs, 3 alternating rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh side8 "CER_NONE=0 CER_WGB_SIDE_FRAC=0.3 CER_WGB_SIDE_FRAC=0.5 CER_WGB_SPLIT_GRID=128 CER_WGB_SPLIT_GRID=64" "8" 3
