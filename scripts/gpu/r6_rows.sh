#!/bin/bash
# Round 6: wgrad-batch rows per split re-checked on the end build
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh rows8 "CER_NONE=0 CER_WGB_ROWS_WIDE=1536 CER_WGB_ROWS_WIDE=3072" "8" 3 || exit 1
bash scripts/gpu/ab.sh rows1 "CER_NONE=0 CER_WGB_ROWS=768 CER_WGB_ROWS=1536" "1" 3
