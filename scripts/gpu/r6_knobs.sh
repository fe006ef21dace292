#!/bin/bash
# Round 6 end: autotune candidate sets and the HL weight image re-checked
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh knobs_end "CER_NONE=0 CER_WHL_MAX_G=8 CER_FP32_WIDE=0 CER_FP32_RING=0 CER_FP32_KSPLIT=0" "8 1" 3
