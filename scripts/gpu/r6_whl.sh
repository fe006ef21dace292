#!/bin/bash
# Round 6: the HL weight image for wide packs again, after the lean epilogues
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/ab.sh whl8 "CER_NONE=0 CER_WHL_MAX_G=8" "8 2" 3
