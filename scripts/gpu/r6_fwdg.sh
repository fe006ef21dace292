#!/bin/bash
# Round 6: lean forward epilogue for the aligned-gather (GM_FWD) forward
# kernels too (the stem).  Full GPU tier, then a same-lease A/B vs HEAD.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/gpu_tier.sh fwdg || exit 1
bash scripts/gpu/ab_trees.sh fwdg "abtree/base ." 3 "headline c1"
