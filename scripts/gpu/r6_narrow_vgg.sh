#!/bin/bash
# Round 6: the 64x128 narrow wgrad tiles on VGG-16 (its block 1 is narrow)
cd "$GRAFT_REPO_ROOT" || exit 1
AB_ARGS="--model vgg16 --steps 30 --warmup 10" bash scripts/gpu/ab.sh narrow_vgg "CER_WGB_NARROW=1 CER_WGB_NARROW=2" "8" 3
