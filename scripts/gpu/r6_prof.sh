#!/bin/bash
# kernel summaries + one-step timelines of the current build at 8 and 1 configs
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r6prof}
bash scripts/gpu/prof_ab.sh $TAG/c8 8 "CER_NONE=0" || exit 1
bash scripts/gpu/prof_ab.sh $TAG/c1 1 "CER_NONE=0" || exit 1
