#!/bin/bash
# GPU tier + smoke + driver-shape bench, then the lagged-Adam A/B (1 / 8
# configs) and the high-priority main stream A/B (with / without a side
# wgrad batch at one config)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/r3_tier.sh || exit $?
bash scripts/gpu/ab.sh lag "CER_LAG=0 CER_LAG=1" "1 8" 2 || exit $?
bash scripts/gpu/ab.sh prio "CER_PRIO=0 CER_PRIO=1 CER_PRIO=1,CER_WGB_SIDE_MIN_G=1" "1" 2 || exit $?
bash scripts/gpu/ab.sh prio8 "CER_PRIO=0 CER_PRIO=1" "8" 1
