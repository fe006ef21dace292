#!/bin/bash
# end of the depthwise work: MobileNetV2 rates + profile (r3_s9.sh), then the
# full GPU tier, smoke and driver bench (r3_tier.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/r3_s9.sh || exit $?
bash scripts/gpu/r3_tier.sh r3dw2 || exit $?
