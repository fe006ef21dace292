#!/bin/bash
# Round 6: forward epilogue skips the bias loads when there is no bias.
# Tests, then a same-lease A/B against HEAD (abtree/base: lean forward
# epilogue only).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_uk_gpu.py tests/test_fp32_gpu.py tests/test_conv_gpu.py tests/test_dres_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r6add_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r6add_tests.log)"; [ $rc -eq 0 ] || exit 1
bash scripts/gpu/ab_trees.sh addepi "abtree/base ." 3 "headline c1"
