#!/bin/bash
# Round 6: lean forward epilogue for the uniform-K kernels (no addend /
# BN-backward operand loads; the 128x128 kernel loses its spills).  Tests,
# then a same-lease A/B against the previous build (abtree/base) and the
# round-4 end build (abtree/r4).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_uk_gpu.py tests/test_fp32_gpu.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r6lean_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r6lean_tests.log)"; [ $rc -eq 0 ] || exit 1
bash scripts/gpu/ab_trees.sh lean "abtree/r4 abtree/base ." 3 "headline c1"
