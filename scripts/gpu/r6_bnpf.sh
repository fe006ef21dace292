#!/bin/bash
# Round 6: BN apply kernels issue their first row chunk before the partial
# fold.  BN GPU tests, then a same-lease A/B against the HEAD build
# (abtree/base) on the headline and the one-config headline.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6bnpf
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_fp32_gpu.py tests/test_hl_gpu.py \
  -x -q -k "bn" --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 "$OUT/tests.log")"; [ $rc -eq 0 ] || exit 1
bash scripts/gpu/ab_trees.sh bnpf "abtree/base ." 2 "headline c1"
# one-config packs: side-stream share of the batched weight gradients again
# (measured -3 % in round 2, before the uniform-K kernels)
bash scripts/gpu/ab.sh side1 "CER_NONE=0 CER_WGB_SIDE_MIN_G=1,CER_WGB_SIDE_MIN_IMAGES=32 CER_WGB_SIDE_MIN_G=1,CER_WGB_SIDE_MIN_IMAGES=32,CER_WGB_SPLIT_GRID=160" "1" 2
