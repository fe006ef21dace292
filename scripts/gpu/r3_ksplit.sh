#!/bin/bash
# Intra-block K-split fp32 conv kernels (ids 24-35): numerics, then a same-box
# A/B of the autotune with / without them at 1 and 8 configs, plus which
# problems picked them.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r3ks
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -k "ksplit" -x -q --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
CER_TUNE_LOG=$OUT/tune4_c1.json timeout -k 10 300 python -u bench.py --configs 1 > $OUT/c1_tuned4.json 2> $OUT/c1_tuned4.err || exit 1
cat $OUT/c1_tuned4.json
bash scripts/gpu/ab.sh ksplit4 "CER_FP32_KSPLIT=2 CER_FP32_KSPLIT=1" "1 8" 2
