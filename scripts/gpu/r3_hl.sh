#!/bin/bash
# HL operand format: tests (bit-identity, format), the fp32 conv/BN tiers,
# then the same-box A/B at 1 and 8 configs; DA ETL re-measure; wgrad knobs
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/hl
timeout -k 10 900 python -u -m pytest tests/test_hl_gpu.py tests/test_fp32_gpu.py tests/test_conv_gpu.py -x -q -s \
  --timeout 300 --timeout-method thread > gpurun_out/hl/tests.log 2>&1 || { tail -40 gpurun_out/hl/tests.log; exit 1; }
tail -2 gpurun_out/hl/tests.log
grep "norm rel diff" gpurun_out/hl/tests.log
bash scripts/gpu/ab.sh hl "CER_HL=0 CER_HL=1" "1 8" 2 || exit 1
DA_ONLY_FULL=1 bash scripts/gpu/r3_da_etl.sh || exit 1
bash scripts/gpu/ab.sh wgbknob "CER_NONE=0 CER_WGB_ROWS=2048 CER_WGB_ROWS=2048,CER_WGB_VARIANT=2" "1 2" 2
