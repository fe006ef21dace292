#!/bin/bash
# One parameterised same-box A/B driver (replaces the round-2 ab_*.sh scripts).
#
#   bash scripts/gpu/ab.sh NAME "VARIANTS" ["CONFIGS"] [ROUNDS] [TESTS]
#
# VARIANTS: space-separated; each is one or more env assignments joined by
#           commas, e.g. "CER_NONE=0 CER_BN_FOLD=256 CER_HIP_LIB=libcerebro_hip_pf34.so"
#           or "CER_WGB_SIDE_FRAC=0.5,CER_WGB_SPLIT_GRID=64" (A/B twins of the
#           kernel library are built beforehand with tools.build --variant)
# CONFIGS:  bench.py --configs values (default "8 1"); AB_ARGS (env) adds
#           bench.py arguments, e.g. AB_ARGS="--model mobilenetv2"
# ROUNDS:   back-to-back rounds over all variants (default 2)
# TESTS:    optional pytest selection run once per variant first (e.g.
#           "tests/test_fp32_gpu.py -k conv"); a failure stops the script
# Output: gpurun_out/ab_NAME/ (one JSON per run) and a table on stdout.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
NAME=${1:?name}
VARIANTS=${2:-"CER_NONE=0"}
CFGS=${3:-"8 1"}
ROUNDS=${4:-2}
TESTS=${5:-}
OUT=gpurun_out/ab_$NAME
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  for V in $VARIANTS; do
    env ${V//,/ } timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread \
      > "$OUT/tests_$V.log" 2>&1 || { tail -30 "$OUT/tests_$V.log"; exit 1; }
    echo "tests $V: $(tail -1 "$OUT/tests_$V.log")"
  done
fi
for R in $(seq 1 "$ROUNDS"); do
  for V in $VARIANTS; do
    for C in $CFGS; do
      F="$OUT/b_${V//[,\/]/_}_c${C}_$R"
      env ${V//,/ } timeout -k 10 300 python -u bench.py --configs "$C" ${AB_ARGS:-} > "$F.json" 2> "$F.err" || exit $?
      echo "$V c$C r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
