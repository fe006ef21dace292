#!/bin/bash
# Round 6, second pass: GM_TAP weight gradient, HL weights for packs <= 2,
# the timed-path test (faulthandler dump if it stalls), bench A/B and the
# kernel profiles of the build.  Output: gpurun_out/r6uk2/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6uk2
mkdir -p "$OUT"
step() {   # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 "$OUT/$name.log")"
  return $rc
}
step tests_uk 600 python -u -m pytest tests/test_uk_gpu.py -x -q --timeout 300 \
  --timeout-method thread || exit 1
step tests_wgb 600 python -u -m pytest tests/test_fp32_gpu.py -x -q -k "wgrad or batch" \
  --timeout 300 --timeout-method thread || exit 1
for R in 1 2; do
  for V in "CER_UK=1" "CER_UK=0"; do
    for C in 8 1; do
      T=${V//[,=]/_}
      env ${V//,/ } timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        --configs $C > "$OUT/b_${T}_c${C}_$R.json" 2> "$OUT/b_${T}_c${C}_$R.err" || exit 1
      echo "$V c$C r$R $(python3 -c "import json;d=json.load(open('$OUT/b_${T}_c${C}_$R.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
bash scripts/gpu/prof_ab.sh r6uk2/prof_c8 8 "CER_UK=1" || exit 1
bash scripts/gpu/prof_ab.sh r6uk2/prof_c1 1 "CER_UK=1" || exit 1
step tests_timed 420 python -u -m pytest tests/test_timed_path_gpu.py -x -q -s --timeout 400 \
  --timeout-method thread || exit 1
