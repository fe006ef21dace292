#!/bin/bash
# Round 6: correctness + first numbers of the uniform-K fp32 GEMM kernels and
# the HL weight image.  Every GPU step has its own time limit; the chain
# stops at the first failure.  Output: gpurun_out/r6uk/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r6uk
mkdir -p "$OUT"
step() {   # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -1 "$OUT/$name.log")"
  return $rc
}
for R in 1 2; do
  for V in "CER_UK=1" "CER_UK=0" "CER_UK=1,CER_WHL=0"; do
    for C in 8 1; do
      T=${V//[,=]/_}
      env ${V//,/ } timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        --configs $C > "$OUT/b_${T}_c${C}_$R.json" 2> "$OUT/b_${T}_c${C}_$R.err" || exit 1
      echo "$V c$C r$R $(python3 -c "import json;d=json.load(open('$OUT/b_${T}_c${C}_$R.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
step tests_timed 900 python -u -m pytest tests/test_timed_path_gpu.py -x -q -s --timeout 800 \
  --timeout-method thread || exit 1
step conv_g8 600 python -u -m cerebro_ds_kpgi_amd.tools.bench_conv --dtype fp32 --G 8 \
  --no_miopen --iters 20 --json "$OUT/conv_g8.json" || exit 1
