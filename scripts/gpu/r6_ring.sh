#!/bin/bash
# Round 6: the LDS-DMA ring forward kernels with the lean forward epilogue
# and pre-split (HL) weights when the image exists.  Tests, then a
# same-lease A/B against HEAD (abtree/base), and with the HL weight image on
# for every pack width.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ring
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_uk_gpu.py tests/test_fp32_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/tests.log | head; exit 1; }
for R in 1 2 3; do
  for V in base new new_whl8; do
    for C in 8 1; do
      case $V in
        base) T=abtree/base; E="CER_NONE=0" ;;
        new) T=.; E="CER_NONE=0" ;;
        new_whl8) T=.; E="CER_WHL_MAX_G=8" ;;
      esac
      [ $V = new_whl8 ] && [ $C = 1 ] && continue
      F=$O/b_${V}_c${C}_$R
      (cd $T && env $E timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --configs $C \
        > $F.json 2> $F.err) || { tail -5 $F.err; exit 1; }
      echo "$V c$C r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
done
