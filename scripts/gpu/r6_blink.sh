#!/bin/bash
# Round 6: lean bias-link epilogue (VGG's conv -> conv dgrads): tests, then
# VGG-16 x 8 against HEAD (abtree/base), 3 alternating rounds
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6blink
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_vgg_links_gpu.py tests/test_uk_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/tests.log | head; exit 1; }
for R in 1 2 3; do
  for T in abtree/base .; do
    F=$O/b_${T//[\/.]/_}_$R
    (cd $T && timeout -k 10 300 python -u bench.py --gpus 1 --model vgg16 --steps 30 --warmup 10 > $F.json 2> $F.err) \
      || { tail -5 $F.err; exit 1; }
    echo "$T vgg16 r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
  done
done
