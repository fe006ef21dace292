#!/bin/bash
# Round 6: Adam split around the last weight-gradient batch (early half on
# the side stream beside it).  Split tests, the timed-path oracle test, then
# a same-lease A/B: this tree with CER_ADAM_EARLY=1 / 0 and the previous
# build (abtree/base), headline + one config.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6early
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_adam_split_gpu.py -x -v -s --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "split tests rc=$rc $(tail -1 $O/tests.log)"; grep "after 6 steps" $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests/test_timed_path_gpu.py -x -q -s --timeout 450 \
  --timeout-method thread > $O/timed.log 2>&1
rc=$?; echo "timed path rc=$rc $(tail -1 $O/timed.log)"; [ $rc -eq 0 ] || exit 1
for R in 1 2 3; do
  for T in abtree/base . ; do
    for V in 1 0; do
      [ "$T" = "abtree/base" ] && [ $V = 0 ] && continue
      for C in 8 1; do
        F=$O/b_${T//[\/.]/_}_e${V}_c${C}_$R
        (cd $T && CER_ADAM_EARLY=$V timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
          --configs $C > $F.json 2> $F.err) || { tail -5 $F.err; exit 1; }
        echo "$T early=$V c$C r$R $(python3 -c "import json;d=json.load(open('$F.json'));print(d['value'],d['ms_per_step'])")"
      done
    done
  done
done
