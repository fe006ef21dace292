#!/bin/bash
# NASNet cell-add fusion: GPU NASNet tests, then an interleaved A/B of the
# G = 10 / G = 1 pack rates with CER_NASNET_FUSED_ADD 1 / 0.
set -o pipefail
O=gpurun_out/r4nasadd; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nasnet or NASNet" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for f in 1 0; do
    for g in 10 1; do
      CER_NASNET_FUSED_ADD=$f timeout -k 10 240 python -u bench.py --model nasnetmobile --batch 4 --configs $g --steps 60 --warmup 20 > $O/f${f}_g${g}_r$r.json 2> $O/f${f}_g${g}_r$r.err || exit 1
      echo "f=$f g=$g r=$r $(cat $O/f${f}_g${g}_r$r.json)"
    done
  done
done
