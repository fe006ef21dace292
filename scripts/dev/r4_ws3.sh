#!/bin/bash
# round 4: the WS kernels after the P = 4 loader sets and the pipelined,
# read-ahead consumer: numerics first, then the isolated wgrad flush (WS off /
# on), then the bench with per-variant autotune times, WGB_WS off / on
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4ws3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -k "wave_specialised or wgrad_batch" \
  -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Timeout" $O/tests.log | head -20; exit $rc; fi
W="scripts/dev/wgrad_batch_bench.py --variants 1 --ws 0,1"
for G in 8 1; do
  timeout -k 10 200 python3 -u $W --G $G > $O/wgb_g$G.log 2>&1 || { tail -5 $O/wgb_g$G.log; exit 1; }
  grep '"G"' $O/wgb_g$G.log
done
for V in 0 1; do
  for C in 8 1; do
    CER_WGB_WS=$V CER_TUNE_LOG=$O/tune_w${V}_c$C.json timeout -k 10 300 python3 -u bench.py --configs $C \
      > $O/b_w${V}_c$C.json 2> $O/b_w${V}_c$C.err || { tail -5 $O/b_w${V}_c$C.err; exit 1; }
    echo "WGB_WS=$V c$C $(python3 -c "import json;d=json.load(open('$O/b_w${V}_c$C.json'));print(d['value'],d['ms_per_step'])")"
  done
done
