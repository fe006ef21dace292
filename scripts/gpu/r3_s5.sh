#!/bin/bash
# ragged channel widths (NASNet-Mobile) on HIP: numerics tests, model-family
# graph tests, then the hetero drill-down's NASNet bs4 step
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py -k "ragged or nasnet or dwconv or pool or bn_act or bn_link" -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for M in "nasnetmobile 4" "mobilenetv2 128"; do
  set -- $M
  timeout -k 10 400 python3 -u bench.py --model $1 --batch $2 --configs 1 --steps 60 --warmup 20 \
    > $O/hetero_$1.json 2> $O/hetero_$1.err || { tail -5 $O/hetero_$1.err; exit 1; }
  tail -1 $O/hetero_$1.json
done
grep -h "running eagerly" $O/*.err | head -3
