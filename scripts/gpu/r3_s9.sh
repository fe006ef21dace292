#!/bin/bash
# depthwise wgrad rewrite (coalesced channel lanes + 4-column sliding window):
# numerics tests, MobileNetV2 8-config / hetero bs128 / NASNet bs4 rates and a
# MobileNetV2 kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_fp32_gpu.py tests/test_kernels_gpu.py \
  -k "dwconv or ragged or nasnet or mobilenet" -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['metric'],d['value'],d['ms_per_step'])")"
}
run size_mobilenetv2 --model mobilenetv2 --steps 30 --warmup 10
run hetero_mbv2_b128 --model mobilenetv2 --batch 128 --configs 1 --steps 30 --warmup 10
run hetero_nasnet_b4 --model nasnetmobile --batch 4 --configs 1 --steps 60 --warmup 20
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_mbv2 -o prof -- \
  python3 bench.py --model mobilenetv2 --steps 20 --warmup 10 --steps_per_round 10 > $O/prof_mbv2.log 2>&1 || exit 1
timeout -k 10 200 python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/prof_mbv2 --last-steps 10 \
  --title "MobileNetV2 x8 MOP step, fp32" > $O/prof_mbv2.md || exit 1
head -30 $O/prof_mbv2.md
