#!/bin/bash
# the reference's secondary published workloads at N = 1 (fp32, HIP path):
# model-size drill-down (8 configs each), e2e 16-config grid, the 48-config
# hetero drill-down's per-config steps, and a dwconv (MobileNetV2) profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3sec
mkdir -p $O
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['metric'],d['value'],d['ms_per_step'])")"
}
for M in mobilenetv2 resnet152 vgg16; do run size_$M --model $M --steps 30 --warmup 10; done
run e2e16 --workload e2e16 --steps 20 --warmup 5 --steps_per_round 10
run hetero_mbv2_b128 --model mobilenetv2 --batch 128 --configs 1 --steps 30 --warmup 10
run hetero_nasnet_b4 --model nasnetmobile --batch 4 --configs 1 --steps 60 --warmup 20
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_mbv2 -o prof -- \
  python3 bench.py --model mobilenetv2 --steps 20 --warmup 10 --steps_per_round 10 > $O/prof_mbv2.log 2>&1 || exit 1
timeout -k 10 200 python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/prof_mbv2 --last-steps 10 \
  --title "MobileNetV2 x8 MOP step, fp32" > $O/prof_mbv2.md || exit 1
head -12 $O/prof_mbv2.md
