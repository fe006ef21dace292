#!/bin/bash
# the reference's secondary published workloads at N = 1 (fp32, HIP path):
# model-size drill-down (8 configs each), e2e 16-config grid, the 48-config
# hetero drill-down's per-config steps, and a dwconv (MobileNetV2) profile.
#   bash scripts/gpu/secondary.sh hetero   -- only the 48-config hetero drill-down:
#     pack rates (NASNet-Mobile bs4 G = 1 / 10, MobileNetV2 bs128 G = 1 / 8) and
#     the CTQ (greedy) and UDAF (rotation) jobs at N = 1, 12 partitions of 512
#     images
#   bash scripts/gpu/secondary.sh hetero_jobs TAG [RUNNER ARGS]  -- only the CTQ / UDAF
#     jobs, outputs under het_TAG_* (e.g. TAG=plain with --pack_order false)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4sec
mkdir -p $O
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['metric'],d['value'],d['ms_per_step'])")"
}
jobs() {  # tag, runner args...
  local T=$1; shift
  for A in ctq run_mop; do
    timeout -k 10 500 python3 -u -m cerebro_ds_kpgi_amd.runners.$A --run --num_epochs 1 \
      --drill_down_hetro --size 1 --slots_per_gpu 12 --train_per_partition 512 \
      --valid_per_partition 64 --backend hip --logs_root $O/het_${T}$A/logs \
      --models_root /tmp/het_models "$@" > $O/het_${T}$A.log 2>&1 || { tail -20 $O/het_${T}$A.log; exit 1; }
    grep SUMMARY $O/het_${T}$A.log | tail -1 | cut -c1-600
    rm -rf /tmp/het_models
  done
}
if [ "$1" = "hetero" ]; then
  run nasnet_b4_g1 --model nasnetmobile --batch 4 --configs 1 --steps 60 --warmup 20
  run nasnet_b4_g10 --model nasnetmobile --batch 4 --configs 10 --steps 60 --warmup 20
  run mbv2_b128_g1 --model mobilenetv2 --batch 128 --configs 1 --steps 30 --warmup 10
  run mbv2_b128_g8 --model mobilenetv2 --batch 128 --configs 8 --steps 30 --warmup 10
  jobs ""
  exit 0
fi
if [ "$1" = "hetero_jobs" ]; then
  T=$2; shift 2
  jobs "${T}_" "$@"
  exit 0
fi
for M in mobilenetv2 resnet152 vgg16; do run size_$M --model $M --steps 30 --warmup 10; done
run e2e16 --workload e2e16 --steps 20 --warmup 5 --steps_per_round 10
run hetero_mbv2_b128 --model mobilenetv2 --batch 128 --configs 1 --steps 30 --warmup 10
run hetero_nasnet_b4 --model nasnetmobile --batch 4 --configs 1 --steps 60 --warmup 20
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_mbv2 -o prof -- \
  python3 bench.py --model mobilenetv2 --steps 20 --warmup 10 --steps_per_round 10 > $O/prof_mbv2.log 2>&1 || exit 1
timeout -k 10 200 python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $O/prof_mbv2 --last-steps 10 \
  --title "MobileNetV2 x8 MOP step, fp32" > $O/prof_mbv2.md || exit 1
head -12 $O/prof_mbv2.md
