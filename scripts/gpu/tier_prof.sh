#!/bin/bash
# GPU test tier, then rocprofv3 kernel stats + roofline of the fp32 headline
# step (8 configs) and of the per-GPU work at N=8 (1 config)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2b}
bash scripts/gpu/gpu_tier.sh "$TAG" || exit $?
for C in 8 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_c$C -o prof -- \
    python3 bench.py --steps 20 --warmup 10 --steps_per_round 10 --configs $C \
    > gpurun_out/prof_${TAG}_c$C.log 2>&1 || exit $?
  tail -1 gpurun_out/prof_${TAG}_c$C.log
  timeout -k 10 300 python3 -m cerebro_ds_kpgi_amd.tools.prof_summary gpurun_out/prof_${TAG}_c$C \
    --last-steps 10 --roofline resnet50,$C,32,fp32 --title "ResNet-50 x$C MOP step, fp32 ($TAG)" \
    > gpurun_out/prof_${TAG}_c$C.md || exit $?
done
