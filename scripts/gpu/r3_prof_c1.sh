#!/bin/bash
# rocprofv3 kernel trace of the one-config (N = 8 per-GPU work) and the
# 8-config fp32 ResNet-50 steps: per-family time per step (last 10 graph
# replays) for profiles/r3_resnet50_1cfg_fp32.md
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r3prof
mkdir -p $OUT
for C in 1 2 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c$C -o prof -- python3 bench.py --configs $C \
    --steps 20 --warmup 10 > $OUT/c$C.log 2>&1 || { tail -20 $OUT/c$C.log; exit 1; }
  tail -1 $OUT/c$C.log
  python3 -m cerebro_ds_kpgi_amd.tools.prof_summary $OUT/c$C --last-steps 10 > $OUT/c$C.md 2> $OUT/c$C.sum.err || { tail $OUT/c$C.sum.err; exit 1; }
  find $OUT/c$C -name "*.db" -delete
  head -30 $OUT/c$C.md
done
echo done
