#!/bin/bash
# 1-epoch makespans at N = 1 of the headline grid (8 ResNet-50 configs, bs 32)
# through the reference entry points: MOP (DA-Cerebro standalone), task
# parallel, MA and DDP -- each config sees 65 536 images per epoch
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3bm
mkdir -p $O
R=/tmp/cer_bm; rm -rf $R
one() {  # name module per_partition extra...
  local n=$1 mod=$2 nt=$3; shift 3
  timeout -k 10 300 python3 -u -m cerebro_ds_kpgi_amd.runners.$mod --run --num_epochs 1 \
    --drill_down_scalability --size 1 --backend hip --train_per_partition $nt \
    --valid_per_partition $((nt / 25)) --logs_root $O/$n --models_root $R/$n "$@" \
    > $O/$n.log 2>&1 || { tail -5 $O/$n.log; rm -rf $R; exit 1; }
  echo "$n $(grep SUMMARY $O/$n.log | tail -1 | cut -c1-400)"
}
one mop run_da_cerebro_standalone 8192
one task run_da_cerebro_standalone 8192 --scheduler task
one ma run_imagenet 65536
one ddp run_pytorchddp 65536
rm -rf $R
