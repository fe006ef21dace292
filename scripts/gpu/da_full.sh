#!/bin/bash
# Full-size DA-Cerebro epoch with ETL at N = 1 (VERDICT r4 #7,
# profiles/r5_da_full.md): 8 partitions x (160 160 train + 6 250 valid)
# ImageNet-112 images = the whole 1 281 280-image training set, stored as
# Greenplum heap / TOAST / pglz pages (float32 payload), loaded into HBM by
# the DA reader and trained for one epoch by the 8-config MOP grid.
# The box's disk (79 GB) holds 5 of the 8 partitions (13.1 GB each on disk):
# partitions 5..7 are hard links to 0..2 (make_da_data --unique 5), so every
# partition's pages are still walked, detoasted, decoded and copied to HBM.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5da_full}
UNIQUE=${UNIQUE:-5}
mkdir -p $O
R=/tmp/cer_da_full
rm -rf $R; mkdir -p $R
{ df -h /tmp | tail -1; nproc; free -g | head -2; } > $O/host.txt
cat $O/host.txt
( time timeout -k 10 420 python -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/da8 \
    --partitions 8 --unique $UNIQUE --jobs 3 --dataset imagenet --train 160160 --valid 6250 ) \
    > $O/make.log 2>&1 || { tail -5 $O/make.log; rm -rf $R; exit 1; }
{ du -sh $R/da8; df -h /tmp | tail -1; } >> $O/make.log
tail -5 $O/make.log
echo "cerebro-da, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > $O/global.log
CER_DA_WINDOW=${WINDOW:-2} timeout -k 10 900 python -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
  --num_epochs 1 --drill_down_scalability --size 1 --backend hip --da --da_root $R/da8 \
  --train_per_partition 160160 --valid_per_partition 6250 \
  --logs_root $O/cerebro-da --models_root $R/models > $O/client.log 2>&1
rc=$?
echo "cerebro-da, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> $O/global.log
grep SUMMARY $O/client.log | tail -1 | cut -c1-1500
rm -rf $R
exit $rc
