#!/bin/bash
# BASELINE configs 3 and 6 as measured jobs at N = 1 (VERDICT r3 "missing" #5):
#   bash scripts/gpu/workloads.sh criteo        -- the 16-config Criteo confA grid,
#       1 epoch over 16 DA partitions at 1/8 of the 13.0 M-row dataset (90/10
#       train/valid; the packed table stores dense 7306-d float32 rows, 29 KB
#       each, so the full 380 GB payload does not fit one call's generation
#       time), through DA-Cerebro with the ETL timed separately;
#   bash scripts/gpu/workloads.sh size udaf|ctq -- the model-size drill-down
#       (8 configs of MobileNetV2 / ResNet-50 / ResNet-152 / VGG-16, 3 epochs)
#       at 1/32 of the ImageNet partition size, through run_mop (UDAF rotation)
#       or ctq (greedy).
#   bash scripts/gpu/workloads.sh makespan      -- one full epoch of the headline
#       8-config ResNet-50 grid at full ImageNet-112 partition sizes through
#       DA-Cerebro standalone (synthetic data generated in HBM)
# Makespans are global.log Start / End as in runner_helper.sh.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4work
mkdir -p $O
R=/tmp/cer_work
rm -rf $R; mkdir -p $R
if [ "$1" = "criteo" ]; then
  ( time timeout -k 10 400 python3 -u -m cerebro_ds_kpgi_amd.tools.make_da_data --root $R/criteo \
      --dataset criteo --partitions 16 --train 91362 --valid 10151 ) > $O/make_criteo.log 2>&1 \
      || { tail -5 $O/make_criteo.log; rm -rf $R; exit 1; }
  du -sh $R/criteo >> $O/make_criteo.log; tail -4 $O/make_criteo.log
  echo "da-criteo, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > $O/criteo_global.log
  timeout -k 10 900 python3 -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
    --criteo --num_epochs 1 --size 1 --backend hip --da --da_root $R/criteo \
    --train_per_partition 91362 --valid_per_partition 10151 \
    --logs_root $O/criteo/logs --models_root $R/models > $O/criteo.log 2>&1
  rc=$?
  echo "da-criteo, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> $O/criteo_global.log
  grep SUMMARY $O/criteo.log | tail -1 | cut -c1-900
  rm -rf $R
  exit $rc
fi
if [ "$1" = "size" ]; then
  A=$2
  [ "$A" = "udaf" ] && M=run_mop || M=ctq
  for ID in s m l x; do
    timeout -k 10 500 python3 -u -m cerebro_ds_kpgi_amd.runners.$M --run --num_epochs 3 \
      --drill_down_model_size --drill_down_model_size_identifier $ID --size 1 --backend hip \
      --train_per_partition 5005 --valid_per_partition 195 \
      --logs_root $O/size_${A}_$ID/logs --models_root $R/models > $O/size_${A}_$ID.log 2>&1 \
      || { tail -20 $O/size_${A}_$ID.log; rm -rf $R; exit 1; }
    echo "$ID $(grep SUMMARY $O/size_${A}_$ID.log | tail -1 | cut -c1-400)"
    rm -rf $R/models
  done
  rm -rf $R
  exit 0
fi
if [ "$1" = "makespan" ]; then
  echo "cerebro-da, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > $O/makespan_global.log
  timeout -k 10 1080 python3 -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
    --num_epochs 1 --drill_down_scalability --size 1 --backend hip \
    --logs_root $O/makespan/logs --models_root $R/models > $O/makespan.log 2>&1
  rc=$?
  echo "cerebro-da, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> $O/makespan_global.log
  grep SUMMARY $O/makespan.log | tail -1 | cut -c1-600
  rm -rf $R
  exit $rc
fi
echo "usage: workloads.sh criteo | size udaf|ctq | makespan"; exit 2
