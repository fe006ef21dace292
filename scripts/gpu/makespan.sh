#!/bin/bash
# One full epoch of the headline workload through the reference's north-star
# entry point (DA-Cerebro standalone, 8-config ResNet-50 scalability grid,
# full ImageNet-112 partition sizes: 8 x 160 160 train + 8 x 6 250 valid
# images, synthetic data generated in HBM), N=1: makespan + per-round log.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/makespan
R=/tmp/cer_makespan
rm -rf $R; mkdir -p $R
echo "cerebro-da, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > gpurun_out/makespan/global.log
timeout -k 10 1080 python -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone --run \
  --num_epochs 1 --drill_down_scalability --size 1 --backend hip \
  --logs_root gpurun_out/makespan/cerebro-da --models_root $R/models \
  > gpurun_out/makespan/client.log 2>&1
rc=$?
echo "cerebro-da, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> gpurun_out/makespan/global.log
tail -3 gpurun_out/makespan/client.log
ls -la $R/models | head -5
rm -rf $R
exit $rc
