#!/bin/bash
# BASELINE config 5: Hyperopt-TPE over MOP with 16 ResNet-50 configs on one
# MI355X (reference search space with the model choice set to resnet50:
# lr ~ logU[1e-5, 1e-1], lambda in {1e-4, 1e-6}, batch in [16, 256]); async
# TPE proposes new configs as trials finish (run_da_cerebro_standalone
# --hyperopt, reference run_cerebro_standalone_helper.py:315-376)
#   bash scripts/gpu/hyperopt.sh [train rows] [epochs] [tag] ["extra runner args"]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
NT=${1:-8192}
E=${2:-3}
TAG=${3:-}
EXTRA=${4:-}
O=gpurun_out/r4hyp$TAG
mkdir -p $O
R=/tmp/cer_hyp; rm -rf $R
echo "da-hyperopt, Start time: $(date "+%Y-%m-%d %H:%M:%S")" > $O/global.log
timeout -k 10 1080 python3 -u -m cerebro_ds_kpgi_amd.runners.run_da_cerebro_standalone_hyperopt --run \
  --hyperopt --max_num_config 16 --hyperopt_models resnet50 --num_epochs $E --size 8 --backend hip \
  --train_per_partition $NT --valid_per_partition $((NT / 16)) \
  --logs_root $O/da-hyperopt --models_root $R/models $EXTRA > $O/client.log 2>&1
rc=$?
echo "da-hyperopt, End time: $(date "+%Y-%m-%d %H:%M:%S")" >> $O/global.log
grep SUMMARY $O/client.log | tail -1 | cut -c1-600
tail -3 $O/client.log
rm -rf $R
exit $rc
