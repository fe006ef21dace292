#!/bin/bash
# The Criteo collection (reference run_criteo_collection.sh:16-60): same
# approaches with --criteo and 5 epochs.
TS=${1:-$(date "+%Y_%m_%d_%H_%M_%S")}
EPOCHS=${2:-5}
SIZE=${3:-8}
D="$(dirname "$0")"
for s in run_imagenet.sh run_mop.sh run_ctq.sh run_da_cerebro_standalone.sh \
         run_filesystem_cerebro_standalone.sh run_pytorchddp.sh; do
  bash "$D/$s" "$TS" "$EPOCHS" "$SIZE" "--criteo --train_name criteo_train_data_packed --valid_name criteo_valid_data_packed ${4:-}"
done
