#!/bin/bash
# The ImageNet experiment collection (reference run_imagenet_collection.sh):
# every approach back to back on the same timestamp.  The reference's
# gpstop/gpstart + 5-minute sleeps between runs restart the database; here
# each run is its own process group, so nothing needs restarting.
TS=${1:-$(date "+%Y_%m_%d_%H_%M_%S")}
EPOCHS=${2:-10}
SIZE=${3:-8}
D="$(dirname "$0")"
for s in run_imagenet.sh run_mop.sh run_ctq.sh run_da_cerebro_standalone.sh \
         run_filesystem_cerebro_standalone.sh run_pytorchddp.sh run_pytorchddp_da.sh; do
  bash "$D/$s" "$TS" "$EPOCHS" "$SIZE" "${4:-}"
done
