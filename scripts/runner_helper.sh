#!/bin/bash
# Shared run-script prologue/epilogue (reference cerebro_gpdb/runner_helper.sh:16-68):
#   bash run_X.sh [TIMESTAMP] [EPOCHS=10] [SIZE=8] [OPTIONS]
# SIZE is the number of GPUs (one rank per GPU, torchrun over 127.0.0.1).
TIMESTAMP=${1:-$(date "+%Y_%m_%d_%H_%M_%S")}
EPOCHS=${2:-10}
SIZE=${3:-8}
OPTIONS=${4:-}
ROOT=${CEREBRO_ROOT:-/tmp/cerebro_runs}
LOG_DIR=$ROOT/logs/run_logs/$TIMESTAMP
MODEL_DIR=$ROOT/models/$TIMESTAMP
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$REPO:$PYTHONPATH"
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
mkdir -p "$LOG_DIR/$EXP_NAME" "$MODEL_DIR"

PRINT_START () {
    echo "$EXP_NAME, Start time: $(date "+%Y-%m-%d %H:%M:%S")" | tee -a "$LOG_DIR/global.log"
    SECONDS=0
}

PRINT_END () {
    echo "$EXP_NAME, End time: $(date "+%Y-%m-%d %H:%M:%S")" | tee -a "$LOG_DIR/global.log"
    echo "$EXP_NAME, TOTAL EXECUTION TIME OVER ALL MST $SECONDS" | tee -a "$LOG_DIR/global.log"
}

# run a runner module on SIZE GPUs
LAUNCH () {
    local module=$1; shift
    if [ "$SIZE" -gt 1 ]; then
        python -m torch.distributed.run --nnodes=1 --nproc-per-node "$SIZE" \
            --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29533} \
            -m "cerebro_ds_kpgi_amd.runners.$module" "$@"
    else
        python -m "cerebro_ds_kpgi_amd.runners.$module" "$@"
    fi
}
