#!/bin/bash
# Legacy Cerebro-Spark grid (reference run_spark.sh): the MOP grid search on
# the GPU engine, own log directory.
EXP_NAME=cerebro-spark
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_filesystem_cerebro_standalone --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --cerebro_spark $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
