#!/bin/bash
# Cerebro-Spark + async TPE (reference run_filesystem_cerebro_spark_hyperopt.sh)
EXP_NAME=cerebro_spark-hyperopt
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_filesystem_cerebro_standalone_hyperopt --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --hyperopt --max_num_config 32 --num_epochs "$EPOCHS" --size "$SIZE" --spark_data_prepared --cerebro_spark $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
