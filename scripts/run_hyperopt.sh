#!/bin/bash
# Hyperopt task parallel (reference run_hyperopt.sh)
EXP_NAME=spark-hyperopt
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_hyperopt --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --hyperopt --max_num_config 32 $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
