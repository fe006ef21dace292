#!/bin/bash
# MA model averaging (reference run_imagenet.sh)
EXP_NAME=ma
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_imagenet --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE"  $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
