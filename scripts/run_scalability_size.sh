#!/bin/bash
# 8-config ResNet-50 scalability point (headline; reference run_scalability.sh)
EXP_NAME=scalability
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_da_cerebro_standalone --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --drill_down_scalability --scheduler rotation $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
