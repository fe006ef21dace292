#!/bin/bash
# hetero {ResNet-50,VGG-16} drill-down, UDAF
EXP_NAME=cerebro-udaf_drill_down_hetro
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_mop --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --drill_down_hetro $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
