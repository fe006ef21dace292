#!/bin/bash
# DA-Cerebro MOP (reference run_da_cerebro_standalone.sh)
EXP_NAME=cerebro-da
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_da_cerebro_standalone --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --da --scheduler greedy $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
