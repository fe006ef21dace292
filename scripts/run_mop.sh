#!/bin/bash
# UDAF rotation MOP (reference run_mop.sh)
EXP_NAME=${EXP_OVERRIDE:-cerebro}
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_mop --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE"  $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
