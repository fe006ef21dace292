#!/bin/bash
# CTQ greedy MOP (reference run_ctq.sh)
EXP_NAME=${EXP_OVERRIDE:-cerebro-ctq}
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH ctq --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE"  $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
