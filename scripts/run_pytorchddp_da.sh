#!/bin/bash
# DA-DDP baseline (reference run_pytorchddp_da.sh)
EXP_NAME=e2e_imagenet_pytorchddp_da
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_pytorchddp_da --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --da $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
