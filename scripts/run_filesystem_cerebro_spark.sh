#!/bin/bash
# Cerebro-Spark (reference run_filesystem_cerebro_spark.sh).  No Spark here:
# the Cerebro-Spark engine's MOP semantics (randomized hopping over
# partitions prepared on shared storage) run on the GPU MOP engine with the
# greedy randomized scheduler over filesystem partitions (--fs_root).
EXP_NAME=e2e_filesystem_cerebro_spark
source "$(dirname "$0")/runner_helper.sh" "$@"
PRINT_START
LAUNCH run_filesystem_cerebro_standalone --logs_root "$LOG_DIR/$EXP_NAME" --models_root "$MODEL_DIR" --run --num_epochs "$EPOCHS" --size "$SIZE" --scheduler greedy --spark_data_prepared --cerebro_spark $OPTIONS 2>&1 | tee "$LOG_DIR/$EXP_NAME/client.log"
PRINT_END
