#!/bin/bash
# Time-breakdown runs (reference run_breakdown.sh:16-28) with tracing and
# 1 Hz telemetry on; analyse with python -m cerebro_ds_kpgi_amd.tools.log_analyzer.
TS=${1:-$(date "+%Y_%m_%d_%H_%M_%S")}
EPOCHS=${2:-1}
SIZE=${3:-8}
D="$(dirname "$0")"
for s in run_ctq.sh run_mop.sh run_da_cerebro_standalone.sh; do
  bash "$D/$s" "$TS" "$EPOCHS" "$SIZE" "--trace ${4:-}"
done
