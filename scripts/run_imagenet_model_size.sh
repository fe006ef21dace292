#!/bin/bash
# Model-size drill-down (reference run_imagenet_model_size.sh:16-87):
# {UDAF (lock-step rotation), CTQ (greedy)} x {s, m, l, x}, 3 epochs each.
TS=${1:-$(date "+%Y_%m_%d_%H_%M_%S")}
SIZE=${3:-8}
for mode in udaf ctq; do
  for ident in s m l x; do
    EXP="drill_down_udaf_ctq_model_size-$mode-$ident"
    if [ "$mode" = udaf ]; then SCRIPT=run_mop.sh; else SCRIPT=run_ctq.sh; fi
    EXP_OVERRIDE="$EXP" bash "$(dirname "$0")/$SCRIPT" "$TS" 3 "$SIZE" \
        "--drill_down_model_size --drill_down_model_size_identifier $ident ${4:-}"
  done
done
