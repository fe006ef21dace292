#!/bin/bash
# Criteo data preparation (reference load_criteo.sh): real click logs when
# CRITEO_DAYS names them (tools.preprocess_criteo), else synthetic data.
ROOT=${CEREBRO_DATA:-/tmp/cerebro_data}
P=${1:-8}
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$REPO:$PYTHONPATH"
if [ -n "$CRITEO_DAYS" ]; then
  python -m cerebro_ds_kpgi_amd.tools.preprocess_criteo --inputs $CRITEO_DAYS --out "$ROOT/criteo" --partitions "$P"
else
  python -m cerebro_ds_kpgi_amd.tools.make_fs_data --root "$ROOT/criteo" --dataset criteo --partitions "$P" --train ${2:-200000} --valid ${3:-20000}
  python -m cerebro_ds_kpgi_amd.tools.make_da_data --root "$ROOT/criteo_da" --dataset criteo --partitions "$P" --train ${2:-200000} --valid ${3:-20000}
fi
