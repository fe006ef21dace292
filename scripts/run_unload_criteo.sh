#!/bin/bash
# Reference run_unload_criteo.sh unloads the packed DB tables to text files
# through gpfdist and re-parses them (etl_criteo.py) into h5 — a DB-side
# ETL this framework does not need: the DA reader parses the segment pages
# directly.  Kept as the DA -> filesystem export: partitions read through
# the C++ page reader and written in the filesystem layout.
ROOT=${CEREBRO_DATA:-/tmp/cerebro_data}
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$REPO:$PYTHONPATH"
python -m cerebro_ds_kpgi_amd.tools.da_export --da_root "$ROOT/criteo_da" --out "$ROOT/criteo_unloaded"
