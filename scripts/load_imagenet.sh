#!/bin/bash
# Data preparation (reference load_imagenet.sh / load_imagenet.py --load --pack):
# write the packed partitions in both access formats the runners read —
# Greenplum-format DA pages (--da) and filesystem partitions (--fs_root).
# With real JPEG folders, run tools.preprocess_imagenet first and point
# DATA_SRC at its output; otherwise synthetic ImageNet-shaped data is used.
ROOT=${CEREBRO_DATA:-/tmp/cerebro_data}
P=${1:-8}
TRAIN=${2:-160160}
VALID=${3:-6250}
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$REPO:$PYTHONPATH"
python -m cerebro_ds_kpgi_amd.tools.make_da_data --root "$ROOT/imagenet_da" --dataset imagenet --partitions "$P" --train "$TRAIN" --valid "$VALID"
python -m cerebro_ds_kpgi_amd.tools.make_fs_data --root "$ROOT/imagenet" --dataset imagenet --partitions "$P" --train "$TRAIN" --valid "$VALID"
