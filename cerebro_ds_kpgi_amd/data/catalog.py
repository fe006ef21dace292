"""Data catalogs and availability matrices.

The reference's Cerebro data catalog is
``{name: {'data_root', 'train': [paths], 'train_availability': [[0/1]*P]*W,
'valid', 'valid_availability'}}`` with rows = workers, cols = partitions
(``run_cerebro_standalone_helper.py:37-183``; DA uses ``np.eye(size)``,
``da.py:149-162``).  Here workers are GPUs and partitions are HBM-resident
shards; a partition is *available* on exactly the GPU that pins it.
"""

import json
import os

import numpy as np


def partition_owner(p, num_partitions, num_gpus):
    """Contiguous blocks: partitions [r*V, (r+1)*V) live on GPU r."""
    V = num_partitions // num_gpus
    return p // V


def availability(num_partitions, num_gpus):
    A = np.zeros((num_gpus, num_partitions), dtype=int)
    for p in range(num_partitions):
        A[partition_owner(p, num_partitions, num_gpus), p] = 1
    return A


def make_data_catalog(name, num_partitions, num_gpus, data_root="hbm://"):
    A = availability(num_partitions, num_gpus).tolist()
    return {name: {
        "data_root": data_root,
        "train": ["{}/train_{}".format(name, p) for p in range(num_partitions)],
        "train_availability": A,
        "valid": ["{}/valid_{}".format(name, p) for p in range(num_partitions)],
        "valid_availability": A,
    }}


def write_manifest(path, catalog, extra=None):
    """Per-run manifest (replaces the reference's ``sys_cat.dill`` on NFS)."""
    doc = {"catalog": catalog}
    if extra:
        doc.update(extra)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1, default=str)
