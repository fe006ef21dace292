"""Criteo click logs -> partitioned training data.

Reference pipeline: ``preprocessing/criteo/gen_train_valid_data.py`` (90/10
train/valid split of ``day_*`` lines with ``random.seed(2018)``) then
``preprocessing_criteo.py`` (fillna(0), ``df.sample(frac, random_state)``,
per-row featurisation to the 7306-wide one-hot vector, npy output), then a
round-robin spread over the workers' partitions.

    python -m cerebro_ds_kpgi_amd.tools.preprocess_criteo --inputs day_1 day_2 day_3 \
        --out /data/criteo --partitions 8 [--dense]

Output (``data.fs`` layout): ``{train,valid}/{split}_{i}.ids.npy`` (int32
[n, 39], -1 padded) + ``.labels.npy`` — or with ``--dense`` the reference's
f32 [n, 7307] ``{split}_{i}.npy``.  Featurisation runs in C++ (murmur3 +
bucketing, multi-threaded; ``csrc/da/criteo.cpp``).
"""

import argparse
import os
import random

import numpy as np

from ..config import catalog as cat
from ..data import criteo

CHUNK = 64 << 20


def split_lines(inputs, valid_fraction=0.1, seed=cat.SEED):
    """The reference's streaming split: one ``random.random()`` draw per line."""
    rnd = random.Random(seed)
    train, valid = [], []
    for path in inputs:
        with open(path, "rb") as f:
            for line in f:
                (valid if rnd.random() < valid_fraction else train).append(line)
    return b"".join(train), b"".join(valid)


def featurize(buf, nthreads=8):
    ids, labels = [], []
    start = 0
    while start < len(buf):
        end = min(len(buf), start + CHUNK)
        if end < len(buf):
            end = buf.rfind(b"\n", start, end) + 1 or len(buf)
        i, l = criteo.featurize_lines(buf[start:end], nthreads)
        ids.append(i)
        labels.append(l)
        start = end
    if not ids:
        return np.empty((0, criteo.FIELDS), np.int32), np.empty(0, np.int32)
    return np.concatenate(ids), np.concatenate(labels)


def write_partitions(out, split, ids, labels, partitions, dense=False):
    os.makedirs(os.path.join(out, split), exist_ok=True)
    for p, sel in enumerate(np.array_split(np.arange(len(labels)), partitions)):
        stem = os.path.join(out, split, "{}_{}".format(split, p))
        if dense:
            np.save(stem + ".npy", criteo.ids_to_dense(ids[sel], labels[sel]))
        else:
            np.save(stem + ".ids.npy", ids[sel])
            np.save(stem + ".labels.npy", labels[sel].astype(np.int32))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--inputs", nargs="+", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--valid_fraction", type=float, default=0.1)
    ap.add_argument("--frac", type=float, default=1.0, help="df.sample fraction")
    ap.add_argument("--dense", action="store_true", help="reference dense f32 [n, 7307] npy")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args(argv)
    train, valid = split_lines(a.inputs, a.valid_fraction)
    rs = np.random.RandomState(cat.SEED)
    stats = {}
    for split, buf in (("train", train), ("valid", valid)):
        ids, labels = featurize(buf, a.threads)
        order = rs.permutation(len(labels))[:int(round(a.frac * len(labels)))]
        write_partitions(a.out, split, ids[order], labels[order], a.partitions, a.dense)
        stats[split] = int(len(order))
    print("criteo:", stats)
    return stats


if __name__ == "__main__":
    main()
