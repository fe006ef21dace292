"""Filesystem partitions: the reference's ``/mnt/imagenet`` / ``/mnt/hdd/criteo``
layout.

Reference: per-partition HDF5 files ``{train,valid}/{train,valid}_{i}.h5``
(``images`` f32[N,112,112,3], ``labels``) read by a 32-thread pool
(``cerebro_gpdb/run_cerebro_standalone_helper.py:379-416``), and Criteo
``{train,valid}_{i}.npy`` = f32[N, 7306 + 1] with the label in the last
column (``:419-429``, catalog ``:30-171``).

Here (h5py is not installed; images are stored as the uint8 they are):

* ImageNet partition ``train/train_{i}`` = ``train_{i}.images.npy`` (uint8
  [N,112,112,3]) + ``train_{i}.labels.npy`` (int32 [N]); the catalog keeps the
  reference's ``.h5`` names and ``resolve`` maps them to the pair;
* Criteo partition ``train/train_{i}.npy`` = exactly the reference's dense
  f32 [N, 7307] layout (``np.load`` compatible).

``input_fn`` / ``input_fn_criteo`` keep the reference contracts;
``fs_partition_loader`` is the engine's loader (memory-mapped reads, pinned
host staging, one copy into HBM; Criteo one-hot rows become the 39 active
column ids consumed by the embedding-bag first layer).
"""

import os
from multiprocessing.dummy import Pool

import numpy as np

from ..config import catalog as cat

N_READERS = 32


def _stem(root, split, i):
    return os.path.join(root, split, "{}_{}".format(split, i))


def resolve(file_path):
    """Reference catalog path (``…/train_3.h5`` or ``…/train_3``) -> our files."""
    base = file_path[:-3] if file_path.endswith(".h5") else file_path
    return base + ".images.npy", base + ".labels.npy"


def fs_catalog(root, dataset, num_partitions):
    """Cerebro DATA_CATALOG entry (identity availability)."""
    ext = ".h5" if dataset == "imagenet" else ".npy"
    eye = np.eye(num_partitions, dtype=int).tolist()
    return {"data_root": root,
            "train": ["train/train_{}{}".format(i, ext) for i in range(num_partitions)],
            "train_availability": eye,
            "valid": ["valid/valid_{}{}".format(i, ext) for i in range(num_partitions)],
            "valid_availability": eye}


def write_fs_dataset(root, dataset, num_partitions, n_train, n_valid, seed=cat.SEED):
    """Synthetic partitions of the dataset's shape in the reference layout."""
    from . import synthetic
    for split, n in (("train", n_train), ("valid", n_valid)):
        os.makedirs(os.path.join(root, split), exist_ok=True)
        for i in range(num_partitions):
            s = seed * 1000 + i * 2 + (split == "valid")
            if dataset == "imagenet":
                x, y = synthetic.image_partition(n, seed=s)
                ip, lp = resolve(_stem(root, split, i))
                np.save(ip, x.numpy())
                np.save(lp, y.numpy().astype(np.int32))
            elif dataset == "criteo":
                idx, y = synthetic.criteo_partition(n, seed=s)
                dense = np.zeros((n, cat.INPUT_SHAPE_CRITEO[0] + 1), np.float32)
                rows = np.repeat(np.arange(n), idx.shape[1])
                dense[rows, idx.numpy().reshape(-1)] = 1.0
                dense[:, -1] = y.numpy()
                np.save(_stem(root, split, i) + ".npy", dense)
            else:
                raise ValueError(dataset)
    return fs_catalog(root, dataset, num_partitions)


def input_fn(file_path, one_hot=True):
    """[{'images': f32[n,112,112,3], 'labels': one-hot f32[n,1000] | int[n]}, ...]
    in N_READERS slices read in parallel (reference contract)."""
    ip, lp = resolve(file_path)
    images = np.load(ip, mmap_mode="r")
    labels = np.load(lp, mmap_mode="r")
    size = images.shape[0]
    step = int(np.ceil(size / float(N_READERS))) or 1

    def read(start):
        x = np.asarray(images[start:start + step], dtype=np.float32)
        y = np.asarray(labels[start:start + step]).astype(int)
        if one_hot:
            y = np.eye(cat.NUM_CLASSES, dtype=np.float32)[y]
        return {"images": x, "labels": y}
    with Pool(N_READERS) as pool:
        return pool.map(read, range(0, size, step))


def input_fn_criteo(file_path):
    """{'images': f32[n,7306], 'labels': one-hot f32[n,2]} (reference contract)."""
    arr = np.load(file_path)
    return {"images": arr[:, :-1].astype(np.float32),
            "labels": np.eye(2, dtype=np.float32)[arr[:, -1].astype(int)]}


def _criteo_ids(dense, width=39):
    """Dense one-hot rows -> [n, 39] int32 active column ids, -1 padded
    (rows with missing features have fewer than 39 actives)."""
    n = dense.shape[0]
    out = np.full((n, width), -1, np.int32)
    rows, cols = np.nonzero(dense)
    counts = np.bincount(rows, minlength=n)
    if counts.max(initial=0) > width:
        raise ValueError("more than {} active features in a Criteo row".format(width))
    pos = np.arange(len(rows)) - np.repeat(np.cumsum(counts) - counts, counts)
    out[rows, pos] = cols
    return out


def fs_partition_loader(root, dataset, device):
    """Loader for ``PartitionStore``: partition p -> (train_x, train_y, valid_x, valid_y)
    in HBM."""
    import torch

    def load(split, p):
        if dataset == "imagenet":
            ip, lp = resolve(_stem(root, split, p))
            x = torch.from_numpy(np.array(np.load(ip, mmap_mode="r")))
            y = torch.from_numpy(np.load(lp).astype(np.int32))
        elif os.path.exists(_stem(root, split, p) + ".ids.npy"):   # compact (preprocess_criteo)
            x = torch.from_numpy(np.load(_stem(root, split, p) + ".ids.npy").astype(np.int32))
            y = torch.from_numpy(np.load(_stem(root, split, p) + ".labels.npy").astype(np.int32))
        else:
            arr = np.load(_stem(root, split, p) + ".npy", mmap_mode="r")
            x = torch.from_numpy(_criteo_ids(arr[:, :-1]))
            y = torch.from_numpy(np.asarray(arr[:, -1]).astype(np.int32))
        if torch.device(device).type == "cuda":
            x = x.pin_memory()
        return x.to(device, non_blocking=True), y.to(device)

    def loader(p):
        tx, ty = load("train", p)
        vx, vy = load("valid", p)
        return tx, ty, vx, vy
    return loader


def is_fs_root(root):
    return bool(root) and os.path.isdir(os.path.join(root, "train"))


def _train_indices(root):
    import re
    idx = set()
    for f in os.listdir(os.path.join(root, "train")):
        m = re.match(r"train_(\d+)\.(images\.npy|ids\.npy|npy)$", f)
        if m:
            idx.add(int(m.group(1)))
    return idx


def count_partitions(root):
    """Number of consecutive training partitions train_0 .. train_{n-1}."""
    idx = _train_indices(root)
    n = 0
    while n in idx:
        n += 1
    return n


def fs_dataset_of(root):
    """"imagenet" (``train_{i}.images.npy``) or "criteo" (``train_{i}.npy`` /
    compact ``train_{i}.ids.npy``) from the files a filesystem root holds."""
    if os.path.exists(os.path.join(root, "train", "train_0.images.npy")):
        return "imagenet"
    if (os.path.exists(os.path.join(root, "train", "train_0.npy"))
            or os.path.exists(os.path.join(root, "train", "train_0.ids.npy"))):
        return "criteo"
    raise ValueError("{} holds no train_0 partition".format(root))
