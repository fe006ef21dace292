"""HBM-resident partition store + device-side batch gather (SURVEY.md §7.1,
K14; replaces the reference's per-sample Python generators and DataLoaders,
``run_cerebro_standalone_helper.py:432-460``, ``run_pytorchddp.py:50-137``).

Each GPU pins its data partitions once.  Per epoch, every partition gets a
device permutation; a training step's batch is gathered from the permuted
partition by index on device (uint8 -> normalised compute dtype, packed
NHWC over the G configs being trained), so there is no host in the loop and
the step is CUDA-graph capturable (the batch cursor is a device scalar).
"""

import torch

from ..config import catalog as cat
from ..ops.backend import use_hip
from . import synthetic


class Partition(object):
    def __init__(self, pid, train_x, train_y, valid_x, valid_y):
        self.pid = pid
        self.train_x, self.train_y = train_x, train_y
        self.valid_x, self.valid_y = valid_x, valid_y

    @property
    def n_train(self):
        return self.train_y.shape[0]

    @property
    def n_valid(self):
        return self.valid_y.shape[0]


class PartitionStore(object):
    """The partitions this rank owns (global ids -> local slot index)."""

    def __init__(self, dataset, partition_ids, n_train, n_valid, device, seed=cat.SEED,
                 loader=None):
        self.dataset = dataset
        self.device = torch.device(device)
        self.pids = list(partition_ids)
        self.local = {p: i for i, p in enumerate(self.pids)}
        self.seed = seed
        parts = []
        if loader is not None and hasattr(loader, "prefetch"):
            loader.prefetch(self.pids)
        for p in self.pids:
            if loader is not None:
                tx, ty, vx, vy = loader(p)
            else:
                tx, ty = self._make(n_train, seed * 1000 + 2 * p)
                vx, vy = self._make(n_valid, seed * 1000 + 2 * p + 1)
            parts.append(Partition(p, tx, ty, vx, vy))
        if loader is not None and parts:
            # loaded partitions: equal-size views (the engine steps all partitions together)
            n_train = min(q.train_x.shape[0] for q in parts)
            n_valid = min(q.valid_x.shape[0] for q in parts)
            for q in parts:
                q.train_x, q.train_y = q.train_x[:n_train], q.train_y[:n_train]
                q.valid_x, q.valid_y = q.valid_x[:n_valid], q.valid_y[:n_valid]
        # stacked so a kernel can index [local_part, row]
        self.train_x = torch.stack([q.train_x for q in parts]) if parts else None
        self.train_y = torch.stack([q.train_y for q in parts]) if parts else None
        self.valid_x = torch.stack([q.valid_x for q in parts]) if parts else None
        self.valid_y = torch.stack([q.valid_y for q in parts]) if parts else None
        self.n_train = n_train
        self.n_valid = n_valid
        self.perm = None
        self.valid_perm = None
        if self.pids:
            ar = torch.arange(n_valid, device=self.device, dtype=torch.int32)
            self.valid_perm = ar.unsqueeze(0).repeat(len(self.pids), 1).contiguous()

    def _make(self, n, seed):
        d = self.dataset
        if d == "imagenet":
            return synthetic.image_partition(n, seed=seed, device=self.device)
        if d == "tiny":
            return synthetic.tiny_partition(n, seed=seed, device=self.device)
        if d == "criteo":
            return synthetic.criteo_partition(n, seed=seed, device=self.device)
        if d == "sanity":
            return synthetic.sanity_partition(n, seed=seed, device=self.device)
        raise ValueError(d)

    def new_epoch(self, epoch):
        """Fresh per-partition shuffles (seeded by partition and epoch).

        Written IN PLACE into one persistent buffer: captured HIP graphs hold
        its address, so it must never be reallocated.
        """
        perms = []
        for p in self.pids:
            g = torch.Generator(device="cpu")
            g.manual_seed(self.seed * 7919 + 104729 * p + epoch)
            perms.append(torch.randperm(self.n_train, generator=g).to(torch.int32))
        new = torch.stack(perms)
        if self.perm is None:
            self.perm = new.to(self.device)
        else:
            self.perm.copy_(new)

    def nbytes(self):
        tot = 0
        for t in (self.train_x, self.train_y, self.valid_x, self.valid_y):
            if t is not None:
                tot += t.numel() * t.element_size()
        return tot


_NORM_CACHE = {}


def _norm_consts(device, dtype=torch.float32):
    """Mean/std*255 tensors, created once per device (never inside a graph capture)."""
    key = (str(device), dtype)
    if key not in _NORM_CACHE:
        mean = torch.tensor(cat.IMAGENET_MEAN, device=device, dtype=dtype) * 255.0
        std = torch.tensor(cat.IMAGENET_STD, device=device, dtype=dtype) * 255.0
        _NORM_CACHE[key] = (mean, std)
    return _NORM_CACHE[key]


def gather_batch(store, train, part_of_row, cursor, B, x_out, y_out):
    """Fill ``x_out`` (packed input of G configs) and ``y_out`` [G, B] int32.

    ``part_of_row`` [G] int32 local partition per config row, ``cursor``
    [1] int32 batch index within the epoch permutation (device).
    """
    X = store.train_x if train else store.valid_x
    Y = store.train_y if train else store.valid_y
    perm = store.perm if train else store.valid_perm
    ds = store.dataset
    if use_hip("gather", X) and ds in ("imagenet", "tiny"):
        from ..ops import _hip
        _hip.gather_images(X, Y, perm, part_of_row, cursor, B, x_out, y_out)
        return
    G = part_of_row.shape[0]
    pr = part_of_row.long()
    pos = cursor.long() * B + torch.arange(B, device=X.device)          # [B]
    rows = perm[pr][:, pos].long()                                       # [G, B]
    y_out.copy_(Y[pr.unsqueeze(1), rows])
    xs = X[pr.unsqueeze(1), rows]                                        # [G, B, ...]
    if ds in ("imagenet", "tiny"):
        mean, std = _norm_consts(X.device)
        xf = (xs.float() - mean) / std                                   # [G, B, H, W, 3]
        xf = xf.permute(1, 2, 3, 0, 4)                                   # [B, H, W, G, 3]
        x_out.copy_(xf.reshape(x_out.shape))
    elif ds == "criteo":
        x_out.copy_(xs)                                                  # [G, B, 39] int32
    else:  # dense features
        x_out.copy_(xs.permute(1, 0, 2).reshape(x_out.shape))            # [B, G*F]


def input_buffers(store, G, B, dtype):
    """Static (graph-capturable) batch buffers for G configs."""
    dev = store.device
    if store.dataset in ("imagenet", "tiny"):
        _norm_consts(dev)
    ds = store.dataset
    if ds in ("imagenet", "tiny"):
        hw = store.train_x.shape[2]
        x = torch.zeros((B, hw, hw, G * 3), dtype=dtype, device=dev)
    elif ds == "criteo":
        x = torch.zeros((G, B, store.train_x.shape[2]), dtype=torch.int32, device=dev)
    else:
        x = torch.zeros((B, G * store.train_x.shape[2]), dtype=dtype, device=dev)
    y = torch.zeros((G, B), dtype=torch.int32, device=dev)
    return x, y
