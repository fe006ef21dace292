"""Synthetic datasets with the reference's shapes (no datasets offline).

* ImageNet-112: uint8 ``[n, 112, 112, 3]`` + int32 labels in [0, 1000)
  (reference preprocessing ``cerebro_gpdb/preprocessing/imagenet/
  generate_h5_file.py``; input shape ``imagenetcat.py:17``).  Images are a
  per-class low-frequency template plus noise, so the task is *learnable*
  and loss curves are meaningful, generated directly on the target device.
* Criteo: the one-hot feature vector of SURVEY.md A14 represented by its 39
  active column ids per row (13 continuous features bucketised into 50
  buckets with boundaries ``1.5**j - 0.51``, 26 categorical features hashed
  into 256 bins), int32 ``[n, 39]``; labels 0/1 from a planted logistic rule.
* ``sanity``: 4 dense features, 3 classes; ``tiny``: 32x32x3, 10 classes.
"""

import numpy as np
import torch

from ..config import catalog as cat


def _gen(seed, device):
    g = torch.Generator(device=device if torch.device(device).type == "cuda" else "cpu")
    g.manual_seed(int(seed))
    return g


def image_partition(n, hw=112, num_classes=1000, seed=0, device="cpu", chunk=8192,
                    template_seed=cat.SEED):
    """uint8 images [n, hw, hw, 3] and int32 labels [n] on ``device``."""
    dev = torch.device(device)
    gt = _gen(template_seed, "cpu")
    tmpl = torch.randint(40, 216, (num_classes, 4, 4, 3), generator=gt, dtype=torch.int16)
    tmpl = tmpl.to(dev)
    g = _gen(seed, dev)
    labels = torch.randint(0, num_classes, (n,), generator=g, device=dev, dtype=torch.int32)
    images = torch.empty((n, hw, hw, 3), dtype=torch.uint8, device=dev)
    rep = (hw + 3) // 4
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        t = tmpl[labels[s:e].long()]                                         # [c, 4, 4, 3]
        t = t.repeat_interleave(rep, 1).repeat_interleave(rep, 2)[:, :hw, :hw]
        noise = torch.randint(-40, 40, (e - s, hw, hw, 3), generator=g, device=dev,
                              dtype=torch.int16)
        images[s:e] = (t + noise).clamp_(0, 255).to(torch.uint8)
    return images, labels


def criteo_partition(n, seed=0, device="cpu"):
    """int32 active-column ids [n, 39] and int32 labels [n]."""
    dev = torch.device(device)
    g = _gen(seed, dev)
    nc, nk = cat.CRITEO_NUM_CONTINUOUS, cat.CRITEO_NUM_CATEGORICAL
    nb, nh = cat.CRITEO_BUCKETS, cat.CRITEO_HASH_BINS
    cont = torch.randint(0, nb, (n, nc), generator=g, device=dev, dtype=torch.int32)
    cont = cont + torch.arange(nc, device=dev, dtype=torch.int32) * nb
    catg = torch.randint(0, nh, (n, nk), generator=g, device=dev, dtype=torch.int32)
    catg = catg + nc * nb + torch.arange(nk, device=dev, dtype=torch.int32) * nh
    idx = torch.cat([cont, catg], 1).contiguous()
    # planted rule: a fixed random weight per column, label = 1 iff score > median
    gw = _gen(cat.SEED, "cpu")
    w = torch.randn(cat.INPUT_SHAPE_CRITEO[0], generator=gw).to(dev)
    score = w[idx.long()].sum(1)
    labels = (score > score.median()).to(torch.int32)
    return idx, labels


def criteo_bucket(x):
    """Bucket id of a continuous Criteo value (boundaries 1.5**j - 0.51, j<49);
    reference ``preprocessing_criteo.py:48-57,84-95``."""
    bounds = 1.5 ** np.arange(cat.CRITEO_BUCKETS - 1) - 0.51
    return int(np.searchsorted(bounds, x, side="right"))


def sanity_partition(n, seed=0, device="cpu"):
    dev = torch.device(device)
    g = _gen(seed, dev)
    labels = torch.randint(0, 3, (n,), generator=g, device=dev, dtype=torch.int32)
    centers = torch.tensor([[0., 0, 1, 1], [1, 1, 0, 0], [1, 0, 1, 0]], device=dev)
    x = centers[labels.long()] + 0.3 * torch.randn((n, 4), generator=g, device=dev)
    return x.float(), labels


def tiny_partition(n, seed=0, device="cpu"):
    return image_partition(n, hw=32, num_classes=10, seed=seed, device=device)
