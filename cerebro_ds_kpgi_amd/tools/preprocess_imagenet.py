"""ImageNet JPEG folders -> 112x112 uint8 partitions.

Reference pipeline (``cerebro_gpdb/preprocessing/imagenet``):
``extract_train.py`` untars the per-synset train tars into ``train/<synset>/``;
``extract_valid.py`` sorts the 50 000 validation JPEGs into
``valid/<synset>/`` using ``ILSVRC2012_mapping.txt`` (line i = synset of
class id i) and ``ILSVRC2012_valid_ground_truth.txt`` (``<file> <class id>``);
``generate_h5_file.py`` assigns label ids to synsets in directory order,
shuffles and packs; the (commented-out) transform resizes to 112x112 and
normalises with mean [0.485, 0.456, 0.406] / std [0.229, 0.224, 0.225].

Here: label ids follow SORTED synset order (deterministic, unlike
``os.listdir``); images are decoded + resized with PIL in a process pool and
stored as uint8 (normalisation happens on the GPU in the batch-gather
kernel, with the same constants); the shuffled set is split into P
partitions in the ``data.fs`` layout.

    python -m cerebro_ds_kpgi_amd.tools.preprocess_imagenet --train_dir train --valid_dir valid \
        --out /data/imagenet --partitions 8 [--valid_tar_layout valid_flat \
        --mapping ILSVRC2012_mapping.txt --ground_truth ILSVRC2012_valid_ground_truth.txt]
"""

import argparse
import os
from multiprocessing import Pool

import numpy as np

from ..config import catalog as cat

HW = cat.INPUT_SHAPE[0]


def synsets(train_dir):
    return sorted(d for d in os.listdir(train_dir) if d.startswith("n") and
                  os.path.isdir(os.path.join(train_dir, d)))


def list_folder(root, label_of):
    items = []
    for syn in sorted(os.listdir(root)):
        d = os.path.join(root, syn)
        if syn not in label_of or not os.path.isdir(d):
            continue
        for f in sorted(os.listdir(d)):
            if f.upper().endswith((".JPEG", ".JPG", ".PNG")):
                items.append((os.path.join(d, f), label_of[syn]))
    return items


def list_flat_valid(flat_dir, mapping, ground_truth, label_of):
    """Validation JPEGs in one folder + the reference's two mapping files."""
    with open(mapping) as f:
        syn_of_id = {str(i): line.strip() for i, line in enumerate(f)}
    items = []
    with open(ground_truth) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            fname, cid = line.split(" ")
            syn = syn_of_id[cid]
            if syn in label_of:
                items.append((os.path.join(flat_dir, fname), label_of[syn]))
    return items


def _load(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB").resize((HW, HW), Image.BILINEAR), dtype=np.uint8)


def pack(items, out, split, partitions, workers=8, seed=cat.SEED):
    rs = np.random.RandomState(seed)
    order = rs.permutation(len(items))
    items = [items[i] for i in order]
    os.makedirs(os.path.join(out, split), exist_ok=True)
    counts = []
    with Pool(workers) as pool:
        for p, sel in enumerate(np.array_split(np.arange(len(items)), partitions)):
            paths = [items[i][0] for i in sel]
            x = np.stack(pool.map(_load, paths, chunksize=64)) if paths else \
                np.zeros((0, HW, HW, 3), np.uint8)
            y = np.asarray([items[i][1] for i in sel], np.int32)
            stem = os.path.join(out, split, "{}_{}".format(split, p))
            np.save(stem + ".images.npy", x)
            np.save(stem + ".labels.npy", y)
            counts.append(len(sel))
    return counts


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--train_dir", required=True)
    ap.add_argument("--valid_dir", default="", help="valid/<synset>/*.JPEG")
    ap.add_argument("--valid_flat", default="", help="flat validation folder (+ mapping files)")
    ap.add_argument("--mapping", default="")
    ap.add_argument("--ground_truth", default="")
    ap.add_argument("--out", required=True)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args(argv)
    syns = synsets(a.train_dir)
    label_of = {s: i for i, s in enumerate(syns)}
    out = {"classes": len(syns)}
    out["train"] = pack(list_folder(a.train_dir, label_of), a.out, "train", a.partitions,
                        a.workers)
    if a.valid_dir:
        valid = list_folder(a.valid_dir, label_of)
    elif a.valid_flat:
        valid = list_flat_valid(a.valid_flat, a.mapping, a.ground_truth, label_of)
    else:
        valid = []
    out["valid"] = pack(valid, a.out, "valid", a.partitions, a.workers)
    with open(os.path.join(a.out, "synsets.txt"), "w") as f:
        f.write("\n".join(syns) + "\n")
    print("imagenet:", out)
    return out


if __name__ == "__main__":
    main()
