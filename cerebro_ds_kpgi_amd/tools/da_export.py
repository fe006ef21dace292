"""Export Direct-Access partitions to the filesystem layout (the role of the
reference's unload + ETL pipeline: ``unload_*.sql`` through gpfdist, then
``etl_imagenet.py`` / ``etl_criteo.py`` parsing the text rows into h5/npy;
SURVEY.md A12).  Pages are parsed by the C++ reader, not via the database.

    python -m cerebro_ds_kpgi_amd.tools.da_export --da_root /data/imagenet_da --out /data/imagenet
"""

import argparse
import os

import numpy as np

from ..data import criteo, da


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--da_root", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    man = da.load_manifest(a.da_root)
    loader = da.da_partition_loader(a.da_root, "cpu")
    counts = {}
    for p in range(man["num_partitions"]):
        tx, ty, vx, vy = loader(p)
        for split, x, y in (("train", tx, ty), ("valid", vx, vy)):
            os.makedirs(os.path.join(a.out, split), exist_ok=True)
            stem = os.path.join(a.out, split, "{}_{}".format(split, p))
            if man["dataset"] == "imagenet":
                np.save(stem + ".images.npy", x.numpy())
                np.save(stem + ".labels.npy", y.numpy().astype(np.int32))
            else:
                np.save(stem + ".npy", criteo.ids_to_dense(x.numpy(), y.numpy()))
            counts.setdefault(split, 0)
            counts[split] += int(y.shape[0])
    print("exported", counts)
    return counts


if __name__ == "__main__":
    main()
