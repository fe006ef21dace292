"""Generate synthetic filesystem partitions in the reference layout
(``{root}/{train,valid}/{train,valid}_{i}.*``) for the
``run_filesystem_*`` entry points.

    python -m cerebro_ds_kpgi_amd.tools.make_fs_data --root /data/imagenet --partitions 8 \
        --dataset imagenet --train 160160 --valid 6250
"""

import argparse
import json
import os
import time

from ..config import catalog as cat
from ..data import fs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", required=True)
    ap.add_argument("--dataset", choices=["imagenet", "criteo"], default="imagenet")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--train", type=int, default=cat.IMAGENET_COUNT_PER_PAR)
    ap.add_argument("--valid", type=int, default=cat.IMAGENET_VALID_TOTAL // 8)
    a = ap.parse_args(argv)
    t = time.time()
    catalog = fs.write_fs_dataset(a.root, a.dataset, a.partitions, a.train, a.valid)
    with open(os.path.join(a.root, "catalog.json"), "w") as f:
        json.dump(catalog, f, indent=1)
    print("wrote {} partitions to {} in {:.1f}s".format(a.partitions, a.root, time.time() - t))


if __name__ == "__main__":
    main()
