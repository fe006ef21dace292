"""Generate a synthetic Direct-Access dataset: Greenplum-format heap + TOAST
segment files per partition (``{root}/gpseg{i}/base/{dboid}/{relfilenode}``)
plus the manifest, replacing the reference's load/pack pipeline
(``load_imagenet.py``, ``load_criteo.py``).

    python -m cerebro_ds_kpgi_amd.tools.make_da_data --root /data/gp --partitions 8 \
        --dataset imagenet --train 160160 --valid 6250
"""

import argparse
import time

from ..config import catalog as cat
from ..data import da


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", required=True)
    ap.add_argument("--dataset", choices=["imagenet", "criteo"], default="imagenet")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--train", type=int, default=cat.IMAGENET_COUNT_PER_PAR)
    ap.add_argument("--valid", type=int, default=cat.IMAGENET_VALID_TOTAL // 8)
    ap.add_argument("--buffer_size", type=int, default=cat.TRAIN_BUFFER_SIZE)
    ap.add_argument("--unique", type=int, default=0,
                    help="generate only this many partitions; the rest are hard links to "
                         "them (for a disk smaller than the whole dataset)")
    ap.add_argument("--jobs", type=int, default=1, help="partitions generated concurrently")
    a = ap.parse_args(argv)
    t = time.time()
    da.write_dataset(a.root, a.dataset, a.partitions, a.train, a.valid, a.buffer_size,
                     verbose=True, unique=a.unique or None, jobs=a.jobs)
    print("wrote {} partitions to {} in {:.1f}s".format(a.partitions, a.root, time.time() - t))


if __name__ == "__main__":
    main()
