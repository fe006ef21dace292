"""Direct-Access ETL throughput on the GPU box: decode Greenplum heap /
TOAST / pglz pages of every partition of a DA dataset through the windowed
loader (``data.da.da_partition_loader``: up to four (partition, split)
decodes in flight, C++ thread pool, pinned host memory) into HBM.

    python -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root /tmp/da [--threads 16]

Prints one JSON line: wall time, payload / on-disk GB, the consumer's wait
for decodes (``decode_s``) and for the pinned -> HBM copies + conversion
(``h2d_s``), the effective end-to-end GB/s, and the host CPU time the run
used (threads busy = CPU seconds / wall seconds).  Reference: the DA ETL of
``cerebro_gpdb/pg_page_reader.py`` took 83 525 s for ImageNet at 1 worker
(``plots/plots.ipynb:5545-5546``)."""

import argparse
import json
import os
import resource
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", required=True)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args(argv)
    import torch
    from ..data import da
    man = da.load_manifest(a.root)
    P = int(man["num_partitions"])
    stats = {}
    loader = da.da_partition_loader(a.root, a.device, nthreads=a.threads, stats=stats)
    pids = list(range(P))
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    loader.prefetch(pids)
    n_img = 0
    for p in pids:
        tx, ty, vx, vy = loader(p)
        n_img += tx.shape[0] + vx.shape[0]
        print("partition {} in HBM at {:.1f}s".format(p, time.perf_counter() - t0), file=sys.stderr,
              flush=True)
        del tx, ty, vx, vy
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    gb = stats["payload_bytes"] / 1e9
    print(json.dumps({
        "partitions": P, "images": n_img, "buffers": stats["buffers"], "threads": a.threads,
        "wall_s": round(wall, 3), "payload_GB": round(gb, 3),
        "stored_GB": round(stats["stored_bytes"] / 1e9, 3),
        "decode_wait_s": round(stats["decode_s"], 3), "h2d_s": round(stats["h2d_s"], 3),
        "end_to_end_GBps": round(gb / max(wall, 1e-9), 3),
        "cpu_s": round(cpu, 1), "threads_busy": round(cpu / max(wall, 1e-9), 2),
        "images_per_s": round(n_img / max(wall, 1e-9), 1)}))


if __name__ == "__main__":
    main()
