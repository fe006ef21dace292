"""Direct-Access ETL throughput on the GPU box: decode Greenplum heap /
TOAST / pglz pages of every partition of a DA dataset through the windowed
loader (``data.da.da_partition_loader``: up to four (partition, split)
decodes in flight, C++ thread pool, pinned host memory) into HBM.

    python -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root /tmp/da [--threads 16]
    python -m cerebro_ds_kpgi_amd.tools.da_etl_bench --root /tmp/da --decode_only \
        --concurrent 8 --threads 2

``--decode_only``: only the C++ reader (open + detoast + pglz into host
memory), per partition; ``--concurrent K`` runs K such readers at once in K
processes, reader i on partition i (the host side of K ranks loading their
own partitions on one node), and reports the aggregate decode GB/s.

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
    ap.add_argument("--decode_only", action="store_true")
    ap.add_argument("--only", type=int, default=-1, help="one partition (decode_only)")
    ap.add_argument("--concurrent", type=int, default=0)
    a = ap.parse_args(argv)
    if a.concurrent:
        return _concurrent(a)
    if a.decode_only:
        return _decode_only(a)
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
        "images_per_s": round(n_img / max(wall, 1e-9), 1),
        # the C++ reader's phases, summed over the (partition, split) decodes;
        # read_busy / read_wall = worker threads busy during the reads
        "phases_s": {k: round(stats.get(k, 0.0), 3) for k in (
            "open_s", "map_s", "heap_s", "index_s", "alloc_read_s", "read_wall_s",
            "read_busy_s", "read_copy_s", "read_pglz_s")},
        "read_threads_busy": round(stats.get("read_busy_s", 0.0) /
                                   max(stats.get("read_wall_s", 0.0), 1e-9), 2),
        "pglz_GBps_per_thread": round(gb / max(stats.get("read_pglz_s", 0.0), 1e-9), 3)}))


def _decode_only(a):
    from ..data import da
    man = da.load_manifest(a.root)
    parts = [a.only] if a.only >= 0 else list(range(int(man["num_partitions"])))
    tot, ph = 0, {}
    py = {"py_open_s": 0.0, "py_read_s": 0.0, "py_release_s": 0.0}
    t0 = time.perf_counter()
    for p in parts:
        for split in ("train", "valid"):
            d = da.seg_dir(a.root, p, man["dboid"])
            ta = time.perf_counter()
            r = da.DirectAccessReader(os.path.join(d, str(man[split]["relfilenode"])),
                                      os.path.join(d, str(man[split]["toast_relfilenode"])),
                                      a.threads)
            tb = time.perf_counter()
            recs = r.read(a.threads)
            tc = time.perf_counter()
            for _, _, x, y in recs:
                tot += x.nbytes + y.nbytes
            for k, v in r.stats().items():
                ph[k] = ph.get(k, 0.0) + v
            # the decoded arrays' pages go back to the OS here, and the
            # segment mappings are unmapped: both scale with the payload
            del recs
            r.close()
            td = time.perf_counter()
            py["py_open_s"] += tb - ta
            py["py_read_s"] += tc - tb
            py["py_release_s"] += td - tc
    ph.update(py)
    wall = time.perf_counter() - t0
    print(json.dumps({"partitions": parts, "threads": a.threads, "wall_s": round(wall, 3),
                      "payload_GB": round(tot / 1e9, 3),
                      "decode_GBps": round(tot / 1e9 / max(wall, 1e-9), 3),
                      "read_threads_busy": round(ph["read_busy_s"] / max(ph["read_wall_s"], 1e-9), 2),
                      "phases_s": {k: round(v, 3) for k, v in ph.items() if k.endswith("_s")}}),
          flush=True)


def _concurrent(a):
    import subprocess
    cmd = [sys.executable, "-m", "cerebro_ds_kpgi_amd.tools.da_etl_bench", "--root", a.root,
           "--decode_only", "--threads", str(a.threads)]
    t0 = time.perf_counter()
    procs = [subprocess.Popen(cmd + ["--only", str(i)], stdout=subprocess.PIPE, text=True)
             for i in range(a.concurrent)]
    outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
    wall = time.perf_counter() - t0
    gb = sum(o["payload_GB"] for o in outs)
    print(json.dumps({"concurrent": a.concurrent, "threads_each": a.threads,
                      "wall_s": round(wall, 3), "payload_GB": round(gb, 3),
                      "aggregate_decode_GBps": round(gb / max(wall, 1e-9), 3),
                      "per_reader_GBps": [o["decode_GBps"] for o in outs],
                      "per_reader_threads_busy": [o["read_threads_busy"] for o in outs]}))
    return 0 if all(p.returncode == 0 for p in procs) else 1


if __name__ == "__main__":
    main()
