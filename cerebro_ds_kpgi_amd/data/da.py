"""Direct Access (DA): read Greenplum-format packed-table partitions straight
from their heap/TOAST segment files, bypassing the database.

* ``DirectAccessReader`` — ctypes front-end of ``libcerebro_da.so``
  (csrc/da): parses heap pages, indexes TOAST chunks, detoasts +
  pglz-decompresses all buffers on a thread pool into *pinned* host memory,
  from which partitions go to HBM with asynchronous copies.
* ``write_partition`` / ``write_dataset`` — produce the same on-disk format
  (``{root}/gpseg{i}/base/{dboid}/{relfilenode}[.N]`` + toast relfilenode +
  a shapes/manifest JSON replacing the reference's ``sys_cat.dill`` catalog,
  ``cerebro_gpdb/da.py:26,96-183``).
* ``input_fn(file_path)`` — the reference's DA worker contract
  (``cerebro_gpdb/da.py:29-58``): ``{buffer_id: {'independent_var': f32[N,...],
  'dependent_var': i16[N, classes]}}``.
* ``da_partition_loader`` — plugs DA partitions into the HBM partition store.

Payloads: independent_var float32 ``[N, 112, 112, 3]`` (or ``[N, 7306]``
one-hot for Criteo), dependent_var int16 one-hot ``[N, classes]``
(``pg_page_reader.py:177-182``).
"""

import ctypes
import json
import os
import re

import numpy as np

from ..config import catalog as cat

_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib",
                        "libcerebro_da.so")
SEG_BYTES = 1 << 30        # Greenplum segment file size
DBOID = 16384
TRAIN_RELFILENODE, TRAIN_TOAST = 24576, 24580
VALID_RELFILENODE, VALID_TOAST = 24590, 24594
MANIFEST = "da_manifest.json"


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            from ..tools.build import build_da
            build_da()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        L.cer_pglz_compress.argtypes = [vp, i64, vp, i64]
        L.cer_pglz_compress.restype = i64
        L.cer_pglz_decompress.argtypes = [vp, i64, vp, i64]
        L.cer_pglz_decompress.restype = i64
        L.cer_da_last_error.restype = ctypes.c_char_p
        L.cer_da_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.cer_da_open.restype = vp
        L.cer_da_open2.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.cer_da_open2.restype = vp
        L.cer_da_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.cer_da_count.argtypes = [vp]
        L.cer_da_info.argtypes = [vp, ctypes.c_int, ctypes.POINTER(i32), ctypes.POINTER(i32),
                                  ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.cer_da_read.argtypes = [vp, ctypes.c_int, vp, vp, vp, ctypes.c_int]
        L.cer_da_close.argtypes = [vp]
        L.cer_da_writer_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32,
                                         ctypes.c_uint32, i64]
        L.cer_da_writer_open.restype = vp
        L.cer_da_writer_add.argtypes = [vp, i32, i32, vp, i64, vp, i64, ctypes.c_int]
        L.cer_da_writer_add_batch.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp,
                                              ctypes.c_int, ctypes.c_int]
        L.cer_da_writer_close.argtypes = [vp]
        _LIB = L
    return _LIB


def _err():
    return lib().cer_da_last_error().decode()


# ---------------------------------------------------------------------------
# pglz
# ---------------------------------------------------------------------------
def pglz_compress(data):
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    dst = np.empty(max(len(src) + 16, 16), dtype=np.uint8)
    n = lib().cer_pglz_compress(src.ctypes.data, len(src), dst.ctypes.data, len(dst))
    if n < 0:
        return None
    return dst[:n].tobytes()


def pglz_decompress(comp, rawsize):
    src = np.frombuffer(bytes(comp), dtype=np.uint8)
    dst = np.empty(rawsize, dtype=np.uint8)
    n = lib().cer_pglz_decompress(src.ctypes.data, len(src), dst.ctypes.data, rawsize)
    if n < 0:
        raise ValueError("compressed data is corrupt")
    return dst.tobytes()


# ---------------------------------------------------------------------------
# reader
# ---------------------------------------------------------------------------
STAT_KEYS = ("map_s", "heap_s", "index_s", "read_wall_s", "read_busy_s", "read_copy_s",
             "read_pglz_s", "read_threads", "index_threads")


class DirectAccessReader(object):
    """``nthreads``: threads of the TOAST index scan at open (the read takes
    its own count)."""

    def __init__(self, heap_path, toast_path, nthreads=16):
        self.h = lib().cer_da_open2(heap_path.encode(), toast_path.encode(), int(nthreads))
        if not self.h:
            raise IOError("DA open failed: {}".format(_err()))

    def stats(self):
        """Phase timings of this reader (s): mmap of the segment files, heap
        parse, TOAST index (open); wall, summed worker busy / TOAST-chunk copy
        / pglz time of the last ``read``; thread counts."""
        out = (ctypes.c_double * 9)()
        lib().cer_da_stats(self.h, out)
        return dict(zip(STAT_KEYS, list(out)))

    def __len__(self):
        return lib().cer_da_count(self.h)

    def info(self, i):
        dk, bid = ctypes.c_int32(), ctypes.c_int32()
        ni, nd = ctypes.c_int64(), ctypes.c_int64()
        if lib().cer_da_info(self.h, i, ctypes.byref(dk), ctypes.byref(bid), ctypes.byref(ni),
                             ctypes.byref(nd)) != 0:
            raise IndexError(i)
        return dk.value, bid.value, ni.value, nd.value

    def read(self, nthreads=16, pinned=False, indices=None):
        """List of (dist_key, buffer_id, indep bytes array, dep bytes array)."""
        idx = list(range(len(self))) if indices is None else list(indices)
        infos = [self.info(i) for i in idx]
        if pinned:
            import torch
            # allocated pinned (``.pin_memory()`` on a pageable tensor would
            # allocate twice and copy)
            ind = [torch.empty(ni, dtype=torch.uint8, pin_memory=True) for _, _, ni, _ in infos]
            dep = [torch.empty(nd, dtype=torch.uint8, pin_memory=True) for _, _, _, nd in infos]
            ip = [t.data_ptr() for t in ind]
            dp = [t.data_ptr() for t in dep]
        else:
            ind = [np.empty(ni, dtype=np.uint8) for _, _, ni, _ in infos]
            dep = [np.empty(nd, dtype=np.uint8) for _, _, _, nd in infos]
            ip = [a.ctypes.data for a in ind]
            dp = [a.ctypes.data for a in dep]
        n = len(idx)
        c_idx = (ctypes.c_int * n)(*idx)
        c_ip = (ctypes.c_void_p * n)(*ip)
        c_dp = (ctypes.c_void_p * n)(*dp)
        rc = lib().cer_da_read(self.h, n, ctypes.cast(c_idx, ctypes.c_void_p),
                               ctypes.cast(c_ip, ctypes.c_void_p),
                               ctypes.cast(c_dp, ctypes.c_void_p), nthreads)
        if rc != 0:
            raise IOError("DA read failed: {}".format(_err()))
        return [(dk, bid, a, b) for (dk, bid, _, _), a, b in zip(infos, ind, dep)]

    def close(self):
        if self.h:
            lib().cer_da_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------
def seg_dir(root, seg, dboid=DBOID):
    return os.path.join(root, "gpseg{}".format(seg), "base", str(dboid))


def write_partition(heap_path, toast_path, buffers, dist_key, toastrelid=99999,
                    first_valueid=1 << 20, seg_bytes=SEG_BYTES, dep_inline=True, log=None,
                    threads=None):
    """buffers: iterable of (buffer_id, indep ndarray, dep ndarray), consumed
    ``threads`` at a time (the native writer compresses a batch's datums in
    parallel); ``log``: optional progress callback (buffers, bytes written)."""
    os.makedirs(os.path.dirname(heap_path), exist_ok=True)
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    w = lib().cer_da_writer_open(heap_path.encode(), toast_path.encode(), toastrelid,
                                 first_valueid, seg_bytes)
    if not w:
        raise IOError("DA writer open failed: {}".format(_err()))
    done = nbytes = 0

    def flush(batch):
        n = len(batch)
        arr = lambda t, v: (t * n)(*v)
        rc = lib().cer_da_writer_add_batch(
            w, n, arr(ctypes.c_int32, [int(dist_key)] * n), arr(ctypes.c_int32, [b[0] for b in batch]),
            arr(ctypes.c_void_p, [b[1].ctypes.data for b in batch]),
            arr(ctypes.c_int64, [b[1].nbytes for b in batch]),
            arr(ctypes.c_void_p, [b[2].ctypes.data for b in batch]),
            arr(ctypes.c_int64, [b[2].nbytes for b in batch]), int(bool(dep_inline)), threads)
        if rc != 0:
            lib().cer_da_writer_close(w)
            raise IOError("DA write failed: {}".format(_err()))
        return sum(b[1].nbytes + b[2].nbytes for b in batch)

    batch = []
    for bid, indep, dep in buffers:
        batch.append((int(bid), np.ascontiguousarray(indep), np.ascontiguousarray(dep)))
        if len(batch) == threads:
            nbytes += flush(batch)
            done += len(batch)
            batch = []
            if log is not None:
                log(done, nbytes)
    if batch:
        nbytes += flush(batch)
        done += len(batch)
        if log is not None:
            log(done, nbytes)
    if lib().cer_da_writer_close(w) != 0:
        raise IOError("DA writer close failed: {}".format(_err()))


def write_dataset(root, dataset, num_partitions, n_train, n_valid, buffer_size=cat.TRAIN_BUFFER_SIZE,
                  seed=cat.SEED, seg_bytes=SEG_BYTES, verbose=False, unique=None, jobs=1):
    """Synthetic packed tables for ``num_partitions`` segments + manifest.
    Buffers are converted to the float32 payload one at a time (a full
    ImageNet partition is 24 GB as float32); ``verbose`` prints progress.

    ``unique``: only the first ``unique`` partitions are generated; segment
    ``p >= unique`` is a directory of HARD LINKS to segment ``p % unique``'s
    files (same bytes, so the same pages are walked, detoasted and decoded
    again for it).  For disks that cannot hold every partition (8 full
    ImageNet-112 partitions are ~105 GB stored); the manifest records the
    links.  ``jobs``: partitions generated by that many processes at once."""
    unique = num_partitions if not unique else min(int(unique), num_partitions)
    args = [(root, dataset, p, n_train, n_valid, buffer_size, seed, seg_bytes, verbose)
            for p in range(unique)]
    if jobs > 1 and unique > 1:
        import concurrent.futures as cf
        import multiprocessing as mp     # spawn: a fork of a process with torch's
        # intra-op thread pool running deadlocks in the child's first torch op
        with cf.ProcessPoolExecutor(min(jobs, unique), mp_context=mp.get_context("spawn")) as ex:
            parts = list(ex.map(_write_one, *zip(*args)))
    else:
        parts = [_write_one(*a) for a in args]
    shapes = {"train": [], "valid": []}
    for sh in parts:
        for split in shapes:
            shapes[split].extend(sh[split])
    links = {}
    for p in range(unique, num_partitions):
        src, dst = seg_dir(root, p % unique), seg_dir(root, p)
        os.makedirs(dst, exist_ok=True)
        for f in sorted(os.listdir(src)):
            if not os.path.exists(os.path.join(dst, f)):
                os.link(os.path.join(src, f), os.path.join(dst, f))
        links[str(p)] = p % unique
        for split in shapes:
            shapes[split].extend(dict(s, dist_key=p) for s in parts[p % unique][split])
    man = {"dataset": dataset, "num_partitions": num_partitions, "dboid": DBOID,
           "train": {"relfilenode": TRAIN_RELFILENODE, "toast_relfilenode": TRAIN_TOAST},
           "valid": {"relfilenode": VALID_RELFILENODE, "toast_relfilenode": VALID_TOAST},
           "shapes": shapes}
    if links:
        man["linked_segments"] = links
    with open(os.path.join(root, MANIFEST), "w") as f:
        json.dump(man, f)
    return man


def _write_one(root, dataset, p, n_train, n_valid, buffer_size, seed, seg_bytes, verbose):
    """One partition's train + valid tables; returns its manifest shapes."""
    import sys
    import time
    from . import synthetic
    shapes = {"train": [], "valid": []}
    for split, n, rel, toast in (("train", n_train, TRAIN_RELFILENODE, TRAIN_TOAST),
                                 ("valid", n_valid, VALID_RELFILENODE, VALID_TOAST)):
        s = seed * 1000 + 2 * p + (split == "valid")
        if dataset == "imagenet":
            x, y = synthetic.image_partition(n, seed=s)
            x = x.numpy()                     # uint8; float32 per buffer below
            classes = cat.NUM_CLASSES
        elif dataset == "criteo":
            idx, y = synthetic.criteo_partition(n, seed=s)
            x = np.zeros((n, cat.INPUT_SHAPE_CRITEO[0]), dtype=np.float32)
            np.put_along_axis(x, idx.numpy().astype(np.int64), 1.0, axis=1)
            classes = cat.NUM_CLASSES_CRITEO
        else:
            raise ValueError(dataset)
        yy = np.zeros((n, classes), dtype=np.int16)
        yy[np.arange(n), y.numpy()] = 1
        for bid, s0 in enumerate(range(0, n, buffer_size)):
            e = min(n, s0 + buffer_size)
            shapes[split].append({"dist_key": p, "buffer_id": bid,
                                  "independent_var_shape": list(x[s0:e].shape),
                                  "dependent_var_shape": [e - s0, classes]})
        bufs = ((bid, x[s0:min(n, s0 + buffer_size)].astype(np.float32),
                 yy[s0:min(n, s0 + buffer_size)])
                for bid, s0 in enumerate(range(0, n, buffer_size)))
        nbuf = (n + buffer_size - 1) // buffer_size
        t0 = time.time()

        def log(i, nb, p=p, split=split, nbuf=nbuf, t0=t0):
            if verbose:
                print("  partition {} {}: {}/{} buffers, {:.2f} GB in {:.1f}s".format(
                    p, split, i, nbuf, nb / 1e9, time.time() - t0), flush=True)
                sys.stdout.flush()
        d = seg_dir(root, p)
        write_partition(os.path.join(d, str(rel)), os.path.join(d, str(toast)), bufs, p,
                        toastrelid=toast, first_valueid=(p + 1) << 20, seg_bytes=seg_bytes,
                        log=log)
    return shapes


# ---------------------------------------------------------------------------
# catalog + reference-compatible input_fn
# ---------------------------------------------------------------------------
def load_manifest(root):
    with open(os.path.join(root, MANIFEST)) as f:
        return json.load(f)


def generate_cats(root, size):
    """(data_cat, sys_cats) like ``DirectAccessClient.generate_cats``: the
    Cerebro data catalog with an identity availability matrix + the system
    catalog (relfilenodes, dboid, shapes)."""
    man = load_manifest(root)
    data_cat = {
        "data_root": root,
        "train": ["gpseg{}/base/{}/train".format(i, man["dboid"]) for i in range(size)],
        "train_availability": np.eye(size, dtype=int).tolist(),
        "valid": ["gpseg{}/base/{}/valid".format(i, man["dboid"]) for i in range(size)],
        "valid_availability": np.eye(size, dtype=int).tolist(),
    }
    return data_cat, man


def _paths(root, file_path, man):
    m = re.search(r"gpseg(\d+)", file_path)
    seg = int(m.group(1))
    split = "valid" if file_path.rstrip("/").endswith("valid") else "train"
    d = seg_dir(root, seg, man["dboid"])
    return (os.path.join(d, str(man[split]["relfilenode"])),
            os.path.join(d, str(man[split]["toast_relfilenode"])), seg, split)


def input_fn(file_path, root=None, nthreads=16):
    """Reference DA worker contract: catalog path -> {buffer_id: {...}}."""
    root = root or os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(file_path))))
    man = load_manifest(root)
    heap, toast, seg, split = _paths(root, file_path, man)
    shapes = {(s["dist_key"], s["buffer_id"]): s for s in man["shapes"][split]}
    r = DirectAccessReader(heap, toast)
    out = {}
    for dk, bid, a, b in r.read(nthreads):
        sh = shapes[(dk, bid)]
        out[bid] = {"independent_var": np.frombuffer(a.tobytes(), np.float32).reshape(
                        sh["independent_var_shape"]),
                    "dependent_var": np.frombuffer(b.tobytes(), np.int16).reshape(
                        sh["dependent_var_shape"])}
    r.close()
    return out


class NonIntegralPixels(ValueError):
    """A DA ImageNet partition holds float pixels that are not integers in
    [0, 255]: storing it as uint8 in HBM would silently change the data."""


def da_partition_loader(root, device, nthreads=16, stats=None):
    """Loader for ``PartitionStore``: DA partition -> HBM tensors (uint8
    images / int32 active-column ids, int32 labels).

    Buffers are detoasted + pglz-decoded by the C++ thread pool into pinned
    host memory, then copied to the device and converted buffer by buffer on
    a side copy stream (the caller's stream only waits at the end).  ImageNet
    payloads are float32 pixels; they are stored as uint8 only after a
    device-side check that every value is an integer in [0, 255]
    (``NonIntegralPixels`` otherwise — never a silent quantisation).
    ``loader.prefetch(pids)`` (called by the partition store) lets up to four
    (partition, split) decodes run ahead on a thread pool.
    ``stats`` (a dict) accumulates ETL timings: ``decode_s`` (wall time the
    consumer waited for the C++ reader), ``h2d_s`` (copies + conversion,
    wall), the reader's phases summed over decodes (``DirectAccessReader.stats``:
    ``map_s``, ``heap_s``, ``index_s``, ``read_wall_s``, ``read_busy_s``,
    ``read_copy_s``, ``read_pglz_s``, plus ``open_s`` and ``alloc_read_s`` as
    seen from Python), ``payload_bytes``
    (decompressed), ``stored_bytes`` (on disk, heap + TOAST) and ``buffers``."""
    import time
    import torch
    man = load_manifest(root)
    dev = torch.device(device)
    cuda = dev.type == "cuda"
    copy_stream = torch.cuda.Stream(device=dev) if cuda else None
    st = stats if stats is not None else {}
    for k in ("decode_s", "h2d_s", "payload_bytes", "stored_bytes", "buffers"):
        st.setdefault(k, 0)

    def convert(x, dataset):
        if dataset == "imagenet":
            q = x.round()
            bad = ((q != x) | (x < 0) | (x > 255)).any()
            return q.to(torch.uint8), bad
        nnz = int((x[0] != 0).sum().item())
        return torch.nonzero(x, as_tuple=False)[:, 1].view(x.shape[0], nnz).to(torch.int32), None

    # decode pipeline: the C++ reader releases the GIL, so up to WINDOW
    # (partition, split) decodes run concurrently ahead of the consumer
    # (bounded: each holds its decompressed payload in pinned memory)
    import concurrent.futures as cf
    # each decode holds its decompressed payload in pinned memory (25 GB for
    # a full ImageNet-112 train split): CER_DA_WINDOW bounds the host memory
    WINDOW = max(1, int(os.environ.get("CER_DA_WINDOW", "4")))
    jobs, futs = [], {}
    # the decode pool lives while a prefetch window is open: created lazily
    # on the first submit, shut down once the window drains (every prefetched
    # job consumed), re-created by the next store that uses this loader
    pool = [None]

    def submit(*a):
        if pool[0] is None:
            pool[0] = cf.ThreadPoolExecutor(max_workers=WINDOW)
        return pool[0].submit(*a)

    def drain():
        if pool[0] is not None and not futs:
            pool[0].shutdown(wait=False)
            pool[0] = None

    def decode(p, split, threads):
        heap = os.path.join(seg_dir(root, p, man["dboid"]), str(man[split]["relfilenode"]))
        toast = os.path.join(seg_dir(root, p, man["dboid"]), str(man[split]["toast_relfilenode"]))
        stored = 0
        for path in (heap, toast):
            seg = 0
            f = path
            while os.path.exists(f):
                stored += os.path.getsize(f)
                seg += 1
                f = "{}.{}".format(path, seg)
        t0 = time.perf_counter()
        r = DirectAccessReader(heap, toast, threads)
        t1 = time.perf_counter()
        recs = sorted(r.read(threads, pinned=cuda), key=lambda t: t[1])
        t2 = time.perf_counter()
        ph = r.stats()
        r.close()
        ph["open_s"] = t1 - t0
        ph["alloc_read_s"] = t2 - t1          # pinned staging allocation + read
        return recs, stored, ph

    def prefetch(pids):
        """The store's partitions, in load order: start decoding ahead."""
        del jobs[:]
        for f in futs.values():                 # a previous window never consumed
            f.cancel()
        futs.clear()
        drain()
        jobs.extend((p, sp) for p in pids for sp in ("train", "valid"))

    def fetch(p, split):
        key = (p, split)
        if key in jobs:
            i = jobs.index(key)
            for k in jobs[i:i + WINDOW]:
                if k not in futs:
                    # every decode gets the whole thread budget: the jobs
                    # are uneven (a train split is ~25x its valid split) and
                    # a 1/WINDOW share left a lone train decode on 4 threads
                    futs[k] = submit(decode, k[0], k[1], nthreads)
        fut = futs.pop(key, None)
        return fut.result() if fut is not None else decode(p, split, nthreads)

    def load_split(p, split):
        shapes = {(s["dist_key"], s["buffer_id"]): s for s in man["shapes"][split]}
        t0 = time.perf_counter()
        recs, stored, ph = fetch(p, split)
        st["stored_bytes"] += stored
        for k, v in ph.items():
            if k.endswith("_s"):
                st[k] = st.get(k, 0.0) + v
            else:
                st[k] = max(st.get(k, 0), v)
        t1 = time.perf_counter()
        st["decode_s"] += t1 - t0
        xs, ys, bads = [], [], []
        ctx = torch.cuda.stream(copy_stream) if cuda else _Null()
        with ctx:
            for dk, bid, a, b in recs:
                sh = shapes[(dk, bid)]
                a = a if isinstance(a, torch.Tensor) else torch.from_numpy(a)
                b = b if isinstance(b, torch.Tensor) else torch.from_numpy(b)
                st["payload_bytes"] += a.numel() * a.element_size() + b.numel() * b.element_size()
                st["buffers"] += 1
                x = a.view(torch.float32).view(sh["independent_var_shape"]).to(dev, non_blocking=True)
                y = b.view(torch.int16).view(sh["dependent_var_shape"]).to(dev, non_blocking=True)
                x, bad = convert(x, man["dataset"])
                xs.append(x)
                ys.append(y.argmax(1).to(torch.int32))
                if bad is not None:
                    bads.append(bad)
            x = torch.cat(xs)
            y = torch.cat(ys)
            bad = torch.stack(bads).any() if bads else None
        if cuda:
            torch.cuda.current_stream(dev).wait_stream(copy_stream)
            for t in (x, y):
                t.record_stream(torch.cuda.current_stream(dev))
        if bad is not None and bool(bad):           # one sync per split
            raise NonIntegralPixels(
                "DA partition {} ({}) holds non-integral or out-of-range pixel values; "
                "the HBM store keeps images as uint8 — re-export integral 0..255 pixels "
                "(raw images) instead of normalised floats".format(p, split))
        st["h2d_s"] += time.perf_counter() - t1
        return x, y

    def loader(p):
        tx, ty = load_split(p, "train")
        vx, vy = load_split(p, "valid")
        if jobs and not futs and (p, "valid") == jobs[-1]:
            drain()
        return tx, ty, vx, vy
    loader.stats = st
    loader.prefetch = prefetch
    return loader


class _Null(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
