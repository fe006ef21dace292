"""Per-config checkpoints in the reference's CTQ layout.

``{models_root}/{i}_{mst_2_str(mst)}`` — raw little-endian float32 weight blob
in the Keras ``get_weights()`` layout of the architecture, i.e. what the
reference's ``serialize_nd_weights`` writes (``cerebro_gpdb/
madlib_keras_wrapper.py:119-131``; key ``ctq.py:319-337``; conversion in
``runtime.serialize.master_to_keras``), plus two sidecars:

* ``….opt``  — Adam m, v (float32, our storage order) and the step count, so
  a resumed run continues with the same optimizer state (the reference resets
  Adam every sub-epoch; ``--hop_optimizer_state false`` reproduces that),
* ``….json`` — metadata (epoch, partitions visited, model key, layout).

Consistency: every commit writes *versioned* files ``{key}@{version}``
(+ ``.opt`` / ``.json``); ``resume.json`` is republished (atomic rename)
after every rank's writes are on disk and names each config's committed
version, so a crash or full disk in the middle of a commit leaves the
previous restart point intact.  Only then are the canonical CTQ names
re-pointed (hard link, or copy) and superseded versions deleted.

Writes never block training: ``HostStager`` snapshots a state row with an
HBM-speed device copy on the compute stream and moves it to pinned host
memory on a side stream; the ``AsyncWriter`` thread waits for that copy's
event, converts and writes.  Job/model logs are written as
``models_info.pkl`` / ``jobs_info.pkl`` (plain dicts) + JSON twins
(``ctq.py:264-278``).
"""

import glob
import json
import os
import pickle
import queue
import shutil
import threading

import numpy as np
import torch

from ..utils.keys import model_key
from .serialize import blob_to_master, weights_blob


def ckpt_path(models_root, index, mst):
    return os.path.join(models_root, model_key(index, mst))


def versioned(path, version):
    return path if not version else "{}@{}".format(path, version)


def layout_signature(layout):
    return [[s.name, list(s.shape)] for s in layout.specs]


def split_state(layout, row):
    """One full state row (numpy float32) -> (Keras weights blob array, opt dict)."""
    weights = np.frombuffer(weights_blob(layout, row[:layout.n_master]), dtype=np.float32)
    m = np.concatenate([row[layout.off_m + s.offset: layout.off_m + s.offset + s.numel]
                        for s in layout.train_specs])
    v = np.concatenate([row[layout.off_v + s.offset: layout.off_v + s.offset + s.numel]
                        for s in layout.train_specs])
    return weights, {"m": m.astype(np.float32), "v": v.astype(np.float32),
                     "step": float(row[layout.off_step])}


def state_to_host(layout, state_row):
    """Synchronous variant of ``HostStager`` + ``split_state`` (tools, tests)."""
    return split_state(layout, state_row.detach().to("cpu").numpy())


def host_to_state(layout, weights, opt, state_row):
    out = np.zeros(state_row.shape[0], dtype=np.float32)
    out[:layout.n_master] = blob_to_master(layout, weights)
    if opt is not None:
        off = 0
        for s in layout.train_specs:
            out[layout.off_m + s.offset: layout.off_m + s.offset + s.numel] = \
                opt["m"][off:off + s.numel]
            out[layout.off_v + s.offset: layout.off_v + s.offset + s.numel] = \
                opt["v"][off:off + s.numel]
            off += s.numel
        out[layout.off_step] = float(opt["step"])
    state_row.copy_(torch.from_numpy(out).to(state_row.device))


class Staged(object):
    """A state row on its way to host memory."""
    __slots__ = ("host", "done", "release")

    def __init__(self, host, done, release):
        self.host, self.done, self.release = host, done, release

    def wait(self):
        if self.done is not None:
            self.done.synchronize()
        return self.host.numpy() if isinstance(self.host, torch.Tensor) else self.host

    def free(self):
        if self.release is not None:
            self.release()
            self.release = None


class HostStager(object):
    """Snapshot state rows for checkpoint writes off the training path.

    ``stage(row)`` enqueues a device copy of the row on the *current* stream
    (HBM speed: ~0.1 ms per ResNet-50 state row), then a D2H of that copy
    into pinned host memory on a side stream; training continues at once and
    may overwrite the row.  Buffers come from a pool keyed by length and go
    back after the writer thread is done with them."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.pool = {}
        self.lock = threading.Lock()
        self.staged_bytes = 0

    def _take(self, n):
        with self.lock:
            free = self.pool.setdefault(n, [])
            if free:
                return free.pop()
        return (torch.empty(n, dtype=torch.float32, device=self.device),
                torch.empty(n, dtype=torch.float32, pin_memory=True))

    def _give(self, n, bufs):
        with self.lock:
            self.pool[n].append(bufs)

    def stage(self, row):
        row = row.detach()
        self.staged_bytes += row.numel() * 4
        if not self.cuda:
            return Staged(row.to("cpu").clone().numpy(), None, None)
        n = row.numel()
        dev, host = self._take(n)
        dev.copy_(row)
        ready = torch.cuda.Event()
        ready.record()
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            host.copy_(dev, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.stream)
        return Staged(host, done, lambda: self._give(n, (dev, host)))

    def clear(self):
        with self.lock:
            self.pool.clear()


def write_checkpoint(path, layout, weights, opt, meta):
    """Write weights + sidecars under ``path`` (each file via tmp + rename)."""
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(np.asarray(weights, np.float32).astype("<f4").tobytes())
    os.replace(tmp, path)
    if opt is not None:
        with open(path + ".opt.tmp", "wb") as f:
            np.savez(f, m=opt["m"], v=opt["v"], step=np.array([opt["step"]], np.float64))
        os.replace(path + ".opt.tmp", path + ".opt")
    meta = dict(meta)
    meta["layout"] = layout_signature(layout)
    with open(path + ".json.tmp", "w") as f:
        json.dump(meta, f)
    os.replace(path + ".json.tmp", path + ".json")


def write_staged(path, layout, staged, meta, with_opt=True):
    """Writer-thread body: wait for the D2H, convert, write, recycle buffers."""
    try:
        weights, opt = split_state(layout, staged.wait())
    finally:
        staged.free()
    write_checkpoint(path, layout, weights, opt if with_opt else None, meta)


def read_checkpoint(path):
    weights = np.fromfile(path, dtype="<f4")
    opt = None
    if os.path.exists(path + ".opt"):
        with np.load(path + ".opt", allow_pickle=False) as z:
            opt = {"m": z["m"], "v": z["v"], "step": float(z["step"][0])}
    meta = None
    if os.path.exists(path + ".json"):
        with open(path + ".json") as f:
            meta = json.load(f)
    return weights, opt, meta


_SUFFIXES = ("", ".opt", ".json")


def _point(src, dst):
    """Make ``dst`` the same file as ``src`` (hard link; copy across devices)."""
    tmp = dst + ".lnk"
    if os.path.exists(tmp):
        os.remove(tmp)
    try:
        os.link(src, tmp)
    except OSError:
        shutil.copyfile(src, tmp)
    os.replace(tmp, dst)


def publish_version(path, version):
    """After ``resume.json`` names ``version``: re-point the canonical CTQ
    files at it and delete every other version of this config (superseded
    commits and writes of a commit that never completed)."""
    src = versioned(path, version)
    for suf in _SUFFIXES:
        if os.path.exists(src + suf):
            _point(src + suf, path + suf)
    for f in glob.glob(glob.escape(path) + "@*"):
        base = f
        for suf in (".opt", ".json", ".tmp"):
            if base.endswith(suf):
                base = base[:-len(suf)]
        if base != src:
            try:
                os.remove(f)
            except FileNotFoundError:
                pass


class AsyncWriter(object):
    """Background file writer; ``flush()`` waits for all queued writes."""

    def __init__(self):
        self.q = queue.Queue()
        self.err = None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                self.q.task_done()
                return
            try:
                item()
            except Exception as e:  # surfaced on flush
                self.err = e
            self.q.task_done()

    def submit(self, fn):
        self.q.put(fn)

    def flush(self):
        self.q.join()
        if self.err is not None:
            e, self.err = self.err, None
            raise e

    def close(self):
        self.flush()
        self.q.put(None)
        self.t.join()


def dump_infos(logs_root, models_info, jobs_info, suffix=""):
    os.makedirs(logs_root, exist_ok=True)
    with open(os.path.join(logs_root, "models_info{}.pkl".format(suffix)), "wb") as f:
        pickle.dump(dict(models_info), f)
    with open(os.path.join(logs_root, "jobs_info{}.pkl".format(suffix)), "wb") as f:
        pickle.dump(dict(jobs_info), f)
    with open(os.path.join(logs_root, "jobs_info{}.json".format(suffix)), "w") as f:
        json.dump({str(e): {"{}|{}".format(*k): v for k, v in d.items()}
                   for e, d in jobs_info.items()}, f, default=str)
