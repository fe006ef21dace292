"""Per-config checkpoints in the reference's CTQ layout.

``{models_root}/{i}_{mst_2_str(mst)}`` — raw little-endian float32 weight blob
in layer order (byte-compatible with ``serialize_nd_weights``,
``cerebro_gpdb/madlib_keras_wrapper.py:119-131``; key ``ctq.py:319-337``),
plus two sidecars:

* ``….opt``  — Adam m, v (float32) and the step count, so a resumed run
  continues with the same optimizer state (the reference resets Adam every
  sub-epoch; ``--hop_optimizer_state false`` reproduces that instead),
* ``….json`` — metadata (epoch, partitions visited, model key, layout hash).

Writes happen on a background thread from host copies, never on the
training critical path.  Job/model logs are written as ``models_info.pkl`` /
``jobs_info.pkl`` (plain dicts) + JSON twins (``ctq.py:264-278``).
"""

import json
import os
import pickle
import queue
import threading

import numpy as np
import torch

from ..utils.keys import model_key


def ckpt_path(models_root, index, mst):
    return os.path.join(models_root, model_key(index, mst))


def layout_signature(layout):
    return [[s.name, list(s.shape)] for s in layout.specs]


def state_to_host(layout, state_row):
    """Split one state row into (weights blob, opt dict) on the host."""
    row = state_row.detach().to("cpu", non_blocking=False)
    weights = torch.cat([row[s.offset:s.offset + s.numel] for s in layout.specs]).numpy()
    m = torch.cat([row[layout.off_m + s.offset: layout.off_m + s.offset + s.numel]
                   for s in layout.train_specs]).numpy()
    v = torch.cat([row[layout.off_v + s.offset: layout.off_v + s.offset + s.numel]
                   for s in layout.train_specs]).numpy()
    step = float(row[layout.off_step])
    return weights.astype(np.float32), {"m": m.astype(np.float32), "v": v.astype(np.float32),
                                        "step": step}


def host_to_state(layout, weights, opt, state_row):
    out = torch.zeros(state_row.shape[0], dtype=torch.float32)
    off = 0
    for s in layout.specs:
        out[s.offset:s.offset + s.numel] = torch.from_numpy(weights[off:off + s.numel])
        off += s.numel
    if opt is not None:
        off = 0
        for s in layout.train_specs:
            out[layout.off_m + s.offset: layout.off_m + s.offset + s.numel] = \
                torch.from_numpy(opt["m"][off:off + s.numel])
            out[layout.off_v + s.offset: layout.off_v + s.offset + s.numel] = \
                torch.from_numpy(opt["v"][off:off + s.numel])
            off += s.numel
        out[layout.off_step] = float(opt["step"])
    state_row.copy_(out.to(state_row.device))


def write_checkpoint(path, layout, weights, opt, meta):
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(weights.astype("<f4").tobytes())
    os.replace(tmp, path)
    if opt is not None:
        with open(path + ".opt", "wb") as f:
            np.savez(f, m=opt["m"], v=opt["v"], step=np.array([opt["step"]], np.float64))
    meta = dict(meta)
    meta["layout"] = layout_signature(layout)
    with open(path + ".json", "w") as f:
        json.dump(meta, f)


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
