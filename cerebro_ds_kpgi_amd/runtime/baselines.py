"""Comparison baselines on the same runtime.

* ``MAEngine`` — model averaging, the reference's in-DB MA approach
  (``madlib_keras_fit``; ``cerebro_gpdb/run_imagenet.py:46-108``, merge format
  ``madlib_keras_wrapper.py:37-116``): every epoch each GPU trains every
  config on its local partition starting from the same weights, then the
  weights (and BN statistics) are averaged weighted by image count — an
  RCCL all-reduce of ``count * w`` and ``count``.  The optimizer is rebuilt
  every epoch, as a MADlib fit transition does.
* ``DDPEngine`` — synchronous data parallel per config (the reference's
  PyTorch DDP baseline, ``cerebro_gpdb/run_pytorchddp.py:204-519``): each
  step every GPU computes gradients on its own partition's batch; the flat
  gradient arena is all-reduced in buckets *during* backward
  (``GradBuckets``: the models place bucket marks between blocks; when the
  gradient flows past a mark, the queued weight-gradient kernels of the
  layers above are flushed and their contiguous arena range is all-reduced
  asynchronously by RCCL while the layers below run backward), and the fused
  Adam step waits for the last bucket.  BatchNorm statistics stay per rank,
  as in the reference (torch DDP without SyncBatchNorm).  Per-rank batch =
  the MST's batch size (reference default; ``--pytorchddp_sanity`` divides
  it by the world size).
* Task parallelism (Hyperopt-Spark, D6) is ``MOPEngine`` with
  ``scheduler="task"``: data replicated on every GPU, whole models per GPU.

All three reuse the pack groups (packed configs, HIP kernels, HIP graphs;
the DDP step is captured as graph segments cut at the bucket boundaries, the
all-reduces run between segment replays -- ``SegmentedGraph``).
"""

import collections
import time

import torch
import torch.distributed as dist

from ..data.store import PartitionStore
from ..models import dataset_of, pack_key
from ..utils.keys import model_key
from .engine import default_sizes
from .group import PackGroup


class _GroupEngine(object):
    """Shared setup: one local partition per GPU, every config on every GPU."""

    mode = "base"

    def __init__(self, msts, ctx, opts):
        self.msts = [dict(m) for m in msts]
        self.ctx = ctx
        self.o = opts
        self.device = ctx.device
        self.dataset = opts.dataset or dataset_of(self.msts[0]["model"])
        self.P = ctx.world
        self.my_parts = [ctx.rank]
        n_tr, n_va = default_sizes(self.dataset, self.P)
        self.n_train = opts.n_train or n_tr
        self.n_valid = opts.n_valid or n_va
        self.dtype = torch.bfloat16 if opts.compute_dtype == "bf16" else torch.float32
        self.store = PartitionStore(self.dataset, self.my_parts, self.n_train, self.n_valid,
                                    self.device, seed=opts.seed, loader=opts.store_loader)
        by_key = collections.defaultdict(list)
        for m in range(len(self.msts)):
            by_key[pack_key(self.msts[m])].append(m)
        self.groups = {k: PackGroup(k, ms, self.msts, self.store, self.device, self.dtype,
                                    seed_base=opts.seed * 100, use_graphs=opts.use_graphs,
                                    l2=opts.l2)
                       for k, ms in by_key.items()}
        self.mst_state = {m: {"train_loss": [], "valid_loss": [], "train_top5_error": [],
                              "valid_top5_error": [], "state": "RUNNING"}
                          for m in range(len(self.msts))}
        self.jobs_info = {}
        self.train_images = 0

    def _record(self, epoch, per_model):
        for m, rec in per_model.items():
            st = self.mst_state[m]
            st["train_loss"].append(rec["train"]["loss"])
            st["valid_loss"].append(rec["valid"]["loss"])
            st["train_top5_error"].append(1 - rec["train"]["top5"])
            st["valid_top5_error"].append(1 - rec["valid"]["top5"])
            self.jobs_info.setdefault(epoch, {})[(model_key(m, self.msts[m]), "ALL")] = rec

    def _gather_metrics(self, w):
        """Average the per-rank metrics (weighted by sample counts)."""
        mets = w.read_metrics()
        allm = self.ctx.all_gather_object(mets)
        out = []
        for row in range(w.G):
            rec = {}
            for ph in ("train", "valid"):
                n = sum(r[row][ph]["n"] for r in allm) or 1
                rec[ph] = {k: sum(r[row][ph][k] * r[row][ph]["n"] for r in allm) / n
                           for k in ("loss", "top1", "top5")}
                rec[ph]["n"] = n
            out.append(rec)
        return out

    def close(self):
        pass


class MAEngine(_GroupEngine):
    mode = "ma"

    def run(self, num_epochs):
        t0 = time.time()
        for epoch in range(1, num_epochs + 1):
            self.store.new_epoch(epoch)
            per_model = {}
            for key, grp in self.groups.items():
                jobs = [(m, 0) for m in grp.model_ids]
                w = grp.begin_round(jobs)
                for row, (m, _) in enumerate(jobs):
                    w.load_local(row, m)
                w.prepare(hop_optimizer_state=False)      # fresh optimizer per fit iteration
                B = grp.batch_size
                steps = self.n_train // B
                w.train_steps(steps)
                self.train_images += steps * B * w.G
                w.validate(max(1, self.n_valid // B))
                mets = self._gather_metrics(w)
                self._average(w, steps * B)
                grp.end_round()
                for row, (m, _) in enumerate(jobs):
                    per_model[m] = mets[row]
            self._record(epoch, per_model)
        return time.time() - t0

    def _average(self, w, count):
        """w <- sum_r count_r * w_r / sum_r count_r over ranks (params + BN
        stats): the reference's count-weighted merge (``madlib_keras_wrapper.py:
        63-116``, the image count travels with the weights as in
        ``serialize_state_with_nd_weights``) as ONE RCCL all-reduce per merge:
        every config row's ``count * w`` and the count packed into one
        contiguous buffer (the master section of the arena is a strided
        ``[G, n]`` view, which collectives reject)."""
        if not self.ctx.initialized:
            return
        master = w.arena.master
        if getattr(self, "keep_pre_average", False):
            self.pre_average = master.detach().clone()
        G, n = master.shape
        buf = torch.empty(G * n + 1, device=master.device, dtype=torch.float32)
        body = buf[:G * n].view(G, n)
        body.copy_(master)
        body.mul_(float(count))
        buf[G * n] = float(count)
        dist.all_reduce(buf)
        self.n_collectives = getattr(self, "n_collectives", 0) + 1
        body.div_(buf[G * n])
        master.copy_(body)
        w.arena.sync_work()


class GradBuckets(object):
    """Bucketed gradient all-reduce overlapped with backward (DDP).

    ``ready_from(lo)`` (called from a model's bucket mark in backward): the
    gradients of arena columns ``[lo, hi)`` are final — flush the queued
    weight-gradient kernels, then, once at least ``bucket_bytes`` are pending
    (per config row), start an asynchronous all-reduce of each config row's
    ``[lo, hi)`` slice.  RCCL's stream waits for everything issued so far on
    the compute stream and runs beside the remaining backward.  ``finish()``
    (before the optimizer) reduces the rest, makes the compute stream wait
    for every bucket and averages.  Bucket sizes are per-link sized: ring
    all-reduce over xGMI is bound by one link (~50 GB/s per direction), so
    25-64 MB buckets keep ~1 ms transfers in flight behind the backward.

    HIP graphs (``capture``): the step is captured as a chain of graph
    SEGMENTS cut at every bucket boundary; the all-reduces stay outside the
    graphs (launched from the host between two segment replays, so they
    still overlap the next segment's backward) -- no collective is captured.
    ``replay()`` runs segment, collective action, segment, ..."""

    def __init__(self, arena, world, bucket_bytes=32 << 20, group=None):
        self.arena = arena
        self.world = world
        self.bucket_cols = max(1, bucket_bytes // 4)
        self.group = group
        self.hi = arena.layout.n_train
        self.works = []
        self.pending = []              # (lo, hi, staging view) awaiting copy-back
        self.stage = None              # contiguous staging: one slice per bucket
        self.stage_off = 0
        self.n_buckets = 0
        self.n_collectives = 0
        self.bucket_log = []           # (lo, hi) per bucket of the last step
        self.seg = None                # SegmentedGraph while capturing

    def _allreduce(self, lo, hi):
        """ONE all-reduce per bucket over all G config rows: the bucket's
        columns of every row (a strided [G, hi-lo] view) are packed into a
        contiguous slice of the staging buffer, reduced, and copied back
        (divided by the world size) in ``_wait``."""
        g = self.arena.grad
        G, n = g.shape[0], hi - lo
        if self.stage is None:
            self.stage = torch.empty(G * self.arena.layout.n_train, device=g.device,
                                     dtype=g.dtype)
        buf = self.stage[self.stage_off:self.stage_off + G * n].view(G, n)
        self.stage_off += G * n
        buf.copy_(g[:, lo:hi])
        self.works.append(dist.all_reduce(buf, group=self.group, async_op=True))
        self.pending.append((lo, hi, buf))
        self.n_collectives += 1

    def _wait(self):
        for w in self.works:
            w.wait()
        g = self.arena.grad
        for lo, hi, buf in self.pending:
            buf.mul_(1.0 / self.world)
            g[:, lo:hi].copy_(buf)
        self.works, self.pending, self.stage_off = [], [], 0

    def ready_from(self, lo, force=False):
        if lo >= self.hi or (not force and self.hi - lo < self.bucket_cols):
            return
        from ..ops import streams
        streams.flush_wgrad()
        # the all-reduce runs on RCCL's stream, which orders only after the
        # CURRENT stream: any side-stream weight-gradient work must be joined
        # first (group.py keeps DDP steps off the side batch; this is the guard)
        streams.join_side()
        if self.seg is not None:
            self.seg.cut(("ar", lo, self.hi))
        else:
            self._allreduce(lo, self.hi)
        self.bucket_log.append((lo, self.hi))
        self.n_buckets += 1
        self.hi = lo

    def finish(self, arena=None):
        self.ready_from(0, force=True)
        if self.seg is not None:
            self.seg.cut(("wait",))
        else:
            self._wait()
        self.hi = self.arena.layout.n_train

    def run_action(self, act):
        if act[0] == "ar":
            self._allreduce(act[1], act[2])
        else:
            self._wait()

    def reset_log(self):
        self.bucket_log = []


class SegmentedGraph(object):
    """A step captured as several HIP graphs with host actions between them
    (``cut(action)`` ends the current segment and opens the next one, sharing
    one memory pool; ``replay(run_action)`` replays them in order).  Used for
    the DDP step: collectives stay outside every graph."""

    def __init__(self):
        self.segs = []
        self.actions = []
        self._cur = None

    def begin(self):
        self._open()

    def _open(self):
        g = torch.cuda.CUDAGraph()
        pool = self.segs[0].pool() if self.segs else None
        g.capture_begin(pool=pool, capture_error_mode="relaxed")
        self._cur = g

    def cut(self, action):
        self._cur.capture_end()
        self.segs.append(self._cur)
        self.actions.append(action)
        self._open()

    def end(self):
        self._cur.capture_end()
        self.segs.append(self._cur)
        self.actions.append(None)
        self._cur = None

    def replay(self, run_action):
        for g, act in zip(self.segs, self.actions):
            g.replay()
            if act is not None:
                run_action(act)


class DDPEngine(_GroupEngine):
    mode = "ddp"

    def run(self, num_epochs):
        t0 = time.time()
        world = self.ctx.world
        for epoch in range(1, num_epochs + 1):
            self.store.new_epoch(epoch)
            per_model = {}
            for key, grp in self.groups.items():
                jobs = [(m, 0) for m in grp.model_ids]
                w = grp.begin_round(jobs)
                for row, (m, _) in enumerate(jobs):
                    w.load_local(row, m)
                w.prepare(hop_optimizer_state=True)
                if self.ctx.initialized and world > 1:
                    gb = GradBuckets(w.arena, world,
                                     int(float(getattr(self.o, "ddp_bucket_mb", 32)) * (1 << 20)))
                    w.net.grad_buckets = gb
                    w.grad_hook = gb.finish
                B = grp.batch_size
                steps = self.n_train // B
                w.train_steps(steps)
                self.train_images += steps * B * w.G
                w.validate(max(1, self.n_valid // B))
                mets = self._gather_metrics(w)
                grp.end_round()
                for row, (m, _) in enumerate(jobs):
                    per_model[m] = mets[row]
            self._record(epoch, per_model)
        return time.time() - t0
