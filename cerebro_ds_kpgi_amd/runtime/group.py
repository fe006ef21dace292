"""Pack groups: the per-GPU execution unit of the MOP runtime.

All configurations with the same (architecture, batch size) form a pack
group.  On every GPU a group owns

* a *home* arena with one state row per member config (where a config's
  state parks between rounds and from where it is shipped on a hop), and
* a *working* arena holding the G configs that train on this GPU in the
  current round, packed into ONE horizontally-fused model: every kernel
  launch trains all G at once, each on its own data partition.

A training step (gather -> forward -> fused loss -> backward -> fused Adam)
has static shapes and device-side cursors, so after a few eager steps it is
captured once in a HIP graph and replayed for the rest of the run.
(Reference equivalents: the per-sub-epoch ``train_fn`` / ``fit_step_ctq``
jobs, ``run_cerebro_standalone_helper.py:270-289``, ``ctq.py:110-121``.)
"""

import os
import time

import torch

from ..data.store import gather_batch, input_buffers
from ..models import create_model_from_mst
from ..ops.loss import eval_metrics, softmax_ce
from ..ops import streams
from ..ops.backend import get_backend, take_fallbacks
from ..ops.optim import optimizer_step
from ..utils.logging import log_once
from .arena import Arena


class PackGroup(object):
    def __init__(self, key, model_ids, msts, store, device, compute_dtype, seed_base,
                 use_graphs=True, l2=True, warmup_eager=3, init=True):
        self.key = key
        self.arch, self.batch_size = key[0], key[1]
        self.optimizer = key[2] if len(key) > 2 else "adam"
        self.model_ids = list(model_ids)
        self.home_row = {m: i for i, m in enumerate(self.model_ids)}
        self.msts = msts
        self.store = store
        self.device = torch.device(device)
        self.dtype = compute_dtype
        # HIP graphs only over our HIP kernels.  A hipMemsetAsync captured
        # into a HIP graph does not re-execute correctly from the second
        # replay on (ROCm 7.x, scripts/debug/graph_memset_repro.py); our
        # kernels therefore never memset on a launch path (csrc/hip/common.h
        # cer_zero_async), but MIOpen's convolutions do, so the PyTorch
        # oracle backend always runs eagerly
        self.use_graphs = (use_graphs and self.device.type == "cuda" and
                           get_backend() == "hip")
        self.l2 = l2
        self.warmup_eager = warmup_eager
        # concurrency lane (engine._build_groups): groups of one batch on
        # different lanes replay on different streams at the same time
        self.lane = 0
        proto = create_model_from_mst({"model": self.arch})
        self.layout = proto.layout
        self.home = Arena(self.layout, len(self.model_ids), device, compute_dtype, trainable=False)
        if init:
            for m in self.model_ids:
                self.home.init_model(self.home_row[m], seed_base + m)
        self._work = {}   # G -> _Working
        self.current = None
        # asynchronous runtime: models whose latest state sits in a working
        # arena row ({G: {model: row}}), and the subset not yet parked in
        # their home rows.  A job that stays on this GPU then costs a
        # part_of_row change, not a state copy in and out.
        self.resident = {}
        self.dirty = set()
        self.n_loads = 0      # state copies home -> working row
        self.n_parks = 0      # state copies working row -> home

    def add_models(self, model_ids, seed):
        """Grow the home arena for configs proposed mid-run (hyperopt)."""
        new = [m for m in model_ids if m not in self.home_row]
        if not new:
            return
        self.park_all()
        old = self.home
        self.model_ids.extend(new)
        self.home_row = {m: i for i, m in enumerate(self.model_ids)}
        self.home = Arena(self.layout, len(self.model_ids), self.device, self.dtype,
                          trainable=False)
        self.home.state[:old.G].copy_(old.state)
        for m in new:
            self.home.init_model(self.home_row[m], seed * 100 + m)
        del old

    # ------------------------------------------------------------------
    def state_row(self, m):
        self.park(m)
        return self.home.state[self.home_row[m]]

    # -- residency (asynchronous runtime) -----------------------------------
    def _where(self, m):
        for G, rows in self.resident.items():
            if m in rows:
                return G, rows[m]
        return None

    def park(self, m):
        """Copy m's working-row state to its home row if only the row has it."""
        if m not in self.dirty:
            return
        G, row = self._where(m)
        self.home.state[self.home_row[m]].copy_(self._work[G].arena.state[row])
        self.dirty.discard(m)
        self.n_parks += 1

    def park_all(self):
        for m in list(self.dirty):
            self.park(m)

    def invalidate(self, m):
        """m's home row was just overwritten by an arriving hop."""
        assert m not in self.dirty, m
        for rows in self.resident.values():
            rows.pop(m, None)

    def drop_residency(self, models):
        """Working copies of ``models`` are no longer valid (failed job)."""
        for m in models:
            self.dirty.discard(m)
            for rows in self.resident.values():
                rows.pop(m, None)

    def begin_batch(self, jobs):
        """Working set for jobs = [(model, local_partition)]: models already
        resident in this working set keep their rows (only part_of_row
        changes), other rows load from the home arena after their previous
        residents are parked.  The batch's models are dirty afterwards."""
        G = len(jobs)
        w = self.working(G)
        batch = {m for m, _ in jobs}
        for G2, rows2 in self.resident.items():
            if G2 != G:
                for m in [m for m in rows2 if m in batch]:
                    self.park(m)
                    del rows2[m]
        res = self.resident.setdefault(G, {})
        rows = [None] * G
        rest = []
        for m, lp in jobs:
            r = res.get(m)
            if r is not None and rows[r] is None:
                rows[r] = (m, lp)
            else:
                rest.append((m, lp))
        for m2 in [m2 for m2 in res if m2 not in batch]:
            self.park(m2)
            del res[m2]
        free = [i for i in range(G) if rows[i] is None]
        for (m, lp), i in zip(rest, free):
            rows[i] = (m, lp)
        w.assign(rows)
        for i, (m, _) in enumerate(rows):
            if res.get(m) != i:
                w.load_local(i, m)
        self.resident[G] = {m: i for i, (m, _) in enumerate(rows)}
        self.dirty |= batch
        self.current = w
        return w

    def working(self, G):
        w = self._work.get(G)
        if w is None:
            w = _Working(self, G)
            self._work[G] = w
        return w

    def begin_round(self, jobs, recv_into=None):
        """jobs: list of (model_id, local_partition_index).  Returns the
        working set; rows whose state arrives by a hop are filled by the
        caller through ``recv_buffer``.  (Lock-step runtime: states are
        copied in here and parked back by ``end_round``.)"""
        self.park_all()
        self.resident.clear()
        G = len(jobs)
        w = self.working(G)
        w.assign(jobs)
        self.current = w
        return w

    def end_round(self, hop_optimizer_state=True):
        """Park the trained states back in the home arena."""
        w = self.current
        for row, (m, _) in enumerate(w.jobs):
            self.home.state[self.home_row[m]].copy_(w.arena.state[row])
        self.n_parks += len(w.jobs)
        self.current = None


# Packs of at most this many configs keep an HL image of their weights
# (Arena.whl): the optimizer writes it (+4 B per param and step) and the
# uniform-K GEMMs read it instead of splitting the weights.  Measured
# (profiles/r6_uk.md, same box): one config +1.0 %, eight configs -0.8 % (the
# extra optimizer traffic outweighs the split it saves in wide packs).
# CER_WHL_MAX_G overrides (0 = off).
WHL_MAX_G = int(os.environ.get("CER_WHL_MAX_G", "2"))


class _Working(object):
    def __init__(self, group, G):
        self.group = group
        self.G = G
        g = group
        self.arena = Arena(g.layout, G, g.device, g.dtype, trainable=True)
        self.arena.grad_clean = True      # the optimizer clears the gradient it consumes
        if (g.device.type == "cuda" and get_backend() == "hip" and g.dtype == torch.float32
                and G <= WHL_MAX_G):
            self.arena.enable_whl()       # HL weight image for the conv GEMMs
        self.net = create_model_from_mst({"model": g.arch})
        self.net.bind(self.arena)
        B = g.batch_size
        self.x, self.y = input_buffers(g.store, G, B, g.dtype)
        self.part_of_row = torch.zeros(G, dtype=torch.int32, device=g.device)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=g.device)
        self.acc = torch.zeros(G, 4, dtype=torch.float32, device=g.device)
        self.unit_grad = torch.ones(G, dtype=torch.float32, device=g.device)
        self.vx, self.vy = input_buffers(g.store, G, B, g.dtype)
        self.vcursor = torch.zeros(1, dtype=torch.int32, device=g.device)
        self.vacc = torch.zeros(G, 4, dtype=torch.float32, device=g.device)
        self.graph = None
        self.vgraph = None        # validation step graph
        self.veager = False       # validation step not capture safe
        self.eager_only = not getattr(self.net, "graph_safe", True)
        self.eager_steps = 0
        self.jobs = []
        # called between backward and the optimizer (DDP gradient all-reduce)
        self.grad_hook = None
        # zeroed buffers for the conv epilogues' atomic BN partials, zeroed
        # once per step (ops._hip._StatsArena)
        self.stats_arena = None
        if g.device.type == "cuda" and get_backend() == "hip":
            from ..ops import _hip
            self.stats_arena = _hip.new_stats_arena(g.device)

    def assign(self, jobs):
        self.jobs = list(jobs)
        parts = torch.tensor([p for _, p in jobs], dtype=torch.int32)
        self.part_of_row.copy_(parts)
        for row, (m, _) in enumerate(jobs):
            mst = self.group.msts[m]
            self.arena.set_hparams(row, mst["learning_rate"], mst["lambda_value"])

    def recv_buffer(self, row, with_optimizer=True):
        st = self.arena.state[row]
        return st if with_optimizer else st[:self.group.layout.n_master]

    def load_local(self, row, m):
        self.arena.state[row].copy_(self.group.state_row(m))
        self.group.n_loads += 1

    def prepare(self, hop_optimizer_state):
        if not hop_optimizer_state:
            self.arena.reset_optimizer()
        self.arena.sync_work()
        self.cursor.zero_()
        self.acc.zero_()
        self.vacc.zero_()

    # ------------------------------------------------------------------
    def _set_lane(self):
        if self.stats_arena is not None:
            from ..ops import _hip
            _hip.set_lane(self.group.lane)

    def replay_ready(self, valid=False):
        """True when the next train (``valid``: validation) steps are pure
        graph replays: no host-side op runs, so they may go to a lane stream
        beside another group's (async_mop._run_batch)."""
        if not self.group.use_graphs or self.eager_only:
            return False
        if valid:
            return self.vgraph is not None and not self.veager and _VALID_GRAPH
        return self.graph is not None and isinstance(self.graph, torch.cuda.CUDAGraph)

    def _step(self):
        self._set_lane()
        if self.stats_arena is None:
            return self._step_body()
        from ..ops import _hip
        _hip.stats_step(self.stats_arena)
        try:
            return self._step_body()
        finally:
            _hip.stats_step(None)

    def _step_body(self):
        g = self.group
        gather_batch(g.store, True, self.part_of_row, self.cursor, g.batch_size, self.x, self.y)
        # weight gradients are queued during backward and launched as a few
        # multi-layer kernels when the block exits (ops.streams); with >=
        # _SIDE_MIN_G packed configs the first half of them runs on the side
        # stream during the rest of backward -- not under a gradient
        # all-reduce hook (DDP): its buckets start mid-backward and must see
        # final gradients, which a side batch still writing would break
        wide = self.G >= _SIDE_MIN_G and self.G * g.batch_size >= _SIDE_MIN_IMAGES
        frac = (_SIDE_FRAC if wide and self.grad_hook is None
                and getattr(self.net, "grad_buckets", None) is None else 0.0)
        if self.x.device.type == "cuda" and get_backend() == "hip":
            streams.set_batch_rows(_WIDE_ROWS if wide else 0)
        with streams.deferred_wgrad(self.x.device.type == "cuda", side_frac=frac, key=id(self)):
            logits = self.net.forward(self.x, True)
            # a unit gradient seed (no loss reduction / fill kernels), and the
            # head's bias gradient out of the loss kernel (ops.loss)
            loss = softmax_ce(logits, self.y, self.acc, self.G,
                              head=getattr(logits, "_cer_head", None), unit=True)
            if loss.is_cuda:
                torch.autograd.backward(loss, self.unit_grad)
            else:               # (measured slower on the CPU autograd path)
                loss.sum().backward()
        streams.join()
        if self.grad_hook is not None:
            self.grad_hook(self.arena)
        # the optimizer launch also advances the cursor and zeroes the BN
        # statistics arena for the next step (ops.optim._aux)
        zero = self.stats_arena.buf if self.stats_arena is not None else None
        if not optimizer_step(self.arena, g.optimizer, l2=g.l2, cursor=self.cursor, zero=zero):
            self.cursor.add_(1)

    def train_steps(self, nsteps):
        done = 0
        streams.join()
        if not self.group.use_graphs or self.eager_only:
            for _ in range(nsteps):
                self._step()
            return nsteps
        if self.graph is None:
            # eager warm-up on a side stream (real steps), then capture once
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            take_fallbacks()
            with torch.cuda.stream(s):
                while self.eager_steps < self.group.warmup_eager and done < nsteps:
                    self._step()
                    self.eager_steps += 1
                    done += 1
            torch.cuda.current_stream().wait_stream(s)
            fb = take_fallbacks()
            if fb:
                # a step with PyTorch-path convs / pools is not capture safe:
                # this working set stays eager (ops.backend.hip_gate)
                self.eager_only = True
                log_once("{} G={}: ops {} have no HIP kernel for these shapes; "
                         "running eagerly (no HIP graph)".format(self.group.arch, self.G,
                                                                 sorted(fb)))
                while done < nsteps:
                    self._step()
                    done += 1
                return done
            if done >= nsteps:
                return done
            streams.join()
            gb = getattr(self.net, "grad_buckets", None)
            if gb is not None:
                # DDP: graph segments cut at the bucket boundaries, the
                # all-reduces run between their replays (baselines.GradBuckets)
                self.graph = self._capture_segmented(gb)
            else:
                self.graph = torch.cuda.CUDAGraph()
                # thread-local capture: the asynchronous runtime's hop thread
                # keeps issuing RCCL transfers / stream syncs while this
                # thread captures
                with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                    self._step()
        gb = getattr(self.net, "grad_buckets", None)
        while done < nsteps:
            if gb is not None and not isinstance(self.graph, torch.cuda.CUDAGraph):
                self.graph.replay(gb.run_action)
            else:
                self.graph.replay()
            done += 1
        return done

    def _capture_segmented(self, gb):
        from .baselines import SegmentedGraph
        sg = SegmentedGraph()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            sg.begin()
            gb.seg = sg
            try:
                self._step()
            finally:
                gb.seg = None
            sg.end()
        torch.cuda.current_stream().wait_stream(s)
        return sg

    def _vstep(self):
        self._set_lane()
        g = self.group
        gather_batch(g.store, False, self.part_of_row, self.vcursor, g.batch_size,
                     self.vx, self.vy)
        logits = self.net.forward(self.vx, False)
        eval_metrics(logits, self.vy, self.vacc, self.G)
        self.vcursor.add_(1)

    def validate(self, nsteps):
        """Forward-only passes over this round's validation rows.  Like the
        training step, the validation step is captured once in a HIP graph
        (after one eager step: kernel-variant tuning for the eval-path shapes)
        and replayed; the device-side cursor advances inside the graph."""
        self.vcursor.zero_()
        done = 0
        with torch.no_grad():
            if not self.group.use_graphs or self.eager_only or not _VALID_GRAPH:
                for _ in range(nsteps):
                    self._vstep()
                return
            if self.vgraph is None and nsteps > 0:
                take_fallbacks()
                self._vstep()
                done += 1
                if take_fallbacks():
                    self.veager = True
                if done < nsteps and not self.veager:
                    self.vgraph = torch.cuda.CUDAGraph()
                    # own memory pool (sharing the training graph's pool let the
                    # two graphs' temporaries alias: invalid eval results)
                    with torch.cuda.graph(self.vgraph,
                                          capture_error_mode="thread_local"):
                        self._vstep()
            while done < nsteps:
                if self.vgraph is not None and not self.veager:
                    self.vgraph.replay()
                else:
                    self._vstep()
                done += 1

    def read_metrics(self):
        """(train, valid) per row: dict(loss, top1, top5, n) — one host sync.

        Also the per-row non-finite guard: our ReLU epilogues (fmaxf) map NaN
        to 0, so a NaN weight can hide behind finite losses; a row whose
        state holds a non-finite value reports NaN losses (``finite`` False)
        and the run log says so, instead of training on silently."""
        # NaN / Inf propagate through a sum: reduce each row's weights + BN
        # statistics (a non-finite Adam moment reaches them within a step) in
        # two stages — [G * 64, n / 64] rows first; torch's one-stage
        # reduction of a [G, 30 M] tensor has only G outputs and took 17 ms
        G, nm = self.G, self.group.layout.n_master
        part = self.arena.state[:, :nm].reshape(G, 64, nm // 64).sum(dim=2)
        fin = torch.isfinite(part.sum(dim=1))
        both = torch.stack([self.acc, self.vacc]).cpu()
        fin = fin.cpu().tolist()
        out = []
        for row in range(self.G):
            rec = {"finite": bool(fin[row])}
            for name, a in (("train", both[0, row]), ("valid", both[1, row])):
                n = max(float(a[3]), 1.0)
                rec[name] = {"loss": float(a[0]) / n if fin[row] else float("nan"),
                             "top1": float(a[1]) / n, "top5": float(a[2]) / n, "n": int(a[3])}
            if not fin[row]:
                log_once("non-finite model state in {} row {} (config {})".format(
                    self.group.arch, row, self.jobs[row][0] if row < len(self.jobs) else "?"))
            out.append(rec)
        return out


# Side-stream share of the batched weight gradients (ops.streams
# deferred_wgrad side_frac) for packs of at least _SIDE_MIN_G configs
# (measured: +2 % at 8, +1 % at 4, -3 % at 1 config; r2_ab_wgrad_chunk.md;
# 0.4 re-measured 0.5 % faster than 0.5 on the round-3 build,
# profiles/r3_final.md; on the round-4 build +1.3 % at 2 configs and
# -0.6 % at 1, so packs of >= 2 take it, profiles/r4_final.md)
_SIDE_FRAC = float(os.environ.get("CER_WGB_SIDE_FRAC", "0.4"))
_SIDE_MIN_G = int(os.environ.get("CER_WGB_SIDE_MIN_G", "2"))
# ... and at least this many images per step (G x batch): small launch-bound
# packs (NASNet-Mobile bs4 in the hetero drill-down) keep the serial batch
_SIDE_MIN_IMAGES = int(os.environ.get("CER_WGB_SIDE_MIN_IMAGES", "64"))
# wgrad-batch rows per split for those packs (fewer, longer splits: +1 % at
# 8 configs; one-config packs keep 1024, where 2048 is 1-2.5 % slower)
_WIDE_ROWS = int(os.environ.get("CER_WGB_ROWS_WIDE", "2048"))

# Graph-captured validation (CER_VALID_GRAPH=0 runs it eagerly).  Its round-1
# failures (invalid eval losses after an epoch boundary) had the same root
# cause as the training-graph corruption: captured hipMemsetAsync nodes.
_VALID_GRAPH = os.environ.get("CER_VALID_GRAPH", "1") == "1"


def now():
    return time.time()
