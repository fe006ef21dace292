"""The MOP runtime: S configurations hop over P = N x V HBM partitions.

One process per GPU.  Every rank runs the same (replicated, deterministic)
scheduler, so the round plan and the hop plan are known everywhere without a
coordinator round trip; only job results travel on the control plane.

Per round (= one sub-epoch on every partition):

1. plan: ``{partition: model}`` from the scheduler;
2. hop:  models whose holder GPU != their partition's GPU are shipped as one
   flat state row each by a single batched P2P group (RCCL over xGMI);
   models staying on the GPU are a local device copy;
3. train: every pack group trains its G configs packed, each on its own
   partition, for ``n_train // batch`` steps (HIP-graph replays), then
   validates on the partition's validation shard;
4. report: metrics gathered to all ranks; job dicts in the reference's CTQ
   format (``ctq.py:429-444``); invariants enforced by the scheduler.

Epoch end: per-config train/valid summaries, ``mst_eval_fn`` (grid stopper or
async TPE) and checkpoints in the CTQ layout.

Failure handling (the reference only re-raises,
``ctq.py:411-423``):

* a *recoverable* job failure (``SoftFault``, e.g. an unreadable partition)
  on one rank fails only that rank's (config, partition) pairs: the other
  ranks' results commit, the failed pairs roll back to their pre-round
  state (still parked in the previous holder's home row) and are re-run as
  a sub-round, up to ``max_retries`` times;
* a crash ends the job; with ``ckpt_every="subepoch"`` every round ends with
  a consistent checkpoint + ``resume.json`` and ``resume=True`` (``--resume``)
  continues from the next unfinished round of the interrupted epoch
  (epoch-level resume with ``ckpt_every="epoch"``);
* ``fault_inject="r:k[:soft|:exit]"`` raises (or soft-fails, or hard-exits)
  rank r at sub-epoch k — the tests' injection hook.
"""

import collections
import json
import math
import os
import time

import torch

from ..data.catalog import make_data_catalog, write_manifest
from ..data.store import PartitionStore
from ..models import dataset_of, pack_key
from ..parallel.hop import execute_moves, plan_moves, validate_plan
from ..scheduler import make_scheduler
from ..utils import safe_pickle
from ..utils.keys import model_key, mst_2_str
from ..utils.logging import logs
from ..utils.trace import Tracer
from .checkpoint import (AsyncWriter, HostStager, ckpt_path, dump_infos, host_to_state,
                         publish_version, read_checkpoint, versioned, write_staged)
from .group import PackGroup


class EngineOptions(object):
    def __init__(self, **kw):
        self.slots_per_gpu = kw.get("slots_per_gpu", 0)
        self.scheduler = kw.get("scheduler", "rotation")
        self.n_train = kw.get("n_train", 0)
        self.n_valid = kw.get("n_valid", 0)
        # fp32 = the reference precision (TF 1.14 / PyTorch 1.4 defaults); bf16 opt-in
        self.compute_dtype = kw.get("compute_dtype", "fp32")
        self.hop_optimizer_state = kw.get("hop_optimizer_state", True)
        self.l2 = kw.get("l2", True)
        self.use_graphs = kw.get("use_graphs", True)
        self.logs_root = kw.get("logs_root", "")
        self.models_root = kw.get("models_root", "")
        self.ckpt_every = kw.get("ckpt_every", "epoch")   # epoch | subepoch | none
        self.seed = kw.get("seed", 2018)
        self.shuffle = kw.get("shuffle", True)
        self.fault_inject = kw.get("fault_inject", "")
        self.verbose = kw.get("verbose", True)
        self.dataset = kw.get("dataset", None)
        self.store_loader = kw.get("store_loader", None)
        self.partitions = kw.get("partitions", 0)
        self.trace = kw.get("trace", False)
        # debug: verify every hop with sender/receiver digests (parallel.hop)
        self.hop_check = kw.get("hop_check", os.environ.get("CER_HOP_CHECK", "0") == "1")
        self.max_retries = kw.get("max_retries", 2)
        self.resume = kw.get("resume", False)
        self.heartbeat = kw.get("heartbeat", 0)     # watchdog timeout (s); 0 = off
        # a rank inside one sub-epoch job for longer than this is STALLED
        # (0 = off; needs the heartbeat)
        self.stall_timeout = kw.get("stall_timeout", 0)
        # runtime: "async" (event driven, hops overlapped with compute),
        # "lockstep" (a barrier per sub-epoch) or "auto" (async unless a
        # feature needs lock-step: sub-epoch checkpoints, task parallelism)
        self.runtime = kw.get("runtime", os.environ.get("CER_RUNTIME", "auto"))
        # pack-aware scheduling order (policies.py): co-schedule configs that
        # pack into one launch stream, most steps per visit first
        self.pack_order = kw.get("pack_order", True)
        # concurrency lanes (async_mop._Lanes); 1 = the groups of a batch run
        # one after another
        self.lanes = kw.get("lanes", LANES)
        self.ctrl_timeout = kw.get("ctrl_timeout", 6 * 3600)
        # test hook: extra seconds per job of config m (heterogeneous jobs)
        self.sim_job_seconds = kw.get("sim_job_seconds", None)
        self.sim_valid_seconds = kw.get("sim_valid_seconds", 0.0)
        self.sim_hop_seconds = kw.get("sim_hop_seconds", 0.0)     # per hop (slow link)
        # test hook: this rank's hop service wedges in its first group
        self.sim_hop_stall = kw.get("sim_hop_stall", None)
        # hop watchdog (parallel.health.HopWatch): an in-flight hop older
        # than this + 2 x the longest job ends every rank with a diagnostic
        # (0 = off)
        self.hop_timeout = kw.get("hop_timeout",
                                  float(os.environ.get("CER_HOP_TIMEOUT", "60")))
        # DDP baseline: gradient bucket size (MB per config row)
        self.ddp_bucket_mb = kw.get("ddp_bucket_mb", 32)


class _StepsPlan(object):
    """Steps per job of a bench session: ``per`` per round, ``last`` in the
    final one of ``n`` rounds (the coordinator passes the round index within
    the epoch; it tracks the session's round count itself)."""

    def __init__(self, per, last, n):
        self.per, self.last, self.n = per, last, n

    def __call__(self, session_round):
        return self.last if session_round == self.n - 1 else self.per


class SoftFault(RuntimeError):
    """A recoverable job failure: the failed pairs are requeued."""


RESUME_FILE = "resume.json"

# default concurrency lanes per rank (EngineOptions.lanes): pack groups of
# one batch (different architectures / batch sizes, e.g. the hetero
# drill-down or a TPE round) replay their step graphs on this many streams at
# once (async_mop._run_batch); each lane has its own split-K workspace (64 MB).
# Default 4 on one GPU: the 16-config Criteo grid (4 batch sizes = 4 pack
# groups of small, launch-bound MLP steps) runs 6.5 % faster with its groups
# concurrent than one after another (same-lease A/B of the round-4 and round-5
# builds, profiles/r6_r4_vs_r5.md; round 5 had set 1 after the lanes measured
# neutral on the hetero jobs).  At world > 1 ``effective_lanes`` clamps them
# to what leaves the hop's two streams within the hardware queues
# (stream_budget, profiles/r5_stream_budget.md).
LANES = 4
# hardware queues per process (HIP's default GPU_MAX_HW_QUEUES)
HW_QUEUES = 4


def default_sizes(dataset, P):
    from ..config import catalog as cat
    if dataset == "imagenet":
        return cat.IMAGENET_TRAIN_TOTAL // P, cat.IMAGENET_VALID_TOTAL // P
    if dataset == "criteo":
        tot = cat.CRITEO_TOTAL
        return int(tot * 0.9) // P, int(tot * 0.1) // P
    return 2048 // P, 512 // P


class MOPEngine(object):
    def __init__(self, msts, ctx, opts):
        self.msts = [dict(m) for m in msts]
        self.ctx = ctx
        self.o = opts
        self.device = ctx.device
        S = len(self.msts)
        self.dataset = opts.dataset or dataset_of(self.msts[0]["model"])
        self.task_parallel = opts.scheduler == "task"
        if self.task_parallel:
            # Hyperopt-Spark semantics: every GPU holds the WHOLE dataset (P
            # partitions replicated; the full ImageNet-112 uint8 fits in HBM)
            # and trains whole models; no hops.
            self.P = opts.partitions or 8
            self.V = self.P
            self.my_parts = list(range(self.P))
        else:
            V = opts.slots_per_gpu or max(1, S // ctx.world)
            self.V = V
            self.P = V * ctx.world
            self.my_parts = list(range(ctx.rank * V, (ctx.rank + 1) * V))
        n_tr, n_va = default_sizes(self.dataset, self.P)
        self.n_train = opts.n_train or n_tr
        self.n_valid = opts.n_valid or n_va
        self.dtype = torch.bfloat16 if opts.compute_dtype == "bf16" else torch.float32
        t0 = time.time()
        self.store = PartitionStore(self.dataset, self.my_parts, self.n_train, self.n_valid,
                                    self.device, seed=opts.seed, loader=opts.store_loader)
        self.data_load_time = time.time() - t0
        if opts.store_loader is not None:      # sizes come from the loaded partitions
            self.n_train, self.n_valid = self.store.n_train, self.store.n_valid
        self.groups = {}
        self.group_of = {}
        self._lanes = {}
        self.lane_batches = 0        # train / validation phases run on lane streams
        self._build_groups(range(S))
        self.holder = {m: None for m in range(S)}    # None = every rank has the init copy
        self.sched = make_scheduler(opts.scheduler, list(range(S)), list(range(self.P)),
                                    seed=opts.seed, shuffle=opts.shuffle)
        self.sched.pack_key_fn = self.pack_order_key()
        self.models_info = collections.defaultdict(list)
        self.jobs_info = {}
        self.mst_state = {m: {"train_loss": [], "valid_loss": [], "train_top5_error": [],
                              "valid_top5_error": [], "train_top1_error": [],
                              "valid_top1_error": [], "state": "RUNNING"} for m in range(S)}
        self.writer = AsyncWriter()
        self.stager = HostStager(self.device)
        self.hb = None               # parallel.health.Heartbeat (when enabled)
        self.ckpt_versions = {}      # config -> committed checkpoint version (rank 0)
        self.train_images = 0
        self.round_idx = 0
        self.hop_bytes = 0
        self.hop_time = 0.0          # exposed: time a rank waited for a hop
        self.hop_busy_time = 0.0     # transfers themselves (async runtime)
        self.hop_hold_time = 0.0     # coordinator hold of the hops this rank received
        self.hop_groups = 0          # batch_isend_irecv groups posted (async runtime)
        self.hop_spans = []
        self.coord_msts = None
        self._asched = {}
        self._chan = None
        self._nsession = 0
        self._hop_group = None
        self.hop_watch = None        # parallel.health.HopWatch while a run is armed
        if ctx.initialized and not self.task_parallel:
            # the hop data plane: one communicator, used only by the hop
            # service (async_mop.HopService / _hop_and_load), warmed here --
            # under the hop watchdog: the first point-to-point traffic of a
            # multi-GPU job happens here, and a wedged peer connection would
            # otherwise hang until the process group's 30-minute timeout
            from ..parallel.hop import hop_group
            watch = None
            if ctx.world > 1:
                # every rank has loaded its partitions before the watchdog
                # starts: ranks finish their (DA) data loads tens of seconds
                # apart, and that skew is not a stalled hop
                ctx.barrier()
            if ctx.world > 1 and self.o.hop_timeout:
                from ..parallel.health import HopWatch
                watch = HopWatch(ctx.rank, ctx.world, self.o.hop_timeout,
                                 logs_root=self.o.logs_root).start()
                tok = watch.begin("p2p warm-up", peers=[r for r in range(ctx.world)
                                                        if r != ctx.rank])
            try:
                self._hop_group = hop_group(ctx.world, ctx.rank, self.device, ctx.backend)
            finally:
                if watch is not None:
                    watch.end(tok)
                    watch.stop()
        self.epoch = 0
        self.failures = []
        self._fired = set()
        self.tracer = Tracer(ctx.rank, enabled=opts.trace)
        self._sync = torch.cuda.synchronize if self.device.type == "cuda" else None
        self._metrics_path = (os.path.join(opts.logs_root, "metrics.jsonl")
                              if opts.logs_root and ctx.rank == 0 else "")
        if ctx.rank == 0 and opts.logs_root:
            write_manifest(os.path.join(opts.logs_root, "manifest.json"),
                           make_data_catalog(self.dataset, self.P, ctx.world),
                           {"msts": self.msts, "partitions": self.P, "gpus": ctx.world,
                            "slots_per_gpu": self.V, "n_train": self.n_train, "n_valid": self.n_valid})

    # ------------------------------------------------------------------
    def _build_groups(self, model_ids):
        by_key = collections.defaultdict(list)
        for m in model_ids:
            by_key[pack_key(self.msts[m])].append(m)
        for key, ms in by_key.items():
            if key in self.groups:
                self.groups[key].add_models(ms, self.o.seed)
            else:
                self.groups[key] = PackGroup(key, ms, self.msts, self.store, self.device,
                                             self.dtype, seed_base=self.o.seed * 100,
                                             use_graphs=self.o.use_graphs, l2=self.o.l2)
                self.groups[key].lane = (len(self.groups) - 1) % self.effective_lanes()
            for m in ms:
                self.group_of[m] = self.groups[key]

    def owner(self, p):
        if self.task_parallel:
            return (p // self.P) % self.ctx.world
        return p // self.V

    def local_part(self, p):
        return p % self.P if self.task_parallel else self.store.local[p]

    def log(self, msg):
        if self.o.verbose and self.ctx.rank == 0:
            logs(msg)

    # ------------------------------------------------------------------
    def _hop_and_load(self, rnd):
        """Ship every model of this round to its partition's GPU."""
        rank = self.ctx.rank
        dest = {m: self.owner(p) for p, m in rnd.items()}
        holder = {m: (self.holder[m] if self.holder[m] is not None else dest[m]) for m in dest}
        moves = plan_moves(holder, dest)
        validate_plan(moves, self.ctx.world)
        # working sets per group on this rank
        mine = sorted(((m, self.local_part(p)) for p, m in rnd.items() if self.owner(p) == rank),
                      key=lambda t: (t[1], t[0]))
        per_group = collections.defaultdict(list)
        for m, lp in mine:
            per_group[self.group_of[m].key].append((m, lp))
        row_of = {}
        for key, jobs in per_group.items():
            w = self.groups[key].begin_round(jobs)
            for row, (m, _) in enumerate(jobs):
                row_of[m] = (w, row)
        incoming = {mv.model for mv in moves if mv.dst == rank}
        for m, (w, row) in row_of.items():
            if m not in incoming:
                w.load_local(row, m)
        hopt = self.o.hop_optimizer_state
        t0 = time.time()
        if moves and self.o.sim_hop_seconds and any(rank in (mv.src, mv.dst) for mv in moves):
            time.sleep(self.o.sim_hop_seconds * sum(mv.src == rank for mv in moves))
        if moves:
            def send_buf(m):
                st = self.group_of[m].state_row(m)
                return st if hopt else st[:self.group_of[m].layout.n_master]

            def recv_buf(m):
                w, row = row_of[m]
                return w.recv_buffer(row, hopt)
            n = execute_moves(moves, rank, send_buf, recv_buf, group=self._hop_group,
                              check=self.o.hop_check, watch=self.hop_watch)
            if n:
                for mv in moves:
                    if mv.src == rank:
                        self.hop_bytes += send_buf(mv.model).numel() * 4
        self.hop_time += time.time() - t0
        for m in dest:
            self.holder[m] = dest[m]
        return per_group, moves

    def _fault_check(self):
        spec = self.o.fault_inject
        if not spec:
            return
        f = spec.split(":")
        r, k = int(f[0]), int(f[1])
        kind = f[2] if len(f) > 2 else "raise"
        if r != self.ctx.rank or k != self.round_idx or (r, k) in self._fired:
            return
        self._fired.add((r, k))
        msg = "FAULT INJECTED at rank {} sub-epoch {}".format(r, k)
        if kind == "soft":
            raise SoftFault(msg)
        if kind == "exit":
            logs(msg + " (process exit)")
            os._exit(3)
        raise RuntimeError(msg)

    def _fault_check_batch(self, k):
        """Async runtime: the injection hook keyed by the job's sub-epoch."""
        saved = self.round_idx
        self.round_idx = k
        try:
            self._fault_check()
        finally:
            self.round_idx = saved

    def _train_local(self, per_group, max_steps):
        """Train + validate every local pack group; returns (results, images)."""
        results = []
        trained = 0
        tr = self.tracer
        for key, jobs in per_group.items():
            grp = self.groups[key]
            w = grp.current
            w.prepare(self.o.hop_optimizer_state)
            B = grp.batch_size
            steps = self.n_train // B
            if max_steps is not None:
                steps = min(steps, max_steps)
            with tr.span("train", sync=self._sync, arch=key[0], G=w.G, steps=steps):
                w.train_steps(steps)
                if self.o.sim_job_seconds:           # test hook: heterogeneous job lengths
                    d = self.o.sim_job_seconds
                    time.sleep(max(d[m % len(d)] for m, _ in jobs))
            trained += steps * B * w.G
            vsteps = self.n_valid // B
            if max_steps is not None:
                # shortened sub-epoch (bench): keep the valid/train ratio
                full = max(self.n_train // B, 1)
                vsteps = max(1, int(math.ceil(vsteps * steps / full)))
            with tr.span("valid", sync=self._sync, arch=key[0], G=w.G, steps=vsteps):
                w.validate(vsteps)
                mets = w.read_metrics()
                if self.o.sim_valid_seconds:
                    time.sleep(self.o.sim_valid_seconds)
            for row, (m, lp) in enumerate(jobs):
                results.append({"model": m, "dist_key": self.store.pids[lp], "metrics": mets[row],
                                "steps": steps, "batch": B, "partition": lp})
        return results, trained

    def run_round(self, rnd, epoch, max_steps=None):
        """One sub-epoch; failed (config, partition) pairs are requeued."""
        pending = dict(rnd)
        trained = 0
        t0 = time.time()
        self.mark_progress(True)
        for attempt in range(self.o.max_retries + 1):
            failed, images = self._attempt(pending, epoch, max_steps, attempt)
            trained += images
            if not failed:
                break
            pending = failed
        else:
            raise RuntimeError("sub-epoch {} failed {} times; giving up".format(
                self.round_idx, self.o.max_retries + 1))
        self.round_idx += 1
        self.mark_progress(False)
        if self.hop_watch is not None:
            # a boundary's hop waits for the slowest rank's previous round
            self.hop_watch.note_job(time.time() - t0)
        return trained

    def _attempt(self, rnd, epoch, max_steps, attempt):
        tr = self.tracer
        prev_holder = dict(self.holder)
        t_start = time.time()
        with tr.span("hop", sync=self._sync, round=self.round_idx, attempt=attempt):
            per_group, moves = self._hop_and_load(rnd)
        t_hop = time.time()
        error = None
        results, trained = [], 0
        try:
            self._fault_check()
            results, trained = self._train_local(per_group, max_steps)
        except SoftFault as e:
            error = str(e)
        if error is None:
            for key in per_group:
                self.groups[key].end_round()
        else:
            # drop the working copies: the pre-round states are still parked
            # in the previous holders' home rows
            for key in per_group:
                self.groups[key].current = None
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        t_end = time.time()
        local = {"rank": self.ctx.rank, "results": results, "t_start": t_start, "t_hop": t_hop,
                 "t_end": t_end, "error": error}
        with tr.span("report", round=self.round_idx):
            gathered = self.ctx.all_gather_object(local)
        failed = {}
        for g in gathered:
            if g["error"] is not None:
                for p, m in rnd.items():
                    if self.owner(p) == g["rank"]:
                        failed[p] = m
                        self.holder[m] = prev_holder[m]
                        fj = {"status": "FAILED", "epoch": epoch, "subepoch": self.round_idx,
                              "attempt": attempt, "rank": g["rank"], "partition": p,
                              "model_key": model_key(m, self.msts[m]), "error": g["error"]}
                        self.failures.append(fj)
                        self.log("JOB FAILED {} on partition {} (rank {}): {} -> requeued".format(
                            fj["model_key"], p, g["rank"], g["error"]))
                continue
            for r in g["results"]:
                self._record_job(epoch, g, r)
        if error is not None:
            trained = 0
        self.train_images += trained
        return failed, trained

    def _bk_msts(self):
        """Config list of the bookkeeping owner (the coordinator's during an
        asynchronous session on rank 0)."""
        return self.coord_msts if self.coord_msts is not None else self.msts

    def _record_job(self, epoch, g, r, subepoch=None):
        m = r["model"]
        mets = r["metrics"]
        sub = self.round_idx if subepoch is None else subepoch
        job = {"status": "SUCCESS", "epoch": epoch, "dist_key": r["dist_key"],
               "model_key": model_key(m, self._bk_msts()[m]),
               "loss_train": mets["train"]["loss"], "metric_train": mets["train"]["top5"],
               "loss_valid": mets["valid"]["loss"], "metric_valid": mets["valid"]["top5"],
               "top1_train": mets["train"]["top1"], "top1_valid": mets["valid"]["top1"],
               "n_train": mets["train"]["n"], "n_valid": mets["valid"]["n"],
               "start_time": g["t_start"], "end_time": g["t_end"],
               "init_time": 0.0, "train_time": g["t_end"] - g["t_hop"],
               "valid_time": 0.0, "exit_time": 0.0, "hop_time": g["t_hop"] - g["t_start"],
               "subepoch": sub, "rank": g["rank"]}
        self.jobs_info.setdefault(epoch, {})[(job["model_key"], r["dist_key"])] = job
        self.models_info[job["model_key"]].append(job)
        if self._metrics_path:
            rec = {"kind": "job", "epoch": epoch, "subepoch": sub, "cfg": job["model_key"],
                   "partition": r["dist_key"], "rank": g["rank"],
                   "loss": job["loss_train"], "top1": job["top1_train"],
                   "top5": job["metric_train"], "valid_loss": job["loss_valid"],
                   "valid_top1": job["top1_valid"], "valid_top5": job["metric_valid"],
                   "img_s": job["n_train"] / max(job["train_time"], 1e-9),
                   "hop_ms": job["hop_time"] * 1e3}
            with open(self._metrics_path, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def hop_estimate_s(self, gbps):
        """Transfer time of the largest hop payload at ``gbps`` GB/s (plus the
        test hook's forced link time): the coordinator's hold margin before
        a hop has been measured."""
        nbytes = 0
        for grp in self.groups.values():
            st = grp.home.state
            n = st.shape[1] if self.o.hop_optimizer_state else grp.layout.n_master
            nbytes = max(nbytes, n * st.element_size())
        return nbytes / (gbps * 1e9) + (self.o.sim_hop_seconds or 0.0)

    def log_hop_records(self, spans_per_rank, hold_log):
        """Rank 0, asynchronous runtime: one ``metrics.jsonl`` record per hop
        endpoint of the session -- sequence number, direction, model, peer,
        bytes, post -> arrival (the group's span, us) and the coordinator's
        hold before publishing it (us).  ``spans_per_rank``: every rank's
        ``HopService.spans``; ``hold_log``: the coordinator's
        ``(ticket, model, src, dst, seconds held, hold margin)``."""
        if not self._metrics_path:
            return
        with open(self._metrics_path, "a") as f:
            for r, spans in enumerate(spans_per_rank):
                for sp in spans:
                    t0, t1, d, m, peer = sp[:5]
                    nbytes, seq, hold = (sp[5], sp[6], sp[7]) if len(sp) > 7 else (0, -1, 0.0)
                    f.write(json.dumps({"kind": "hop", "seq": seq, "rank": r, "dir": d,
                                        "model": m, "peer": peer, "bytes": nbytes,
                                        "t_post": t0, "post_to_arrival_us": round((t1 - t0) * 1e6, 1),
                                        "hold_us": round(hold * 1e6, 1)}) + "\n")
            if hold_log:
                holds = [h[4] for h in hold_log]
                f.write(json.dumps({"kind": "hop_hold", "hops": len(holds),
                                    "hold_us_max": round(max(holds) * 1e6, 1),
                                    "hold_us_mean": round(sum(holds) / len(holds) * 1e6, 1),
                                    "margin_us_max": round(max(h[5] for h in hold_log) * 1e6, 1)})
                        + "\n")

    # ------------------------------------------------------------------
    def _epoch_summary(self, epoch):
        jobs = self.jobs_info.get(epoch, {})
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for (mk, _), j in jobs.items():
            a = agg[mk]
            a["tl"] += j["loss_train"] * j["n_train"]
            a["t5"] += j["metric_train"] * j["n_train"]
            a["t1"] += j["top1_train"] * j["n_train"]
            a["nt"] += j["n_train"]
            a["vl"] += j["loss_valid"] * j["n_valid"]
            a["v5"] += j["metric_valid"] * j["n_valid"]
            a["v1"] += j["top1_valid"] * j["n_valid"]
            a["nv"] += j["n_valid"]
        msts = self._bk_msts()
        for m in range(len(msts)):
            mk = model_key(m, msts[m])
            if mk not in agg:
                continue
            a = agg[mk]
            st = self.mst_state[m]
            nt, nv = max(a["nt"], 1), max(a["nv"], 1)
            st["train_loss"].append(a["tl"] / nt)
            st["valid_loss"].append(a["vl"] / nv)
            st["train_top5_error"].append(1 - a["t5"] / nt)
            st["valid_top5_error"].append(1 - a["v5"] / nv)
            st["train_top1_error"].append(1 - a["t1"] / nt)
            st["valid_top1_error"].append(1 - a["v1"] / nv)

    def checkpoint_all(self, epoch, models=None, holder_ok=False, version=None):
        """Queue async checkpoints (files ``{key}@{version}``) of the configs
        parked on this rank (``holder_ok``: the caller already picked this
        rank's configs).  The rows are snapshotted on the device and copied
        to pinned host memory on a side stream; nothing here waits."""
        if not self.o.models_root:
            return
        os.makedirs(self.o.models_root, exist_ok=True)
        ids = range(len(self.msts)) if models is None else models
        for m in ids:
            h = self.holder.get(m)
            if h is None:
                h = 0
            if not holder_ok and h != self.ctx.rank:
                continue
            grp = self.group_of[m]
            staged = self.stager.stage(grp.state_row(m))
            path = versioned(ckpt_path(self.o.models_root, m, self.msts[m]), version)
            meta = {"epoch": epoch, "subepoch": self.round_idx,
                    "model_key": model_key(m, self.msts[m]),
                    "mst": self.msts[m], "mst_str": mst_2_str(self.msts[m]),
                    "partitions_visited": sorted(
                        j["dist_key"] for j in self.jobs_info.get(epoch, {}).values()
                        if j["model_key"] == model_key(m, self.msts[m]))}
            self.writer.submit(lambda p=path, st=staged, mt=meta, L=grp.layout:
                               write_staged(p, L, st, mt))

    @staticmethod
    def ckpt_version(epoch, rounds_done=-1):
        return "e{}".format(epoch) if rounds_done < 0 else "e{}r{}".format(epoch, rounds_done)

    def _commit(self, epoch, rounds_done, epoch_done, sched_rng, models=None):
        """Consistent restart point: every rank's checkpoint writes are on
        disk before rank 0 publishes ``resume.json`` (atomic rename) naming
        them; superseded versions are dropped only after that."""
        if not self.o.models_root:
            return
        with self.tracer.span("checkpoint", epoch=epoch, rounds=rounds_done):
            self.writer.flush()
            self.ctx.barrier()
            if self.ctx.rank == 0:
                self.write_resume(epoch, rounds_done, epoch_done, sched_rng, models=models,
                                  version=self.ckpt_version(epoch, rounds_done))

    def write_resume(self, epoch, rounds_done, epoch_done, sched_rng, models=None, version=None):
        """Publish ``resume.json`` (atomic rename); every checkpoint it names
        is on disk already.  ``models`` (None = all) were just written as
        ``version``; afterwards their canonical CTQ files point at it."""
        if not self.o.models_root:
            return
        changed = []
        if version is not None:
            ids = range(len(self._bk_msts())) if models is None else models
            for m in ids:
                if self.ckpt_versions.get(m) != version:
                    self.ckpt_versions[m] = version
                    changed.append(m)
        if self.o.logs_root:
            dump_infos(self.o.logs_root, self.models_info, self.jobs_info)
        st = {"epoch": epoch, "rounds_done": rounds_done, "epoch_done": epoch_done,
              "round_idx": self.round_idx, "msts": self._bk_msts(),
              "states": {str(m): self.mst_state[m]["state"] for m in self.mst_state},
              "sched_rng": sched_rng, "failures": self.failures,
              "versions": {str(m): v for m, v in self.ckpt_versions.items()}}
        path = os.path.join(self.o.models_root, RESUME_FILE)
        with open(path + ".tmp", "w") as f:
            json.dump(st, f, default=str)
        os.replace(path + ".tmp", path)
        msts = self._bk_msts()
        for m in changed:
            publish_version(ckpt_path(self.o.models_root, m, msts[m]), self.ckpt_versions[m])

    def _resume(self):
        """Load ``resume.json`` + checkpoints; returns (epoch, rounds_to_skip, rng)."""
        path = os.path.join(self.o.models_root or "", RESUME_FILE)
        if not self.o.models_root or not os.path.exists(path):
            self.log("RESUME: no {} under models_root; starting fresh".format(RESUME_FILE))
            return 1, 0, None
        with open(path) as f:
            st = json.load(f)
        if len(st["msts"]) > len(self.msts):
            self.add_msts(st["msts"][len(self.msts):])
        versions = st.get("versions")
        fresh = []
        for m in range(len(self.msts)):
            path = ckpt_path(self.o.models_root, m, self.msts[m])
            if versions is not None:
                v = versions.get(str(m))
                path = versioned(path, v) if v else None
                if v:
                    self.ckpt_versions[m] = v
            if path is None:
                # never committed (e.g. more configs than partitions and a
                # crash before its first round): the deterministic seeded
                # initial state this engine built is exactly its start state
                fresh.append(m)
            else:
                weights, opt, _ = read_checkpoint(path)
                grp = self.group_of[m]
                host_to_state(grp.layout, weights, opt, grp.state_row(m))
            self.holder[m] = None            # every rank now holds the same copy
            self.mst_state[m]["state"] = st["states"].get(str(m), "RUNNING")
        lr = self.o.logs_root
        if lr and os.path.exists(os.path.join(lr, "jobs_info.pkl")):
            # files this framework wrote itself (dump_infos)
            with open(os.path.join(lr, "jobs_info.pkl"), "rb") as f:
                self.jobs_info = safe_pickle.load(f)
            with open(os.path.join(lr, "models_info.pkl"), "rb") as f:
                self.models_info = collections.defaultdict(list, safe_pickle.load(f))
        for e in sorted(self.jobs_info):
            if e < st["epoch"] or st["epoch_done"]:
                self._epoch_summary(e)
        if fresh:
            self.log("RESUME: configs {} had no committed checkpoint: seeded initial state"
                     .format(fresh))
        self.round_idx = st["round_idx"]
        self.failures = list(st.get("failures", []))
        self.log("RESUME: epoch {} after {} sub-epochs{}".format(
            st["epoch"], st["rounds_done"], " (epoch complete)" if st["epoch_done"] else ""))
        if st["epoch_done"]:
            return st["epoch"] + 1, 0, None
        return st["epoch"], st["rounds_done"], st.get("sched_rng")

    # ------------------------------------------------------------------
    # asynchronous runtime hooks (runtime.async_mop)
    def use_async(self, sub_epoch_resume=False):
        rt = self.o.runtime
        if rt not in ("auto", "async", "lockstep"):
            raise ValueError("unknown runtime {!r}".format(rt))
        lock_only = (self.task_parallel or self.o.ckpt_every == "subepoch" or sub_epoch_resume
                     or self.o.scheduler not in ("rotation", "greedy"))
        if rt == "async" and lock_only:
            raise ValueError("runtime='async' does not support scheduler={} / ckpt_every={} / "
                             "sub-epoch resume".format(self.o.scheduler, self.o.ckpt_every))
        return rt == "async" or (rt == "auto" and not lock_only)

    def stream_budget(self, pack_sizes=None):
        """The streams this engine can have active at once in training
        (name -> what it carries), for the queue budget
        (``profiles/r5_stream_budget.md``).  ``pack_sizes``: {pack key: G}
        of one batch (default: every group at its size on this rank)."""
        from ..models.resnet import _SC_BRANCH
        from .group import _SIDE_MIN_G, _SIDE_MIN_IMAGES
        out = {"compute": "step / validation graph replays, parking copies"}
        if pack_sizes is None:
            pack_sizes = {k: min(len(g.model_ids), self.V) for k, g in self.groups.items()}
        for key, G in pack_sizes.items():
            grp = self.groups[key]
            if (_SC_BRANCH and grp.arch.startswith("resnet") and "nobn" not in grp.arch
                    and self.dtype == torch.float32):
                out["branch"] = "ResNet projection shortcuts (fork / join in the step graph)"
            if G >= _SIDE_MIN_G and G * grp.batch_size >= _SIDE_MIN_IMAGES:
                out["side_wgrad"] = "first ~40 % of the batched weight gradients"
        nl = self.effective_lanes(len(pack_sizes))
        for i in range(1, nl):
            out["lane{}".format(i)] = "concurrent pack group"
        if self.ctx.world > 1 and not self.task_parallel:
            out["hop"] = "waits on parking events (RCCL's stream waits on it)"
            out["rccl_hop"] = "send / recv kernels of the hop communicator"
        return out

    def effective_lanes(self, ngroups=None):
        """Lanes actually used: at most ``o.lanes``, one per group, and -- at
        world > 1 -- no more than leaves the hop's two streams within the
        hardware queues."""
        n = max(1, int(self.o.lanes))
        if ngroups is not None:
            n = min(n, max(1, ngroups))
        if self.ctx.world > 1 and n > 1:
            n = max(1, min(n, HW_QUEUES - 3))      # compute/branch + hop + RCCL
        return n

    def lane_stream(self, lane):
        """The stream of concurrency lane ``lane`` (created on first use)."""
        st = self._lanes.get(lane)
        if st is None:
            st = torch.cuda.Stream(device=self.device)
            self._lanes[lane] = st
        return st

    def pack_order_key(self):
        """The schedulers' pack-aware order (``MOPScheduler.pack_key_fn``):
        key(m) = (-steps per partition visit, pack key).  None with
        ``pack_order`` off (the policies' own orders: rotation by config id,
        greedy shuffled).  Reads the coordinator's config list at call time,
        so configs added later (hyperopt) are keyed too."""
        if not self.o.pack_order:
            return None
        n = max(int(self.n_train), 1)

        def key(m):
            mst = self._bk_msts()[m]
            bs = max(int(mst["batch_size"]), 1)
            return (-((n + bs - 1) // bs), tuple(str(v) for v in pack_key(mst)))
        return key

    def async_scheduler(self, policy):
        """One scheduler per policy for the engine's lifetime (the greedy
        shuffle RNG continues across epochs and sessions)."""
        from ..scheduler.policies import GreedyScheduler, RotationScheduler
        sch = self._asched.get(policy)
        if sch is None:
            ids = list(range(len(self._bk_msts())))
            if policy == "rotation":
                sch = RotationScheduler(ids, list(range(self.P)), seed=self.o.seed)
            else:
                sch = GreedyScheduler(ids, list(range(self.P)), seed=self.o.seed,
                                      shuffle=self.o.shuffle)
            sch.pack_key_fn = self.pack_order_key()
            self._asched[policy] = sch
        return sch

    def control_channel(self):
        from .async_mop import Channel, LocalStore, rendezvous_addr, tcp_client
        self._nsession += 1
        # a fresh key space per session: the rendezvous store outlives engines
        tok = self.ctx.broadcast_object(os.urandom(6).hex() if self.ctx.rank == 0 else None)
        pfx = "cerebro_ctl/{}/{}".format(tok, self._nsession)
        if self.ctx.world <= 1:
            if self._chan is None:
                self._chan = LocalStore()
            return Channel(self._chan, pfx, self.o.ctrl_timeout)
        if self._chan is None:
            addr = rendezvous_addr()
            if addr is None:
                raise RuntimeError("asynchronous runtime needs MASTER_ADDR / MASTER_PORT")
            self._chan = (tcp_client(addr, self.o.ctrl_timeout), addr)
        return Channel(self._chan[0], pfx, self.o.ctrl_timeout, self._chan[1])

    def hop_group(self):
        """The process group (one communicator) every hop of this engine uses."""
        return self._hop_group

    def coord_begin(self):
        self.coord_msts = [dict(m) for m in self.msts]

    def coord_log(self, msg):
        self.log(msg)

    def coord_add_msts(self, new_msts):
        base = len(self.coord_msts)
        self.coord_msts.extend(dict(m) for m in new_msts)
        ids = list(range(base, len(self.coord_msts)))
        for m in ids:
            self.mst_state[m] = {"train_loss": [], "valid_loss": [], "train_top5_error": [],
                                 "valid_top5_error": [], "train_top1_error": [],
                                 "valid_top1_error": [], "state": "RUNNING"}
        for sch in self._asched.values():
            if sch is not None:
                sch.add_models(ids)
        return ids

    def worker_add_msts(self, new_msts):
        base = len(self.msts)
        self.msts.extend(dict(m) for m in new_msts)
        ids = list(range(base, len(self.msts)))
        for m in ids:
            self.holder[m] = None
        self._build_groups(ids)
        self.sched.add_models(ids)

    def coord_end(self, fin):
        """Adopt rank 0's end-of-session bookkeeping (JSON round trip)."""
        self.holder = {int(m): h for m, h in fin["holder"].items()}
        if self.coord_msts is None:          # ranks > 0
            self.mst_state = {int(m): v for m, v in fin["mst_state"].items()}
            self.jobs_info = {int(e): {(j[0], j[1]): j[2] for j in jobs}
                              for e, jobs in fin["jobs_info"].items()}
            self.models_info = collections.defaultdict(list, fin["models_info"])
            self.failures = list(fin["failures"])
            self.round_idx = fin["round_idx"]
        self.coord_msts = None
        assert len(self.msts) == len(fin["msts"]), "config lists diverged"

    def _run_async(self, first, num_epochs, mst_eval_fn=None, steps_of=None, round_budget=None):
        from .async_mop import run_session
        policy = "greedy" if self.o.scheduler == "greedy" else "rotation"
        return run_session(self, policy, first, num_epochs, mst_eval_fn, steps_of, round_budget)

    def run(self, num_epochs, mst_eval_fn=None):
        """Full semantic run: ``num_epochs`` MOP epochs (reference ``schedule``)."""
        t0 = time.time()
        first, skip, rng = (self._resume() if self.o.resume else (1, 0, None))
        hb = self._start_heartbeat()
        self._arm_watch()
        if self.use_async(sub_epoch_resume=bool(skip or rng)):
            try:
                if first <= num_epochs:
                    self._run_async(first, num_epochs, mst_eval_fn)
                self.writer.flush()
            finally:
                if hb is not None:
                    hb.stop()
                self._disarm_watch()
            return time.time() - t0
        try:
            for epoch in range(first, num_epochs + 1):
                active = [m for m in range(len(self.msts))
                          if self.mst_state[m]["state"] == "RUNNING"]
                if not active:
                    break
                self.epoch = epoch
                self.sched.models = list(active)
                if rng is not None:
                    self.sched.set_rng_state(rng)
                rng_at_start = self.sched.rng_state()
                self.sched.start_epoch(epoch)
                self.store.new_epoch(epoch)
                self.log("EPOCH:{}".format(epoch))
                self._run_epoch_rounds(epoch, skip=skip, rng=rng_at_start)
                skip, rng = 0, None
                self._epoch_summary(epoch)
                if self.ctx.rank == 0 and self.o.logs_root:
                    dump_infos(self.o.logs_root, self.models_info, self.jobs_info)
                if mst_eval_fn is not None:
                    decision = mst_eval_fn(self.mst_state) if self.ctx.rank == 0 else None
                    decision = self.ctx.broadcast_object(decision)
                    stop, _, new_msts = decision
                    for m in stop:
                        self.mst_state[m]["state"] = "COMPLETED"
                    if new_msts:
                        self.add_msts(new_msts)
                if self.o.ckpt_every != "none":
                    self.checkpoint_all(epoch, version=self.ckpt_version(epoch))
                    self._commit(epoch, -1, True, None)
            self.writer.flush()
        finally:
            if hb is not None:
                hb.stop()
            self._disarm_watch()
        return time.time() - t0

    def _arm_watch(self):
        """Collective: arm the hop watchdog for one run (world > 1, hops on)."""
        if (self.ctx.world <= 1 or self.task_parallel or not self.o.hop_timeout
                or self.hop_watch is not None):
            return None
        from ..parallel.health import HopWatch
        from .async_mop import rendezvous_addr, tcp_client
        tok = self.ctx.broadcast_object(os.urandom(6).hex() if self.ctx.rank == 0 else None)
        addr = rendezvous_addr()
        store = tcp_client(addr, 60) if addr is not None else None
        self.hop_watch = HopWatch(self.ctx.rank, self.ctx.world, self.o.hop_timeout,
                                  store=store, key="cerebro_hopwatch/" + tok,
                                  logs_root=self.o.logs_root).start()
        return self.hop_watch

    def _disarm_watch(self):
        if self.hop_watch is not None:
            self.hop_watch.stop()
            self.hop_watch = None

    def _start_heartbeat(self):
        if not getattr(self.o, "heartbeat", 0) or not self.ctx.initialized:
            return None
        from ..parallel.health import Heartbeat, default_store
        store = default_store()
        if store is None:
            return None
        self.hb = Heartbeat(store, self.ctx.rank, self.ctx.world, timeout=self.o.heartbeat,
                            logs_root=self.o.logs_root,
                            stall_timeout=getattr(self.o, "stall_timeout", 0) or None).start()
        return self.hb

    def mark_progress(self, busy):
        if self.hb is not None:
            self.hb.progress(self.round_idx, busy)

    def _after_round(self, epoch, rnd, rounds_done, rng):
        if self.o.ckpt_every == "subepoch":
            models = sorted(set(rnd.values()))
            self.checkpoint_all(epoch, models=models, version=self.ckpt_version(epoch, rounds_done))
            self._commit(epoch, rounds_done, False, rng, models=models)

    def _run_task_epoch(self, epoch, active, max_steps=None, skip=0, rng=None):
        """Task parallel: models are pinned to ranks round-robin; in round r
        every rank trains all its models on (its replica of) partition r.
        Round keys are pseudo-partitions m * P + r (see ``owner``)."""
        for r in range(skip, self.P):
            rnd = {m * self.P + r: m for m in active}
            self.run_round(rnd, epoch, max_steps)
            self._after_round(epoch, rnd, r + 1, rng)

    def _run_epoch_rounds(self, epoch, max_steps=None, skip=0, rng=None):
        if self.task_parallel:
            self._run_task_epoch(epoch, list(self.sched.models), max_steps, skip, rng)
            return
        k = 0
        if self.sched.lockstep:
            while True:
                rnd = self.sched.next_round()
                if rnd is None:
                    break
                if k >= skip:
                    self.run_round(rnd, epoch, max_steps)
                self.sched.finish_round(rnd)
                k += 1
                if k > skip:
                    self._after_round(epoch, rnd, k, rng)
        else:
            while not self.sched.epoch_done():
                pairs = self.sched.assign_all_idle()
                if not pairs:
                    raise RuntimeError("scheduler stalled")
                rnd = {w: m for m, w in pairs}
                if k >= skip:
                    self.run_round(rnd, epoch, max_steps)
                for m, w in pairs:
                    self.sched.complete(m, w)
                k += 1
                if k > skip:
                    self._after_round(epoch, rnd, k, rng)
        self.sched.monitor.check_epoch_complete(self.sched.models)

    def add_msts(self, new_msts):
        base = len(self.msts)
        self.msts.extend(dict(m) for m in new_msts)
        ids = list(range(base, len(self.msts)))
        for m in ids:
            self.holder[m] = None
            self.mst_state[m] = {"train_loss": [], "valid_loss": [], "train_top5_error": [],
                                 "valid_top5_error": [], "train_top1_error": [],
                                 "valid_top1_error": [], "state": "RUNNING"}
        self._build_groups(ids)
        self.sched.add_models(ids)

    def run_steps(self, total_steps, steps_per_round, epoch_start=1):
        """Bench mode: rounds of ``steps_per_round`` steps until ``total_steps``
        packed steps are done (the schedule continues across epochs)."""
        if total_steps <= 0:
            return 0
        self._arm_watch()
        try:
            return self._run_steps(total_steps, steps_per_round, epoch_start)
        finally:
            self._disarm_watch()

    def _run_steps(self, total_steps, steps_per_round, epoch_start):
        if self.use_async() and self.o.scheduler == "rotation":
            n = -(-total_steps // steps_per_round)
            last = total_steps - (n - 1) * steps_per_round
            self._run_async(epoch_start, 1 << 30, None,
                            steps_of=_StepsPlan(steps_per_round, last, n),
                            round_budget=n)
            return total_steps
        done = 0
        epoch = epoch_start
        while done < total_steps:
            self.sched.start_epoch(epoch)
            self.store.new_epoch(epoch)
            while done < total_steps:
                if self.sched.lockstep:
                    rnd = self.sched.next_round()
                    if rnd is None:
                        break
                else:
                    pairs = self.sched.assign_all_idle()
                    if not pairs:
                        break
                    rnd = {w: m for m, w in pairs}
                k = min(steps_per_round, total_steps - done)
                self.run_round(rnd, epoch, max_steps=k)
                if self.sched.lockstep:
                    self.sched.finish_round(rnd)
                else:
                    for w, m in rnd.items():
                        self.sched.complete(m, w)
                done += k
            epoch += 1
        return done

    def close(self):
        self.writer.close()
        self.stager.clear()
        # release captured HIP graphs deterministically (device drained first)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for grp in self.groups.values():
            for w in grp._work.values():
                if w.graph is not None:
                    w.graph.reset()
                    w.graph = None
                if w.vgraph is not None:
                    w.vgraph.reset()
                    w.vgraph = None
        if self.o.trace and self.o.logs_root:
            self.tracer.dump(os.path.join(self.o.logs_root, "traces"))
