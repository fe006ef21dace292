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
"""

import collections
import math
import os
import time

import torch

from ..data.catalog import make_data_catalog, write_manifest
from ..data.store import PartitionStore
from ..models import dataset_of, pack_key
from ..parallel.hop import execute_moves, plan_moves, validate_plan
from ..scheduler import make_scheduler
from ..utils.keys import model_key, mst_2_str
from ..utils.logging import logs
from .checkpoint import AsyncWriter, ckpt_path, dump_infos, state_to_host, write_checkpoint
from .group import PackGroup


class EngineOptions(object):
    def __init__(self, **kw):
        self.slots_per_gpu = kw.get("slots_per_gpu", 0)
        self.scheduler = kw.get("scheduler", "rotation")
        self.n_train = kw.get("n_train", 0)
        self.n_valid = kw.get("n_valid", 0)
        self.compute_dtype = kw.get("compute_dtype", "bf16")
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
        self.groups = {}
        self.group_of = {}
        self._build_groups(range(S))
        self.holder = {m: None for m in range(S)}    # None = every rank has the init copy
        self.sched = make_scheduler(opts.scheduler, list(range(S)), list(range(self.P)),
                                    seed=opts.seed, shuffle=opts.shuffle)
        self.models_info = collections.defaultdict(list)
        self.jobs_info = {}
        self.mst_state = {m: {"train_loss": [], "valid_loss": [], "train_top5_error": [],
                              "valid_top5_error": [], "train_top1_error": [],
                              "valid_top1_error": [], "state": "RUNNING"} for m in range(S)}
        self.writer = AsyncWriter()
        self.train_images = 0
        self.round_idx = 0
        self.hop_bytes = 0
        self.hop_time = 0.0
        self.epoch = 0
        if ctx.rank == 0 and opts.logs_root:
            write_manifest(os.path.join(opts.logs_root, "manifest.json"),
                           make_data_catalog(self.dataset, self.P, ctx.world),
                           {"msts": self.msts, "partitions": self.P, "gpus": ctx.world,
                            "slots_per_gpu": V, "n_train": self.n_train, "n_valid": self.n_valid})

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
        if moves:
            def send_buf(m):
                st = self.group_of[m].state_row(m)
                return st if hopt else st[:self.group_of[m].layout.n_master]

            def recv_buf(m):
                w, row = row_of[m]
                return w.recv_buffer(row, hopt)
            n = execute_moves(moves, rank, send_buf, recv_buf)
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
        r, k = [int(v) for v in spec.split(":")]
        if r == self.ctx.rank and k == self.round_idx:
            raise RuntimeError("FAULT INJECTED at rank {} sub-epoch {}".format(r, k))

    def run_round(self, rnd, epoch, max_steps=None):
        t_start = time.time()
        per_group, moves = self._hop_and_load(rnd)
        t_hop = time.time()
        self._fault_check()
        results = []
        trained = 0
        for key, jobs in per_group.items():
            grp = self.groups[key]
            w = grp.current
            w.prepare(self.o.hop_optimizer_state)
            B = grp.batch_size
            steps = self.n_train // B
            if max_steps is not None:
                steps = min(steps, max_steps)
            w.train_steps(steps)
            trained += steps * B * w.G
            vsteps = self.n_valid // B
            if max_steps is not None:
                # shortened sub-epoch (bench): keep the valid/train ratio
                full = max(self.n_train // B, 1)
                vsteps = max(1, int(math.ceil(vsteps * steps / full)))
            w.validate(vsteps)
            mets = w.read_metrics()
            for row, (m, lp) in enumerate(jobs):
                results.append({"model": m, "dist_key": self.store.pids[lp], "metrics": mets[row],
                                "steps": steps, "batch": B})
            grp.end_round()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        t_end = time.time()
        self.train_images += trained
        local = {"rank": self.ctx.rank, "results": results, "t_start": t_start, "t_hop": t_hop,
                 "t_end": t_end}
        gathered = self.ctx.all_gather_object(local)
        for g in gathered:
            for r in g["results"]:
                m = r["model"]
                mets = r["metrics"]
                job = {"status": "SUCCESS", "epoch": epoch, "dist_key": r["dist_key"],
                       "model_key": model_key(m, self.msts[m]),
                       "loss_train": mets["train"]["loss"], "metric_train": mets["train"]["top5"],
                       "loss_valid": mets["valid"]["loss"], "metric_valid": mets["valid"]["top5"],
                       "top1_train": mets["train"]["top1"], "top1_valid": mets["valid"]["top1"],
                       "n_train": mets["train"]["n"], "n_valid": mets["valid"]["n"],
                       "start_time": g["t_start"], "end_time": g["t_end"],
                       "init_time": 0.0, "train_time": g["t_end"] - g["t_hop"],
                       "valid_time": 0.0, "exit_time": 0.0, "hop_time": g["t_hop"] - g["t_start"],
                       "subepoch": self.round_idx}
                self.jobs_info.setdefault(epoch, {})[(job["model_key"], r["dist_key"])] = job
                self.models_info[job["model_key"]].append(job)
        self.round_idx += 1
        return trained

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
        for m in range(len(self.msts)):
            mk = model_key(m, self.msts[m])
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

    def checkpoint_all(self, epoch):
        if not self.o.models_root:
            return
        os.makedirs(self.o.models_root, exist_ok=True)
        for m in range(len(self.msts)):
            h = self.holder[m]
            if h is None:
                h = 0
            if h != self.ctx.rank:
                continue
            grp = self.group_of[m]
            weights, opt = state_to_host(grp.layout, grp.state_row(m))
            path = ckpt_path(self.o.models_root, m, self.msts[m])
            meta = {"epoch": epoch, "model_key": model_key(m, self.msts[m]),
                    "mst": self.msts[m], "mst_str": mst_2_str(self.msts[m])}
            self.writer.submit(lambda p=path, w=weights, o=opt, mt=meta, L=grp.layout:
                               write_checkpoint(p, L, w, o, mt))

    def run(self, num_epochs, mst_eval_fn=None):
        """Full semantic run: ``num_epochs`` MOP epochs (reference ``schedule``)."""
        t0 = time.time()
        for epoch in range(1, num_epochs + 1):
            active = [m for m in range(len(self.msts)) if self.mst_state[m]["state"] == "RUNNING"]
            if not active:
                break
            self.epoch = epoch
            self.sched.models = list(active)
            self.sched.start_epoch(epoch)
            self.store.new_epoch(epoch)
            self.log("EPOCH:{}".format(epoch))
            self._run_epoch_rounds(epoch)
            self._epoch_summary(epoch)
            if self.ctx.rank == 0 and self.o.logs_root:
                dump_infos(self.o.logs_root, self.models_info, self.jobs_info)
            if self.o.ckpt_every != "none":
                self.checkpoint_all(epoch)
            if mst_eval_fn is not None:
                decision = mst_eval_fn(self.mst_state) if self.ctx.rank == 0 else None
                decision = self.ctx.broadcast_object(decision)
                stop, _, new_msts = decision
                for m in stop:
                    self.mst_state[m]["state"] = "COMPLETED"
                if new_msts:
                    self.add_msts(new_msts)
        self.writer.flush()
        return time.time() - t0

    def _run_task_epoch(self, epoch, active, max_steps=None):
        """Task parallel: models are pinned to ranks round-robin; in round r
        every rank trains all its models on (its replica of) partition r.
        Round keys are pseudo-partitions m * P + r (see ``owner``)."""
        for r in range(self.P):
            rnd = {m * self.P + r: m for m in active}
            self.run_round(rnd, epoch, max_steps)

    def _run_epoch_rounds(self, epoch, max_steps=None):
        if self.task_parallel:
            self._run_task_epoch(epoch, list(self.sched.models), max_steps)
            return
        if self.sched.lockstep:
            while True:
                rnd = self.sched.next_round()
                if rnd is None:
                    break
                self.run_round(rnd, epoch, max_steps)
                self.sched.finish_round(rnd)
        else:
            while not self.sched.epoch_done():
                pairs = self.sched.assign_all_idle()
                if not pairs:
                    raise RuntimeError("scheduler stalled")
                rnd = {w: m for m, w in pairs}
                self.run_round(rnd, epoch, max_steps)
                for m, w in pairs:
                    self.sched.complete(m, w)
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
