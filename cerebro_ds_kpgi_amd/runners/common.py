"""Shared driver for every ``run_*`` entry point.

Each reference approach maps onto one engine of this framework:

=================================  ============================================
reference approach                  here
=================================  ============================================
DA-Cerebro / Cerebro standalone     MOP, greedy randomized scheduler
                                    (``--da`` reads Greenplum-format pages)
UDAF (``madlib_keras_fit_multiple``) MOP, lock-step rotation scheduler
CTQ                                 MOP, greedy scheduler (seeded shuffle)
CTQ-Hyperopt                        TPE batches of ``--concurrency`` configs, one
                                    fresh greedy-MOP session per batch
                                    (``run_batched_hyperopt``)
MA (``madlib_keras_fit``)           ``MAEngine`` (RCCL weighted averaging)
PyTorch DDP / DA-DDP                ``DDPEngine`` (RCCL gradient all-reduce)
Hyperopt-Spark                      MOP ``task`` scheduler + TPE batches
*-Hyperopt over MOP                 MOP + async TPE ``mst_eval_fn``
=================================  ============================================

Timing follows ``runner_helper.sh``: ``global.log`` gets the Start/End lines
and ``TOTAL EXECUTION TIME OVER ALL MST {s}``; data loading (ETL) is timed
and reported separately (the reference's ``DA`` vs ``DA_w_ETL``).
"""

import json
import os
import time

from ..ops import set_backend
from ..parallel import init_distributed, shutdown
from ..runtime.baselines import DDPEngine, MAEngine
from ..runtime.engine import EngineOptions, MOPEngine
from ..selection import hyperopt_helper as hh
from ..utils.cli import main_prepare
from ..utils.logging import GlobalLog, logs


def _loader(args, device):
    if getattr(args, "fs_root", ""):
        from ..data import fs
        if not fs.is_fs_root(args.fs_root):
            raise SystemExit("--fs_root {} holds no train/ partitions".format(args.fs_root))
        return fs.fs_partition_loader(args.fs_root, "criteo" if args.criteo else "imagenet",
                                      device)
    if not getattr(args, "da", False):
        return None
    from ..data import da
    root = args.da_root or os.path.join(args.logs_root or "/tmp", "da_data")
    if not os.path.exists(os.path.join(root, da.MANIFEST)):
        raise SystemExit("--da needs a DA dataset at --da_root (create one with "
                         "python -m cerebro_ds_kpgi_amd.tools.make_da_data)")
    return da.da_partition_loader(root, device)


def _opts(args, scheduler, loader):
    return EngineOptions(
        slots_per_gpu=args.slots_per_gpu, scheduler=scheduler,
        n_train=args.train_per_partition, n_valid=args.valid_per_partition,
        compute_dtype=args.compute_dtype, hop_optimizer_state=args.hop_optimizer_state,
        pack_order=getattr(args, "pack_order", True), lanes=getattr(args, "lanes", 1),
        l2=(args.l2_mode == "adam_wd"), logs_root=args.logs_root, models_root=args.models_root,
        seed=2018, shuffle=args.shuffle or scheduler == "greedy", fault_inject=args.fault_inject,
        dataset=("criteo" if args.criteo else None), store_loader=loader,
        trace=args.trace, resume=args.resume, max_retries=args.max_retries,
        heartbeat=args.heartbeat,
        stall_timeout=args.stall_timeout,
        ckpt_every=args.ckpt_every or ("subepoch" if args.best_model_run else "epoch"))


class _BatchedRun(object):
    """What ``run_approach`` reports for a batched TPE run."""

    def __init__(self, msts, mst_state, images, etl):
        self.msts, self.mst_state, self.train_images = msts, mst_state, images
        self.data_load_time = etl


def hyperopt_grid(args):
    """The reference search space (``run_ctq_hyperopt.py:76-91``), with the
    model choices replaced by ``--hyperopt_models`` when given."""
    grid = dict(hh.param_grid_hyperopt)
    models = [m for m in (getattr(args, "hyperopt_models", "") or "").split(",") if m]
    if models:
        grid["model"] = models
    buckets = getattr(args, "hyperopt_batch_buckets", "none") or "none"
    if buckets != "none":
        grid["batch_size_buckets"] = [int(b) for b in buckets.split(",") if b]
        from ..utils.logging import logs
        logs("HYPEROPT: batch sizes restricted to {} -- NOT the reference search space "
             "(every integer in [{}, {}]); results are not comparable with the reference's"
             .format(grid["batch_size_buckets"], grid["batch_size"][0], grid["batch_size"][1]))
    return grid


def run_batched_hyperopt(args, ctx, loader, param_grid=None, engine_kw=None):
    """CTQ-Hyperopt (reference ``run_ctq_hyperopt.py:122-160``): TPE proposes
    ``concurrency`` configs, ONE greedy MOP session trains that batch for
    ``num_epochs``, every config's last validation loss goes back to TPE
    (by its own trial id), repeat until ``max_num_config`` trials exist.
    Per-batch model/job logs: ``{logs_root}/models_info_grand.pkl`` /
    ``jobs_info_grand.pkl`` ({batch: ...}) as in the reference."""
    import pickle
    import argparse
    conc = args.concurrency or args.size or ctx.world
    grid = param_grid or hyperopt_grid(args)
    hp, msts, trials, domain, rand, _ = hh.init_hyperopt(grid, argparse.Namespace(size=conc))
    start, end = 0, len(msts)
    all_state, images, etl = {}, 0, 0.0
    models_grand, jobs_grand = {}, {}
    batch = 0
    while True:
        logs("STARTING BATCH:{}, FINISHED:{}".format(batch, start))
        opts = _opts(args, "greedy", loader)
        for k, v in (engine_kw or {}).items():
            setattr(opts, k, v)
        eng = MOPEngine(msts[start:end], ctx, opts)
        etl += getattr(eng, "data_load_time", 0.0)
        eng.run(args.num_epochs, mst_eval_fn=hh.mst_eval_fn(args.num_epochs))
        losses = [eng.mst_state[i]["valid_loss"][-1] for i in range(end - start)]
        hh.report_batch(trials, hp, start, end, losses)
        for i in range(end - start):
            all_state[start + i] = eng.mst_state[i]
        images += eng.train_images
        models_grand[batch] = dict(eng.models_info)
        jobs_grand[batch] = dict(eng.jobs_info)
        eng.close()
        if ctx.rank == 0 and args.logs_root:
            os.makedirs(args.logs_root, exist_ok=True)
            with open(os.path.join(args.logs_root, "models_info_grand.pkl"), "wb") as f:
                pickle.dump(models_grand, f)
            with open(os.path.join(args.logs_root, "jobs_info_grand.pkl"), "wb") as f:
                pickle.dump(jobs_grand, f)
        logs("ENDING BATCH:{}, FINISHED:{}".format(batch, end))
        batch += 1
        if len(hp) >= args.max_num_config:
            break
        n = min(conc, args.max_num_config - len(hp))
        hp, msts, start, end = hh.hyperopt_add_one_batch_configs(
            None, hp, msts, domain, trials, n, rand=rand)
    return _BatchedRun(msts, all_state, images, etl)


def run_approach(approach, argv=None, shuffle=True):
    args, msts = main_prepare(argv, shuffle=shuffle, verbose=True)
    if not args.run:
        logs("nothing to do (pass --run)")
        return None
    ctx = init_distributed(backend=args.dist_backend)
    set_backend(args.backend)
    exp = approach
    glog = None
    if ctx.rank == 0 and args.logs_root:
        glog = GlobalLog(os.path.dirname(os.path.abspath(args.logs_root)) or ".", exp)
        glog.start()
    t0 = time.time()
    mon = None
    if args.trace and args.logs_root and ctx.local_rank == 0:
        from ..utils.sysmon import SysMonitor
        mon = SysMonitor(os.path.join(args.logs_root, "sys_logs")).start()
    loader = _loader(args, ctx.device)
    tpe_state = None
    if approach == "ctq_hyperopt":
        eng = run_batched_hyperopt(args, ctx, loader)
    elif args.hyperopt and approach not in ("ma", "ddp"):
        # initial batch proposed by TPE (model ids == trial order)
        tpe_state = hh.init_hyperopt(hyperopt_grid(args), args=args)
        msts = tpe_state[1]
    if approach == "ctq_hyperopt":
        pass
    elif approach in ("ma",):
        eng = MAEngine(msts, ctx, _opts(args, "rotation", loader))
    elif approach in ("ddp",):
        from ..models.registry import TORCH_MODEL_NAMES
        msts = [dict(m, model=TORCH_MODEL_NAMES.get(m["model"], m["model"])) for m in msts]
        eng = DDPEngine(msts, ctx, _opts(args, "rotation", loader))
    else:
        sched = {"udaf": "rotation", "ctq": "greedy", "cerebro": args.scheduler,
                 "task": "task"}[approach]
        eng = MOPEngine(msts, ctx, _opts(args, sched, loader))
    etl = getattr(eng, "data_load_time", 0.0)
    mst_eval = None
    if approach == "ctq_hyperopt":
        pass
    elif isinstance(eng, MOPEngine):
        if tpe_state is not None:
            hp, _, trials, domain, rand, _ = tpe_state
            mst_eval = hh.mst_eval_fn_hyperopt(args.num_epochs, hp, trials, domain,
                                               args.max_num_config, rand, len(msts),
                                               param_grid=hyperopt_grid(args))
        else:
            mst_eval = hh.mst_eval_fn(args.num_epochs)
        epochs = 10 ** 6 if args.hyperopt else args.num_epochs
        eng.run(epochs, mst_eval_fn=mst_eval)
    else:
        eng.run(args.num_epochs)
    train_s = time.time() - t0
    images = eng.train_images
    if ctx.initialized:
        images = sum(ctx.all_gather_object(images))
    if ctx.rank == 0:
        makespan = glog.end() if glog else train_s
        summary = {"approach": approach, "gpus": ctx.world, "configs": len(eng.msts),
                   "epochs": args.num_epochs, "makespan_s": makespan, "etl_s": etl,
                   "train_images": images, "agg_img_per_s": images / max(train_s, 1e-9),
                   "lane_batches": getattr(eng, "lane_batches", 0),
                   "mst_state": {str(k): v for k, v in eng.mst_state.items()}}
        st = getattr(loader, "stats", None)
        if st and st.get("buffers"):
            # Direct-Access ETL (rank 0's partitions): C++ page walk + detoast +
            # pglz into pinned memory, then pinned -> HBM copies + conversion
            summary["etl_da"] = dict(
                st, payload_GB=st["payload_bytes"] / 1e9, stored_GB=st["stored_bytes"] / 1e9,
                decode_GBps=st["payload_bytes"] / 1e9 / max(st["decode_s"], 1e-9),
                h2d_GBps=st["payload_bytes"] / 1e9 / max(st["h2d_s"], 1e-9))
        logs("SUMMARY {}".format(json.dumps({k: v for k, v in summary.items()
                                              if k != "mst_state"})))
        if args.logs_root:
            os.makedirs(args.logs_root, exist_ok=True)
            with open(os.path.join(args.logs_root, "summary.json"), "w") as f:
                json.dump(summary, f, indent=1, default=str)
    if hasattr(eng, "close"):
        eng.close()
    if mon is not None:
        mon.stop()
    shutdown(ctx)
    return eng
