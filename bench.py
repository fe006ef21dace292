#!/usr/bin/env python3
"""Headline benchmark: 8-config ResNet-50 ImageNet-112 MOP, aggregate img/s.

Workload = the reference's scalability experiment (BASELINE.md §1;
``cerebro_gpdb/imagenetcat.py:62-67`` ``param_grid_scalability``): 8
configurations lr{1e-3,1e-4,1e-5,1e-6} x lambda{1e-4,1e-6}, batch 32,
ResNet-50 at 112x112x3, 1000 classes, Adam, trained by Model Hopper
Parallelism over 8 data partitions on N GPUs (8/N partitions per GPU).

A *step* = one training iteration of every active configuration on its own
partition (8 x 32 = 256 images, whatever N is: total work is fixed, so
scaling is "strong").  Every step is a full fwd + bwd + Adam update.  The
timed region also contains the sub-epoch boundaries that fall inside it —
validation (3.9 % of train images, the reference's 50 000 / 1 281 280 ratio)
and the model hops over xGMI — every ``--steps_per_round`` steps, which is far
more often than the 5 005-step sub-epochs of the real run (conservative).

Data: synthetic ImageNet-shaped uint8 partitions generated in HBM; random-init
weights (no datasets/checkpoints offline).

Before the W warm-up steps one untimed priming round of PRIME_STEPS steps
runs (eager steps with per-problem kernel autotuning, HIP-graph capture of
the step and of validation, and the round's hops), so the timed window
never contains setup whatever W is; the JSON reports it as prime_steps.

value = (train images in the timed K steps, all GPUs) / max-over-ranks time.
vs_baseline = value / DA-Cerebro's aggregate img/s at the same worker count
(289 / 577 / 1002 / 1794 at 1 / 2 / 4 / 8).
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

BASELINE_IMG_S = {1: 289.0, 2: 577.0, 4: 1002.0, 8: 1794.0}
PRIME_STEPS = 4     # > group.warmup_eager (3 eager steps) -> the 4th is captured
TRAIN_IMAGES_PER_EPOCH = 1281280


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--steps_per_round", type=int, default=20)
    ap.add_argument("--train_per_partition", type=int, default=8192)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="fp32 = the reference's training precision (headline); bf16 is "
                         "reported as a diag_ metric")
    ap.add_argument("--no_graphs", action="store_true")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--workload", default="headline",
                    choices=["headline", "criteo16", "hetero8", "e2e16"],
                    help="headline = BASELINE.json's metric; criteo16 / hetero8 = the other "
                         "BASELINE configs (16-config Criteo confA grid; {ResNet-50, VGG-16} x "
                         "{lr, batch}); e2e16 = the reference's end-to-end 16-config grid "
                         "{vgg16, resnet50} x bs{32, 256} x lr x lambda (imagenetcat.py:44-49); "
                         "all but headline reported as diag_* metrics")
    ap.add_argument("--batch", type=int, default=0,
                    help="diagnostic: override the headline grid's batch size")
    ap.add_argument("--da", action="store_true",
                    help="diagnostic: write the synthetic partitions as Greenplum-format DA "
                         "pages first (untimed) and load them through the C++ page / TOAST / "
                         "pglz reader; the ETL is reported separately (etl_da)")
    ap.add_argument("--configs", type=int, default=0,
                    help="diagnostic: train only the first K configs (per-GPU work of N = 8/K "
                         "GPUs), or K > 8 configs packed (more learning rates); the headline "
                         "number always uses all 8")
    ap.add_argument("--logs_root", default="",
                    help="diagnostic: write the engine's metrics.jsonl (per-job and, at N > 1, "
                         "per-hop records: bytes, post -> arrival, hold, peer) here")
    ap.add_argument("--lanes", type=int, default=0,
                    help="diagnostic: concurrency lanes per rank (0 = the engine default)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not launched by torchrun: start one rank per GPU ourselves, as child
        # processes, BEFORE anything touches the GPU, and exit with their code
        sys.exit(_spawn_ranks(args.gpus))

    import torch
    from cerebro_ds_kpgi_amd.ops import set_backend
    from cerebro_ds_kpgi_amd.parallel import init_distributed, shutdown
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import get_msts
    from cerebro_ds_kpgi_amd.config import catalog as cat

    ctx = init_distributed()
    N = ctx.world
    if N != args.gpus:
        raise SystemExit("bench: --gpus {} but the job has {} ranks".format(args.gpus, N))
    backend = set_backend(args.backend)
    if args.workload == "criteo16":
        grid = dict(cat.param_grid_criteo)            # 2 lr x 2 lambda x 4 batch = 16
    elif args.workload == "hetero8":
        grid = dict(cat.param_grid_hetero_rv)         # 2 lr x 2 batch x {resnet50, vgg16}
    elif args.workload == "e2e16":
        grid = dict(cat.param_grid)                   # {vgg16, resnet50} x bs{32,256} x lr x l
    else:
        grid = dict(cat.param_grid_scalability)
        grid["model"] = [args.model]
        if args.batch:
            grid["batch_size"] = [args.batch]
    msts = get_msts(grid)
    if args.configs:
        if args.configs > len(msts):
            # a wider pack than the grid (e.g. the hetero workload's 10
            # NASNet configs as one G = 10 launch stream): more learning rates
            base = list(msts)
            msts = [dict(base[i % len(base)],
                         learning_rate=base[i % len(base)]["learning_rate"] * (1 + i // len(base)))
                    for i in range(args.configs)]
        msts = msts[:args.configs]
    S = len(msts)
    B = max(m["batch_size"] for m in msts)
    n_train = max(args.train_per_partition, B * args.steps_per_round)
    n_valid = max(B, int(round(n_train * cat.IMAGENET_VALID_TOTAL / cat.IMAGENET_TRAIN_TOTAL)))
    loader, da_stats, da_root = None, None, None
    if args.da:
        import tempfile
        from cerebro_ds_kpgi_amd.data import da
        da_root = ctx.broadcast_object(tempfile.mkdtemp(prefix="cer_da_") if ctx.rank == 0
                                       else None)
        if ctx.rank == 0:
            da.write_dataset(da_root, "criteo" if args.workload == "criteo16" else "imagenet",
                             max(1, S // N) * N, n_train, n_valid)
        ctx.barrier()
        da_stats = {}
        loader = da.da_partition_loader(da_root, ctx.device, stats=da_stats)
    opts = EngineOptions(slots_per_gpu=max(1, S // N), scheduler="rotation", n_train=n_train,
                         n_valid=n_valid, compute_dtype=args.dtype, use_graphs=not args.no_graphs,
                         verbose=False, ckpt_every="none", store_loader=loader,
                         logs_root=args.logs_root,
                         **({"lanes": args.lanes} if args.lanes else {}))
    mon = None
    if args.logs_root and int(os.environ.get("LOCAL_RANK", "0")) == 0:
        # 1 Hz host / GPU / xGMI sampler (sys_logs/sysmon_<host>.jsonl)
        from cerebro_ds_kpgi_amd.utils.sysmon import SysMonitor
        mon = SysMonitor(os.path.join(args.logs_root, "sys_logs")).start()
    t_etl = time.time()
    eng = MOPEngine(msts, ctx, opts)
    t_etl = time.time() - t_etl
    sync = (torch.cuda.synchronize if ctx.device.type == "cuda" else (lambda: None))

    # priming round, untimed, whatever --warmup is: the first steps of a
    # working set are eager (per-problem kernel-variant autotuning, the
    # MIOpen "find" step) and the step after them is captured as a HIP graph;
    # the round's validation is captured too and, at N > 1, its hops run.
    # This is setup (like compilation), so it precedes the W warm-up steps
    # and is reported separately as prime_steps
    prime = PRIME_STEPS
    eng.run_steps(prime, prime)
    # warm-up, untimed (every RCCL peer connection a hop may use was opened
    # when the engine created its hop communicator, parallel.hop.hop_group)
    if args.warmup > 0:
        eng.run_steps(args.warmup, args.steps_per_round)
    # xGMI link counters around the timed window (rank 0, outside it; the
    # hops' bytes on the wire at N > 1; None where amd-smi has no xgmi data)
    xg0 = _xgmi_sample() if N > 1 and ctx.rank == 0 else None
    sync()
    ctx.barrier()
    sync()
    img0, hop0, hopt0, hold0 = eng.train_images, eng.hop_bytes, eng.hop_time, eng.hop_hold_time
    t0 = time.time()
    eng.run_steps(args.steps, args.steps_per_round, epoch_start=2)
    sync()
    ctx.barrier()
    sync()
    dt = time.time() - t0
    dt_max = ctx.allreduce_max(dt)
    per_rank = ctx.all_gather_object({"images": eng.train_images - img0,
                                      "hop_bytes": eng.hop_bytes - hop0,
                                      "hop_s": eng.hop_time - hopt0,
                                      "hold_s": eng.hop_hold_time - hold0})
    imgs = sum(r["images"] for r in per_rank)
    value = imgs / dt_max
    xg = _xgmi_delta_gb(xg0, _xgmi_sample()) if xg0 else None
    if ctx.rank == 0:
        base = BASELINE_IMG_S.get(N)
        headline = (S == 8 and args.workload == "headline" and args.model == "resnet50"
                    and args.dtype == "fp32" and args.batch in (0, 32))
        out = {
            "metric": ("agg_train_images_per_sec_8cfg_resnet50_mop" if headline else
                       "diag_train_{}_per_sec_{}cfg_{}_mop_{}".format(
                           "samples" if args.workload == "criteo16" else "images", S,
                           {"headline": args.model, "criteo16": "criteo_confA",
                            "hetero8": "resnet50_vgg16", "e2e16": "e2e_vgg16_resnet50"}[
                               args.workload], args.dtype)),
            "value": round(value, 2),
            "unit": "samples/s" if args.workload == "criteo16" else "images/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "prime_steps": prime,
            "ms_per_step": round(1000.0 * dt_max / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / base, 3) if base and headline else None,
            "dtype": args.dtype,
            # how the conv / linear products are computed: fp32 storage and
            # accumulation with 3-pass split-bf16 MFMA products (hi*hi + hi*lo
            # + lo*hi, ~2^-16 relative per product; every op within 1e-4
            # relative L2 of fp64, tests/test_fp32_gpu.py) on our HIP kernels
            "math": ({"fp32": "3xbf16-split MFMA, fp32 accumulate/storage",
                      "bf16": "bf16 MFMA, fp32 accumulate"}[args.dtype]
                     if backend == "hip" else "PyTorch-ROCm/MIOpen " + args.dtype),
            "data": "synthetic via DA pages (C++ reader)" if args.da else "synthetic",
            "config": {"model": {"headline": args.model, "criteo16": "confA",
                                 "hetero8": "resnet50+vgg16",
                                 "e2e16": "vgg16+resnet50"}[args.workload],
                       "global_batch": sum(m["batch_size"] for m in msts), "seq_len": None,
                       "parallelism": "mop{}x{}".format(N, max(1, S // N)),
                       "configs": S,
                       "batch_per_config": sorted({m["batch_size"] for m in msts}),
                       "input": "7306-d sparse (39 ids)" if args.workload == "criteo16"
                       else "112x112x3",
                       "partitions": eng.P},
            "projected_makespan_s": round(S * (cat.CRITEO_TOTAL if args.workload == "criteo16"
                                               else TRAIN_IMAGES_PER_EPOCH) / value, 1),
            "baseline_makespan_s": ({1: 35440, 2: 17754, 4: 10229, 8: 5715}.get(N)
                                    if args.workload == "headline" else None),
            "backend": backend,
            "world_size": N,
            "dist_backend": ctx.backend or "none",
            "hop_bytes": sum(r["hop_bytes"] for r in per_rank),
            "hop_ms_max": round(1000.0 * max(r["hop_s"] for r in per_rank), 3),
            # the coordinator's hold of the hops a rank received (burst
            # grouping, runtime/async_mop.py), summed over the timed window
            "hold_ms_max": round(1000.0 * max(r["hold_s"] for r in per_rank), 3),
            # xGMI GB written per GPU over the timed window (amd-smi link
            # counters; includes any other traffic on the links), or null
            "xgmi_write_gb": xg,
        }
        if da_stats is not None:
            st = da_stats
            out["etl_da"] = {"engine_setup_s": round(t_etl, 3), "decode_s": round(st["decode_s"], 3),
                             "h2d_s": round(st["h2d_s"], 3),
                             "payload_GB": round(st["payload_bytes"] / 1e9, 3),
                             "stored_GB": round(st["stored_bytes"] / 1e9, 3),
                             "decode_GBps": round(st["payload_bytes"] / 1e9 /
                                                  max(st["decode_s"], 1e-9), 2),
                             "h2d_GBps": round(st["payload_bytes"] / 1e9 /
                                               max(st["h2d_s"], 1e-9), 2)}
        print(json.dumps(out))
        sys.stdout.flush()
    if mon is not None:
        mon.stop()
    if ctx.rank == 0:
        tune_log = os.environ.get("CER_TUNE_LOG")
        if tune_log and backend == "hip":
            from cerebro_ds_kpgi_amd.ops import _hip
            tt = _hip.tune_times()
            with open(tune_log, "w") as f:
                # [op, problem key, chosen variant, {variant: ms per launch}]
                json.dump([[op, list(key), v, tt.get((op, key), {})]
                           for (op, key), v in _hip.tuned_variants().items()], f)
    eng.close()
    if da_root and ctx.rank == 0:
        import shutil
        shutil.rmtree(da_root, ignore_errors=True)
    shutdown(ctx)


def _xgmi_sample():
    from cerebro_ds_kpgi_amd.utils.sysmon import xgmi_metrics
    return xgmi_metrics()


def _xgmi_delta_gb(first, last):
    from cerebro_ds_kpgi_amd.utils.sysmon import _xgmi_delta
    if not first or not last:
        return None
    d = _xgmi_delta(first, last, "write_kb")
    return {k: round(v, 3) for k, v in d.items()} or None


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _spawn_ranks(n):
    """``torch.distributed.run`` with n local ranks on 127.0.0.1 as a child
    process (the driver's own launch shape); returns its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ))


if __name__ == "__main__":
    main()
