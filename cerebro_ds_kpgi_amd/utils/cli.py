"""Command-line surface shared by every ``run_*`` entry point.

Every flag of the reference's ``get_main_parser``
(``cerebro_gpdb/in_rdbms_helper.py:34-123``) is accepted with the same name
and default, so existing run scripts keep working.  DB-only flags
(``--db_name``, ``--load``, ``--client``/``--worker``, Spark/HDFS flags) are
accepted and recorded; they have no DB to act on here.

MI355X additions: ``--synthetic``, ``--num_gpus``,
``--scheduler``, ``--hop_optimizer_state``, ``--slots_per_gpu``,
``--data_dtype``, ``--compute_dtype``, ``--train_per_partition``,
``--valid_per_partition``, ``--backend`` and fault-injection/resume flags.
"""

import argparse
import random

from ..selection.grid import get_exp_specific_msts
from .logging import logs
from .seed import set_seed
from ..config.catalog import SEED


def _bool(v):
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("1", "true", "yes", "on")


def get_main_parser():
    p = argparse.ArgumentParser()
    # ---- reference flags (same names, same defaults) ----
    p.add_argument("--logs_root", type=str, default="")
    p.add_argument("--models_root", type=str, default="")
    p.add_argument("--train_name", type=str, default="imagenet_train_data_packed")
    p.add_argument("--valid_name", type=str, default="imagenet_valid_data_packed")
    p.add_argument("--run", action="store_true")
    p.add_argument("--load", action="store_true")
    p.add_argument("--db_name", type=str, default="cerebro")
    p.add_argument("--size", type=int, default=8)
    p.add_argument("--concurrency", type=int, default=0,
                   help="CTQ-Hyperopt: configs per TPE batch (default: --size)")
    p.add_argument("--num_epochs", type=int, default=10)
    p.add_argument("--drill_down_hetro", action="store_true")
    p.add_argument("--drill_down_model_size", action="store_true")
    p.add_argument("--drill_down_model_size_identifier", type=str, default="n")
    p.add_argument("--drill_down_scalability", action="store_true")
    p.add_argument("--best_model_run", action="store_true")
    p.add_argument("--criteo", action="store_true")
    p.add_argument("--criteo_breakdown", action="store_true")
    p.add_argument("--run_single", action="store_true")
    p.add_argument("--sanity", action="store_true")
    p.add_argument("--pytorchddp_sanity", action="store_true")
    p.add_argument("--client", action="store_true")
    p.add_argument("--worker", action="store_true")
    p.add_argument("--shuffle", action="store_true")
    p.add_argument("--drill_down_hetro_db_load", action="store_true")
    p.add_argument("--single_mst_index", type=int, default=0)
    p.add_argument("--hyperopt", action="store_true")
    p.add_argument("--cerebro_spark", action="store_true")
    p.add_argument("--spark_data_prepared", action="store_true")
    p.add_argument("--hdfs", action="store_true")
    p.add_argument("--max_num_config", type=int, default=32)
    p.add_argument("--hyperopt_models", type=str, default="",
                   help="comma list replacing the hyperopt space's model choices (reference: "
                        "resnet18,resnet34; BASELINE config 5: resnet50)")
    p.add_argument("--hyperopt_batch_buckets", type=str, default="none",
                   help="'none' (default) = the reference search space, every integer batch "
                        "size in [16, 256] (run_ctq_hyperopt.py:85-90). Opt-in performance "
                        "mode: a comma list of sizes inside that range (e.g. 16,32,64,128,256) "
                        "that TPE chooses from, so configs with equal (model, batch) train as "
                        "one packed launch stream -- a different search space, logged as such")
    # ---- MI355X engine flags ----
    p.add_argument("--synthetic", type=_bool, default=True,
                   help="generate ImageNet/Criteo-shaped data on the GPUs (no datasets offline)")
    p.add_argument("--tiny", action="store_true", help="tiny-CNN 32x32 plumbing grid (BASELINE config 1)")
    p.add_argument("--drill_down_hetero_rv", action="store_true",
                   help="{ResNet-50, VGG-16} x {lr, batch} heterogeneous grid (BASELINE config 4)")
    p.add_argument("--num_gpus", type=int, default=0,
                   help="GPUs (ranks) to use; 0 = WORLD_SIZE from the launcher")
    p.add_argument("--slots_per_gpu", type=int, default=0,
                   help="data partitions (virtual workers) per GPU; 0 = auto")
    p.add_argument("--scheduler", choices=["rotation", "greedy", "task", "ma", "ddp"],
                   default="rotation")
    p.add_argument("--pack_order", type=_bool, default=True,
                   help="co-schedule configs that pack into one launch stream, most steps per "
                        "partition visit first (false: the policies' own orders)")
    p.add_argument("--lanes", type=int, default=1,
                   help="pack groups of one batch replayed concurrently on this many streams "
                        "(1 = one after another)")
    p.add_argument("--hop_optimizer_state", type=_bool, default=True,
                   help="ship Adam moments with the model (False = reset per sub-epoch, reference CTQ semantics)")
    p.add_argument("--l2_mode", choices=["adam_wd", "none"], default="adam_wd",
                   help="lambda as torch Adam weight_decay (reference DDP path) or a no-op (Keras path quirk)")
    p.add_argument("--compute_dtype", choices=["bf16", "fp32"], default="fp32")
    p.add_argument("--optimizer", choices=["adam", "sgd"], default="adam",
                   help="per-config optimizer (reference: Adam); sgd = momentum 0.9, coupled L2")
    p.add_argument("--data_dtype", choices=["uint8", "fp32"], default="uint8")
    p.add_argument("--train_per_partition", type=int, default=0,
                   help="train images per partition (0 = full ImageNet split: 1 281 280 / partitions)")
    p.add_argument("--valid_per_partition", type=int, default=0,
                   help="valid images per partition (0 = 50 000 / partitions)")
    p.add_argument("--backend", choices=["auto", "hip", "torch"], default="auto",
                   help="kernel backend: our HIP kernels or the PyTorch oracle")
    p.add_argument("--dist_backend", choices=["auto", "nccl", "gloo"], default="auto")
    p.add_argument("--resume", action="store_true",
                   help="resume from models_root/resume.json (+ jobs_info in logs_root)")
    p.add_argument("--fault_inject", type=str, default="",
                   help="'rank:subepoch[:soft|:exit]' — fail that sub-epoch (fault-injection tests)")
    p.add_argument("--ckpt_every", choices=["epoch", "subepoch", "none"], default="",
                   help="checkpoint cadence (default: subepoch with --best_model_run, else epoch)")
    p.add_argument("--max_retries", type=int, default=2,
                   help="requeues of a (config, partition) pair after a recoverable failure")
    p.add_argument("--heartbeat", type=float, default=0.0,
                   help="watchdog timeout in seconds for worker heartbeats (0 = off)")
    p.add_argument("--stall_timeout", type=float, default=0.0,
                   help="flag a rank that stays inside one sub-epoch job longer than this "
                        "many seconds (hung collective / kernel; 0 = off)")
    p.add_argument("--trace", action="store_true",
                   help="write chrome-trace spans (logs_root/traces) and 1 Hz system telemetry")
    p.add_argument("--da", action="store_true", help="read partitions through the Direct-Access page reader")
    p.add_argument("--da_root", type=str, default="", help="root of GP-format segment files")
    p.add_argument("--fs_root", type=str, default="",
                   help="root of filesystem partitions ({train,valid}/{train,valid}_{i}.*; "
                        "create with python -m cerebro_ds_kpgi_amd.tools.make_fs_data)")
    return p


def main_prepare(argv=None, shuffle=True, to_set_seed=True, verbose=True):
    """Parse flags, seed, build the MST list (reference in_rdbms_helper.py:126-153)."""
    args = get_main_parser().parse_args(argv)
    if verbose:
        logs("Size:{}".format(args.size))
    if args.size == 1:
        args.train_name = "imagenet_train_data_packed_1"
        args.valid_name = "imagenet_valid_data_packed_1"
    if to_set_seed:
        set_seed(SEED)
    msts = get_exp_specific_msts(args)
    if args.optimizer != "adam":
        for m in msts:
            m["optimizer"] = args.optimizer
    if args.shuffle or shuffle:
        random.shuffle(msts)
    if verbose:
        logs(msts)
    if args.sanity:
        args.train_name = args.valid_name
        args.num_epochs = 1
    return args, msts
