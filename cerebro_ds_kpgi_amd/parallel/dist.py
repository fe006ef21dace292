"""Process groups: one process per GPU.

* data plane   — ``nccl`` backend (= RCCL on ROCm) over xGMI for model hops
                 (point-to-point) and the MA / DDP collectives; ``gloo`` when
                 running on CPU (plumbing tests),
* control plane — a ``gloo`` group for scheduler decisions, job results and
                 heartbeats (replaces the reference's SQL / XML-RPC / NFS
                 control channels).

Rendezvous always uses 127.0.0.1 by default (single node).
"""

import datetime
import os

import torch
import torch.distributed as dist


class DistContext(object):
    def __init__(self, rank=0, world=1, local_rank=0, device="cpu", backend=None, ctrl=None):
        self.rank, self.world, self.local_rank = rank, world, local_rank
        self.device = torch.device(device)
        self.backend = backend
        self.ctrl = ctrl

    @property
    def initialized(self):
        return self.world > 1 and dist.is_initialized()

    def barrier(self):
        if self.initialized:
            dist.barrier(group=self.ctrl)

    def all_gather_object(self, obj):
        if not self.initialized:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.ctrl)
        return out

    def broadcast_object(self, obj, src=0):
        if not self.initialized:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.ctrl)
        return box[0]

    def allreduce_max(self, value):
        if not self.initialized:
            return value
        t = torch.tensor([float(value)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        return float(t.item())


def init_distributed(backend="auto", device_type="auto", timeout_s=1800):
    """Initialise from torchrun-style env vars; single-process if absent."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type == "auto":
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        # one process per GPU.  More local ranks than GPUs is refused unless
        # CER_ALLOW_DEVICE_WRAP=1 (a rehearsal of the multi-rank path on a
        # small box, gloo data plane): the ranks then share devices, and a
        # result of such a run must not be mistaken for an N-GPU one
        ndev = torch.cuda.device_count()
        if ndev > 0 and local_rank >= ndev:
            if os.environ.get("CER_ALLOW_DEVICE_WRAP") != "1":
                raise RuntimeError(
                    "local rank {} but only {} GPU(s) visible; set CER_ALLOW_DEVICE_WRAP=1 "
                    "(with CER_DIST_BACKEND=gloo) to rehearse several ranks per GPU"
                    .format(local_rank, ndev))
            import sys
            sys.stderr.write("cerebro: rank {} (local {}) wraps onto cuda:{} of {} GPU(s) "
                             "(CER_ALLOW_DEVICE_WRAP rehearsal)\n".format(
                                 rank, local_rank, local_rank % ndev, ndev))
        dev_idx = local_rank % ndev if ndev > 0 else local_rank
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    if world <= 1:
        return DistContext(0, 1, 0, device, None, None)
    if backend == "auto":
        backend = os.environ.get("CER_DIST_BACKEND",
                                 "nccl" if device.type == "cuda" else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    kw = {}
    if backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    ctrl = dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD
    return DistContext(rank, world, local_rank, device, backend, ctrl)


def shutdown(ctx):
    if ctx is not None and ctx.initialized:
        try:
            dist.barrier(group=ctx.ctrl)
        finally:
            dist.destroy_process_group()
