"""The hop data plane on RCCL (GPU box, one GPU).

RCCL refuses two ranks on one device ("Duplicate GPU detected",
``scripts/dev/rccl_probe.py`` on the 1-GPU box, profiles/r4_hop_design.md),
so a multi-rank RCCL run needs the driver's 8-GPU node; the multi-rank
protocol (ordering, grouping, deadlock freedom) is covered on gloo by
tests/test_async_runtime.py.  Here, at world size 1 on the ``nccl`` backend
(RCCL), in a child process:

* the hop communicator is created the way ``parallel.hop.hop_group`` does
  and warmed (``warm_p2p``: no peer at world 1);
* the hop service's exact call pattern runs -- a side thread, its own HIP
  stream, a parking event to wait on, ONE ``batch_isend_irecv`` group on
  the hop communicator (a self send/recv of a ResNet-50-sized state row),
  an arrival event the compute stream then waits on -- and the row arrives
  bit-exact;
* RCCL's matching rule, which the tag-blind hop plane (``parallel.hop.p2p``)
  and its gloo tests rely on: two self-transfers whose receives are posted
  in swapped order, with distinct tags, pair in POSTING order (the tags are
  ignored) -- and the transfer headers expose the swap;
* the header + payload group of ``parallel.hop.post_transfers`` round-trips
  its int64 headers on RCCL;
* a MOP engine then runs one round with the RCCL process group live.
"""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import datetime, json, os, socket, sys, threading, time
sys.path.insert(0, {root!r})
import torch
import torch.distributed as dist
from cerebro_ds_kpgi_amd.parallel.dist import DistContext
from cerebro_ds_kpgi_amd.parallel.hop import warm_p2p

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                        timeout=datetime.timedelta(seconds=60))
hop = dist.new_group(ranks=[0], backend="nccl")
assert warm_p2p(1, 0, dev, group=hop) == 0
out = {{}}

# a ResNet-50 state row (params + Adam m, v): 3 x 25.6 M fp32
n = 3 * 25_636_712
row = torch.randn(n, device=dev)
dst = torch.empty(n, device=dev)
park = torch.cuda.Event()
row.mul_(1.0)                      # the "parking copy" on the compute stream
park.record()
arrived = {{}}

def service():
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.device(dev), torch.cuda.stream(s):
        s.wait_event(park)
        t0 = time.time()
        ops = [dist.P2POp(dist.isend, row, 0, hop, tag=1),
               dist.P2POp(dist.irecv, dst, 0, hop, tag=1)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        ev = torch.cuda.Event()
        ev.record(s)
        s.synchronize()
        arrived["ev"] = ev
        arrived["s"] = time.time() - t0

th = threading.Thread(target=service)
th.start()
th.join()
torch.cuda.current_stream().wait_event(arrived["ev"])
out["equal"] = bool(torch.equal(dst, row))
out["GBps"] = n * 4 / 1e9 / arrived["s"]

# RCCL pairs per peer in posting order, ignoring tags
from cerebro_ds_kpgi_amd.parallel.hop import HDR_MAGIC
def pair(swap):
    pay = {{m: torch.full((4096,), float(m + 1), device=dev) for m in (0, 1)}}
    hdr = {{m: torch.tensor([HDR_MAGIC, m, m, 4096], dtype=torch.int64, device=dev)
           for m in (0, 1)}}
    rp = {{m: torch.zeros(4096, device=dev) for m in (0, 1)}}
    rh = {{m: torch.zeros(4, dtype=torch.int64, device=dev) for m in (0, 1)}}
    ops = []
    for m in (0, 1):
        ops += [dist.P2POp(dist.isend, hdr[m], 0, hop, tag=10 + 2 * m),
                dist.P2POp(dist.isend, pay[m], 0, hop, tag=11 + 2 * m)]
    for m in ((1, 0) if swap else (0, 1)):
        ops += [dist.P2POp(dist.irecv, rh[m], 0, hop, tag=10 + 2 * m),
                dist.P2POp(dist.irecv, rp[m], 0, hop, tag=11 + 2 * m)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    torch.cuda.synchronize()
    return {{m: (rh[m].tolist()[1], float(rp[m][0])) for m in (0, 1)}}
out["in_order"] = pair(False)
out["swapped"] = pair(True)

# a MOP round with the RCCL process group live
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
msts = [{{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": 8, "model": "resnet18"}}
        for lr in (1e-3, 1e-4)]
eng = MOPEngine(msts, DistContext(0, 1, 0, dev, "nccl", None),
                EngineOptions(n_train=32, n_valid=8, slots_per_gpu=2, verbose=False,
                              ckpt_every="none", compute_dtype="fp32"))
eng.run_steps(2, 2)
torch.cuda.synchronize()
out["images"] = eng.train_images
out["finite"] = all(bool(torch.isfinite(g.home.state).all()) for g in eng.groups.values())
eng.close()
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
"""


def test_hop_pattern_on_rccl_world1():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-u", "-c", CHILD.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    import json
    out = json.loads(lines[-1][len("RESULT "):])
    print(out)
    assert out["equal"]
    # posted in order: each receive gets its own transfer (header names it)
    assert out["in_order"] == {"0": [0, 1.0], "1": [1, 2.0]}
    # posted swapped: RCCL pairs by posting order, not by tag -- the receive
    # posted first (model 1's) gets model 0's transfer, and its header says so
    assert out["swapped"] == {"0": [1, 2.0], "1": [0, 1.0]}
    assert out["images"] > 0 and out["finite"]


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]
