"""Probe: can several RCCL ranks share one GPU on this box?

Run under torchrun with --nproc-per-node K on a 1-GPU box.  Every rank binds
cuda:0, initialises the ``nccl`` (RCCL) backend, runs an all-reduce, a ring
shift as one ``batch_isend_irecv`` group on a dedicated process group from a
side thread (the hop-service shape), and prints one line per rank.  If RCCL
refuses duplicate devices the error is printed and the rank exits 3.
"""

import datetime
import os
import sys
import threading

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev,
                                timeout=datetime.timedelta(seconds=60))
        t = torch.full((4,), float(rank + 1), device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
    except Exception as e:                      # noqa: BLE001 -- report and stop
        print("rank {} nccl init/all_reduce failed: {}: {}".format(rank, type(e).__name__, e),
              flush=True)
        sys.exit(3)
    hop = dist.new_group(backend="nccl")
    out = {}

    def ring():
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            snd = torch.full((1 << 20,), float(rank), device=dev)
            rcv = torch.empty(1 << 20, device=dev)
            ops = [dist.P2POp(dist.isend, snd, (rank + 1) % world, hop),
                   dist.P2POp(dist.irecv, rcv, (rank - 1) % world, hop)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            s.synchronize()
            out["got"] = float(rcv[0])

    th = threading.Thread(target=ring)
    th.start()
    th.join()
    print("rank {} all_reduce={} ring_got={} (expect {})".format(
        rank, float(t[0]), out.get("got"), float((rank - 1) % world)), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
