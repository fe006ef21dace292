"""Model hops: flat state rows moved GPU->GPU by point-to-point send/recv.

Replaces the reference's hop paths — weights returned as ``bytea`` through
SQL and rewritten to NFS after every sub-epoch (``cerebro_gpdb/ctq.py:110-121,
404-405``), MADlib model tables (UDAF), Cerebro ``ckpt_root`` files — with
one RCCL send/recv of one contiguous buffer over the direct xGMI link
(SURVEY.md E2, §2.9).  A hop plan is computed identically on every rank from
the replicated scheduler state, so every send has its matching recv by
construction; ``validate_plan`` checks the pairing.

All of a boundary's transfers are issued as one batched group
(``batch_isend_irecv`` -> ``ncclGroupStart/Send/Recv/GroupEnd``) on the
one hop communicator (``hop_group``), so independent links run concurrently.
"""

import torch
import torch.distributed as dist


class Move(object):
    __slots__ = ("model", "src", "dst", "nbytes")

    def __init__(self, model, src, dst, nbytes=0):
        self.model, self.src, self.dst, self.nbytes = model, src, dst, nbytes

    def __repr__(self):
        return "Move(m={}, {}->{})".format(self.model, self.src, self.dst)


def plan_moves(holder, destination):
    """holder: {model: rank now}, destination: {model: rank next round}."""
    moves = []
    for m in sorted(destination):
        s, d = holder[m], destination[m]
        if s != d:
            moves.append(Move(m, s, d))
    return moves


def validate_plan(moves, world):
    sends = {}
    for mv in moves:
        if not (0 <= mv.src < world and 0 <= mv.dst < world):
            raise ValueError("bad rank in {}".format(mv))
        if mv.model in sends:
            raise ValueError("model {} moved twice in one boundary".format(mv.model))
        sends[mv.model] = mv
    return True


class HopChecksumError(RuntimeError):
    pass


def checksum(t):
    """Position-sensitive fp64 digest of a state buffer (debug hop check):
    total sum, stride-7 subsample sum, first-half sum."""
    v = t.reshape(-1)
    n = v.numel()
    return torch.stack([v.sum(dtype=torch.float64), v[::7].sum(dtype=torch.float64),
                        v[:n // 2].sum(dtype=torch.float64)])


def execute_moves(moves, rank, send_buf, recv_buf, group=None, check=False):
    """Post this rank's part of the plan; returns after all transfers land.

    ``send_buf(model) -> tensor`` and ``recv_buf(model) -> tensor`` give the
    contiguous buffers.  Model id doubles as the tag (gloo matching).

    ``check`` (debug, ``CER_HOP_CHECK=1``; SURVEY.md §5.2 stream-ordering
    checks): after the transfers every sender ships the digest of what it
    sent, every receiver compares it with the digest of what landed, after a
    device synchronisation — a hop racing a kernel that still writes the
    buffer, or a mis-paired send/recv, raises ``HopChecksumError``.
    """
    n = _post(moves, rank, send_buf, recv_buf, group)
    if not check or not n:
        return n
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    ops, mine = [], {}
    for mv in moves:
        if mv.src == rank:
            ops.append(dist.P2POp(dist.isend, checksum(send_buf(mv.model)), mv.dst, group,
                                  tag=100000 + mv.model))
        elif mv.dst == rank:
            buf = recv_buf(mv.model)
            mine[mv.model] = (checksum(buf), torch.empty(3, dtype=torch.float64,
                                                         device=buf.device))
            ops.append(dist.P2POp(dist.irecv, mine[mv.model][1], mv.src, group,
                                  tag=100000 + mv.model))
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    for m, (got, sent) in mine.items():
        if not torch.equal(got, sent):
            raise HopChecksumError("model {} arrived corrupted on rank {}: digest {} != sent {}"
                                   .format(m, rank, got.tolist(), sent.tolist()))
    return n


def _post(moves, rank, send_buf, recv_buf, group):
    ops = []
    for mv in moves:
        if mv.src == rank:
            ops.append(dist.P2POp(dist.isend, send_buf(mv.model), mv.dst, group, tag=mv.model))
        elif mv.dst == rank:
            ops.append(dist.P2POp(dist.irecv, recv_buf(mv.model), mv.src, group, tag=mv.model))
    if not ops:
        return 0
    reqs = dist.batch_isend_irecv(ops)
    for r in reqs:
        r.wait()
    return len(ops)


def warm_p2p(world, rank, device, group=None):
    """Open every point-to-point connection this rank may use for a hop
    (RCCL sets peer connections up lazily, on the first send/recv to a peer:
    that setup must not land in the first real hop).  One tiny send/recv
    with every other rank, as one batched group."""
    if world <= 1:
        return 0
    ops = []
    bufs = []
    for peer in range(world):
        if peer == rank:
            continue
        s = torch.full((16,), float(rank), device=device)
        r = torch.empty(16, device=device)
        bufs.append((s, r, peer))
        ops.append(dist.P2POp(dist.isend, s, peer, group, tag=900000 + rank))
        ops.append(dist.P2POp(dist.irecv, r, peer, group, tag=900000 + peer))
    for q in dist.batch_isend_irecv(ops):
        q.wait()
    for s, r, peer in bufs:
        if float(r[0]) != float(peer):
            raise RuntimeError("p2p warm-up: rank {} got {} from {}".format(rank, float(r[0]), peer))
    return len(bufs)


def hop_group(world, rank, device, backend=None):
    """The hop data plane: ONE process group over all ranks (one RCCL
    communicator), created collectively and warmed -- every rank exchanges a
    tiny buffer with every other rank in one group, which initialises the
    communicator with all ranks taking part (a first call by a subset is
    undefined behaviour) and opens every peer connection a hop may use.

    Only the hop service uses it (the asynchronous runtime's hop thread, or
    the lock-step runtime's main thread): no other thread issues work on
    this communicator, so its operations are posted in the same global order
    on every rank (``async_mop.HopService``).  Replaces round 3's C(N, 2)
    two-rank communicators driven from one thread per peer."""
    if world <= 1:
        return None
    g = dist.new_group(ranks=list(range(world)), backend=backend)
    warm_p2p(world, rank, device, group=g)
    return g

