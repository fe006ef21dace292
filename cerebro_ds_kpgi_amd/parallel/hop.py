"""Model hops: flat state rows moved GPU->GPU by point-to-point send/recv.

Replaces the reference's hop paths — weights returned as ``bytea`` through
SQL and rewritten to NFS after every sub-epoch (``cerebro_gpdb/ctq.py:110-121,
404-405``), MADlib model tables (UDAF), Cerebro ``ckpt_root`` files — with
one RCCL send/recv of one contiguous buffer over the direct xGMI link
(SURVEY.md E2, §2.9).  A hop plan is computed identically on every rank from
the replicated scheduler state, so every send has its matching recv by
construction; ``validate_plan`` checks the pairing.

All of a boundary's transfers are issued as one batched group
(``batch_isend_irecv`` -> ``ncclGroupStart/Send/Recv/GroupEnd``) so
independent links run concurrently.
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


def execute_moves(moves, rank, send_buf, recv_buf, group=None):
    """Post this rank's part of the plan; returns after all transfers land.

    ``send_buf(model) -> tensor`` and ``recv_buf(model) -> tensor`` give the
    contiguous buffers.  Model id doubles as the tag (gloo matching).
    """
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
