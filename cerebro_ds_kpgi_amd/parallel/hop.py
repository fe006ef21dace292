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

**Matching rules.**  RCCL ignores point-to-point tags: it pairs a send with
a receive per peer, in posting order.  gloo pairs them by tag.  So that the
CPU (gloo) tests exercise the rules the GPUs run under, every hop-plane
operation is posted with tag 0 (``CER_HOP_TAGS=1`` restores per-transfer
tags, for A/B only): gloo then matches per peer in posting order too, and
an ordering bug fails on the CPU exactly as it would on RCCL.

**Headers.**  Every transfer is preceded by a 4 x int64 header
``[MAGIC, model, hop id, numel]`` in the same group; each receiver checks
the headers it got against the transfers it posted.  Two ranks that
disagree on the order (a swapped plan, a skipped hop) stop with
``HopOrderError`` instead of silently swapping two models' states (a size
mismatch cannot complete: the hop watchdog, ``health.HopWatch``, reports
it).  The cost is one 32-byte message per hop.
"""

import os

import torch
import torch.distributed as dist

HDR_MAGIC = 0x43455242            # "CERB"


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


class HopOrderError(RuntimeError):
    """Two endpoints posted their transfers in different orders."""


def tags_on():
    """Per-transfer tags (gloo-only matching aid); default off = RCCL rules."""
    return os.environ.get("CER_HOP_TAGS", "0") == "1"


def p2p(op, tensor, peer, group, tag):
    return dist.P2POp(op, tensor, peer, group, tag=tag if tags_on() else 0)


def checksum(t):
    """Position-sensitive fp64 digest of a state buffer (debug hop check):
    total sum, stride-7 subsample sum, first-half sum."""
    v = t.reshape(-1)
    n = v.numel()
    return torch.stack([v.sum(dtype=torch.float64), v[::7].sum(dtype=torch.float64),
                        v[:n // 2].sum(dtype=torch.float64)])


def _run_group(ops):
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


# test hook: reverse this rank's receive posting order (a mis-ordered plan)
_TEST_SWAP_RECVS = False


def post_transfers(items, rank, group, digest_of=None, watch=None):
    """Post this rank's transfers as ONE group and wait for it.

    ``items``: ``(hop_id, model, src, dst, buf)`` in the global hop order
    (identical on both endpoints).  Every transfer is three consecutive
    operations to / from its peer: the header, the payload and (with
    ``digest_of``) an fp64 digest.  Headers ride in the same group as their
    payloads on purpose: a group must stay one contiguous range of the
    rank's transfers in global order for the deadlock-freedom argument
    (``async_mop.HopService``); a separate header group before the payloads
    breaks it (tests/test_async_runtime.py caught that design deadlocking
    tag-blind).  After the group completes every receiver checks its
    headers, so a mis-ordered pair raises ``HopOrderError`` before anyone
    uses the states; a size mismatch cannot complete and is reported by the
    hop watchdog.  Returns ``[(hop_id, model, buf, sent_digest_or_None)]``
    for the receives.  ``watch`` (a ``health.HopWatch``) sees the group as
    an in-flight operation."""
    mine = [it for it in items if rank in (it[2], it[3])]
    if _TEST_SWAP_RECVS:
        rv = [i for i, it in enumerate(mine) if it[3] == rank]
        for i, j in zip(rv, rv[::-1]):
            if i < j:
                mine[i], mine[j] = mine[j], mine[i]
    if not mine:
        return []
    info = dict(hops=[it[0] for it in mine], models=[it[1] for it in mine],
                peers=sorted({it[3] if it[2] == rank else it[2] for it in mine}),
                bytes=sum(it[4].numel() * it[4].element_size() for it in mine))
    tok = watch.begin("group", **info) if watch is not None else None
    try:
        ops, out = [], []
        for hid, m, src, dst, buf in mine:
            if src == rank:
                h = torch.tensor([HDR_MAGIC, m, hid, buf.numel()], dtype=torch.int64,
                                 device=buf.device)
                ops.append(p2p(dist.isend, h, dst, group, tag=3 * hid))
                ops.append(p2p(dist.isend, buf, dst, group, tag=3 * hid + 1))
                if digest_of is not None:
                    ops.append(p2p(dist.isend, digest_of(m, buf), dst, group, tag=3 * hid + 2))
            else:
                h = torch.zeros(4, dtype=torch.int64, device=buf.device)
                ops.append(p2p(dist.irecv, h, src, group, tag=3 * hid))
                ops.append(p2p(dist.irecv, buf, src, group, tag=3 * hid + 1))
                sent = None
                if digest_of is not None:
                    sent = torch.empty(3, dtype=torch.float64, device=buf.device)
                    ops.append(p2p(dist.irecv, sent, src, group, tag=3 * hid + 2))
                out.append((hid, m, src, buf, sent, h))
        _run_group(ops)
    finally:
        if tok is not None:
            watch.end(tok)
    for hid, m, src, buf, sent, h in out:
        v = h.tolist()
        if v != [HDR_MAGIC, m, hid, buf.numel()]:
            raise HopOrderError(
                "rank {} posted the receive of model {} (hop {}, {} elements) from rank {}, "
                "but the sender's transfer in that slot is model {} (hop {}, {} elements, "
                "magic {:#x}): the endpoints posted in different orders"
                .format(rank, m, hid, buf.numel(), src, v[1], v[2], v[3], v[0]))
    return [(hid, m, buf, sent) for hid, m, src, buf, sent, h in out]


def verify_digests(recvs, rank):
    for hid, m, buf, sent in recvs:
        if sent is None:
            continue
        got = checksum(buf)
        if not torch.equal(got, sent):
            raise HopChecksumError("model {} arrived corrupted on rank {}: digest {} != sent {}"
                                   .format(m, rank, got.tolist(), sent.tolist()))


def execute_moves(moves, rank, send_buf, recv_buf, group=None, check=False, watch=None):
    """Lock-step runtime: post this rank's part of the plan; returns after
    all transfers land.  ``send_buf(model) -> tensor`` and
    ``recv_buf(model) -> tensor`` give the contiguous buffers; a move's
    index in the (replicated) plan is its hop id.

    ``check`` (debug, ``CER_HOP_CHECK=1``; SURVEY.md §5.2 stream-ordering
    checks): every sender ships the digest of its buffer (taken after a
    device synchronisation, from a second ``send_buf`` call) right behind
    the payload; every receiver compares it with the digest of what landed
    -- a hop racing a kernel that still writes the buffer raises
    ``HopChecksumError``."""
    items = []
    for i, mv in enumerate(moves):
        if mv.src == rank:
            items.append((i, mv.model, mv.src, mv.dst, send_buf(mv.model)))
        elif mv.dst == rank:
            items.append((i, mv.model, mv.src, mv.dst, recv_buf(mv.model)))
    if not items:
        return 0
    digest_of = None
    if check:
        if torch.cuda.is_available():
            torch.cuda.synchronize()

        def digest_of(m, buf):
            return checksum(send_buf(m))
    try:
        recvs = post_transfers(items, rank, group, digest_of=digest_of, watch=watch)
        if check:
            verify_digests(recvs, rank)
    except (HopOrderError, HopChecksumError) as e:
        if watch is not None:
            # the peers that completed their side of the group would block in
            # the next collective until the process group's timeout
            watch.abort("{} on rank {}: {}".format(type(e).__name__, rank, e))
        raise
    return len(items)


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
        ops.append(p2p(dist.isend, s, peer, group, tag=900000 + rank))
        ops.append(p2p(dist.irecv, r, peer, group, tag=900000 + peer))
    # gloo with device tensors (the one-GPU rehearsal) stages them through
    # the host outside the stream order: the fills must have landed before
    # it reads them and its copies before the check reads them (RCCL orders
    # both on its own; the syncs cost nothing at warm-up)
    cuda = torch.device(device).type == "cuda"
    if cuda:
        torch.cuda.synchronize(device)
    _run_group(ops)
    if cuda:
        torch.cuda.synchronize(device)
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
