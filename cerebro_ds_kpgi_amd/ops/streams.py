"""Weight-gradient scheduling: batched (deferred) wgrads, one optional side batch.

Batched wgrads (default on, ``CER_WGRAD_BATCH=0`` disables): inside
``deferred_wgrad()`` (the engine's training step) a layer's weight-gradient
GEMM is only queued (``cer_wgrad_batch_add``); ``join`` — at the end of the
context and before the optimizer — launches the queue as a few multi-layer
kernels (``wgrad_batch`` in csrc/hip/conv.hip).  The operands stay referenced
here until the flush.

Split batch (packs of >= 4 configs, ``deferred_wgrad(side_frac=0.4)`` from
runtime/group.py): in backward a layer's input gradient (dgrad) is on the
critical path while its weight gradient is only needed by the optimizer.
Once 40 % of the previous step's layer count is queued, that batch -- the
upper stages' wgrads -- launches ONCE on a per-device side stream (forked
from the current stream at that point) on a capped, persistent grid
(``CER_WGB_SPLIT_GRID`` = 96 blocks), so it runs on a slice of the CUs while
the dgrad / BN-backward chain of the lower stages keeps the rest; the
remaining layers launch at the end on the current stream with the full grid;
``join`` makes the current stream wait for the side batch before the
optimizer.  Both are plain stream/event operations, so a captured HIP graph
keeps the fork / join.  Measured (profiles/r2_ab_wgrad_chunk.md): +1.6 % at 8
packed configs, +1.3 % at 4; one-config packs keep the single batch (a split
costs them 3 %).  Per-layer side-stream wgrads, fixed chunks, more side
batches and an optimizer update split across the streams all measured
slower or neutral (same file) and were removed in round 3.

Tensors read by the side batch are ``record_stream``-ed so the caching
allocator does not hand their memory to the main stream while it may still
read them.
"""

import contextlib
import os

import torch

_SIDE = {}
_PENDING = set()

_BATCH = os.environ.get("CER_WGRAD_BATCH", "1") != "0"
_BATCH_VARIANT = int(os.environ.get("CER_WGB_VARIANT", "1"))   # reg 128x128 (A/B in profiles/)
# blocks of the side batch: a small grid walks its tiles persistently on a
# few CUs, leaving the rest to the dgrad chain
_SPLIT_GRID = int(os.environ.get("CER_WGB_SPLIT_GRID", "96"))
_DEFER = 0
_HELD = []          # operands of queued wgrads (alive until the flush)
_NSTEP = 0          # layers queued in the current deferred block
_LAST = {}          # ... in the previous block of the same key
_SPLIT_AT = 0       # layers after which the side batch launches (0: no split)
_FORCE_SPLIT = [0]  # test hook: split after exactly this many layers (0: off)


def batching():
    """True while wgrads are being queued (inside ``deferred_wgrad``)."""
    return _DEFER > 0


def hold(*tensors, grad_ptr=None):
    """Keep a queued layer's operands alive until its batch is launched; the
    ``_SPLIT_AT``-th queued layer of a split step launches the side batch.
    (``grad_ptr``: where the layer's gradient lands; kept for API stability.)"""
    global _NSTEP, _SPLIT_AT
    _HELD.extend(t for t in tensors if t is not None)
    _NSTEP += 1
    if _DEFER and _SPLIT_AT > 0 and _NSTEP >= _SPLIT_AT and torch.cuda.is_available():
        flush_wgrad(side=True)
        _SPLIT_AT = 0                              # one side batch per step


_ROWS = [None]


def set_batch_rows(rows):
    """Rows of the reduction per split for the next queued fp32/bf16 wgrads
    (0: the library default, CER_WGB_ROWS or 1024)."""
    if _ROWS[0] != rows:
        from . import _hip
        _hip.lib().cer_wgrad_batch_set_rows(int(rows))
        _ROWS[0] = rows


def set_batch_variant(v):
    global _BATCH_VARIANT
    _BATCH_VARIANT = int(v)


@contextlib.contextmanager
def deferred_wgrad(enabled=True, side_frac=0.0, key=None):
    """Queue HIP weight gradients issued inside the block; flush them on exit.

    ``side_frac`` > 0: once that fraction of the previous block's layer count
    (same ``key``) is queued, the batch so far launches ONCE on the side
    stream on a capped grid (``CER_WGB_SPLIT_GRID`` blocks) and overlaps the
    rest of backward; the remaining layers launch at the end as usual, with
    the full grid."""
    global _DEFER, _NSTEP, _SPLIT_AT
    on = enabled and _BATCH
    if on:
        if _DEFER == 0:
            _SPLIT_AT = 0
            _FORKED.clear()
            if side_frac > 0 and _LAST.get(key, 0) > 1:
                _SPLIT_AT = -(-int(round(side_frac * 1000)) * _LAST[key] // 1000)
                if _FORCE_SPLIT[0]:
                    _SPLIT_AT = _FORCE_SPLIT[0]
            _NSTEP = 0
        _DEFER += 1
    try:
        yield
    finally:
        if on:
            _DEFER -= 1
            if _DEFER == 0:
                flush_wgrad()
                _LAST[key] = _NSTEP
                _SPLIT_AT = 0


def flush_wgrad(discard=False, side=False):
    if not _HELD:
        return
    from . import _hip
    if side and not discard:
        cur = torch.cuda.current_stream()
        dev = cur.device.index
        st = _side(dev)
        st.wait_stream(cur)              # the fork: every queued dy is issued by now
        # the queued layers' operands may come from BOTH streams of a block
        # with a branch (ResNet projection shortcut): when the split fires
        # on the branch, the main stream's earlier work (e.g. c2's dz) is
        # not ordered before it, and vice versa -- wait on the other one too
        other = _other_stream(dev, cur)
        if other is not None:
            st.wait_stream(other)
        L = _hip.lib()
        L.cer_wgrad_batch_set_grid(_SPLIT_GRID)
        try:
            rc = L.cer_wgrad_batch_flush(_BATCH_VARIANT, 0, _hip.c_p(st.cuda_stream))
        finally:
            L.cer_wgrad_batch_set_grid(0)
        for t in _HELD:
            t.record_stream(st)
        _PENDING.add(dev)
    else:
        cur = torch.cuda.current_stream()
        for t in _HELD:                  # operands made on a branch stream
            t.record_stream(cur)
        rc = _hip.lib().cer_wgrad_batch_flush(_BATCH_VARIANT, 1 if discard else 0, _hip._stream())
    del _HELD[:]
    _hip._check(rc, "cer_wgrad_batch_flush")


_BRANCH = {}


def branch_stream(dev):
    """Per-device stream for a model's parallel branch (ResNet projection
    shortcuts, models/resnet.py); autograd runs the branch's backward there."""
    s = _BRANCH.get(dev)
    if s is None:
        s = torch.cuda.Stream(device=dev)
        _BRANCH[dev] = s
    return s


_PARENT = {}
_FORKED = {}        # device -> parent stream of a branch forked in this deferred block


def set_branch_parent(dev, stream):
    """The stream a model's branch forked from (None: no branch open)."""
    _PARENT[dev] = stream
    if stream is not None and _DEFER:
        _FORKED[dev] = stream


def _other_stream(dev, cur):
    """The stream besides ``cur`` that produced operands of this deferred
    block: the parent when ``cur`` is the branch, the branch when a branch
    was forked in the block and ``cur`` is its parent; else None.  (A
    branch forked in the block is part of the same capture, so the wait is
    legal inside a HIP graph capture.)"""
    parent = _FORKED.get(dev)
    if parent is None:
        return None
    br = _BRANCH.get(dev)
    if cur == br:
        return parent
    return br


def branch_parent(device):
    """Parent stream while the current stream is the branch, else None."""
    dev = torch.device(device).index
    return _PARENT.get(dev) if on_branch(device) else None


def on_branch(device):
    """True while the current stream of ``device`` is its branch stream."""
    dev = torch.device(device).index
    s = _BRANCH.get(dev)
    return s is not None and torch.cuda.current_stream(dev) == s


def _side(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = torch.cuda.Stream(device=dev)
        _SIDE[dev] = s
    return s


def join_side():
    """Current stream waits for every side-stream launch (no flush)."""
    if not _PENDING:
        return
    cur = torch.cuda.current_stream()
    for dev in list(_PENDING):
        if dev == cur.device.index:
            cur.wait_stream(_SIDE[dev])
            _PENDING.discard(dev)


def join():
    """Launch queued wgrads; current stream waits for every side-stream launch."""
    if _HELD and not _DEFER:
        flush_wgrad()
    join_side()
