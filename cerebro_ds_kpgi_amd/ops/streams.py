"""Weight-gradient scheduling: batched (deferred) wgrads, optional side stream.

Batched wgrads (default on, ``CER_WGRAD_BATCH=0`` disables): inside
``deferred_wgrad()`` (the engine's training step) a layer's weight-gradient
GEMM is only queued (``cer_wgrad_batch_add``); ``join`` — at the end of the
context and before the optimizer — launches the queue as a few multi-layer
kernels (``wgrad_batch`` in csrc/hip/conv.hip).  The operands stay referenced
here until the flush.  Measured effect in profiles/.

Side stream (``CER_WGRAD_STREAM=1``, default off):

In backward, a layer's input gradient (dgrad) is on the critical path — the
next layer down needs it — while its weight gradient (wgrad) is only needed
by the optimizer at the end of the step.  ``run_side`` launches the wgrad on a
per-device side stream that first waits for everything issued so far on the
current stream (the fork), so the wgrads of layer L overlap the dgrad / BN
backward chain of layers L-1, L-2, ...; ``join`` makes the current stream wait
for the side stream (before the optimizer reads the gradient arena).  Both
are plain stream/event operations, so a captured HIP graph keeps the fork /
join as parallel branches.  Small steps (the one-config-per-GPU case at 8
GPUs) leave most CUs idle during a dgrad; the wgrads fill them.

Split batches (default for packs of >= 4 configs, ``deferred_wgrad(side_frac=
0.5)`` from runtime/group.py): once half of the previous step's layer count
is queued, that batch -- the upper stages' wgrads -- launches ONCE on the
side stream (forked from the current stream at that point) on a capped,
persistent grid (``CER_WGB_SPLIT_GRID`` = 96 blocks), so it runs on a slice
of the CUs while the dgrad / BN-backward chain of the lower stages keeps the
rest; the remaining layers launch at the end on the current stream with the
full grid; ``join`` waits for the side batch before the optimizer.  Measured
(profiles/r2_ab_wgrad_chunk.md): +1.6 % at 8 packed configs, +1.3 % at 4;
one-config packs keep the single batch (a split costs them 3 %), as do more
or smaller side batches and capped tail batches (10-25 % slower).
``CER_WGB_CHUNK=n`` / ``CER_WGB_GRID`` force fixed chunks (A/B only).

Tensors read by a side-stream launch are ``record_stream``-ed so the caching
allocator does not hand their memory to the main stream while the wgrad may
still read it.  ``CER_WGRAD_STREAM=0`` keeps everything on one stream.
"""

import contextlib
import os

import torch

_ON = os.environ.get("CER_WGRAD_STREAM", "0") == "1"
_SIDE = {}
_PENDING = set()

_BATCH = os.environ.get("CER_WGRAD_BATCH", "1") != "0"
_BATCH_VARIANT = int(os.environ.get("CER_WGB_VARIANT", "1"))   # reg 128x128 (A/B in profiles/)
_CHUNK = int(os.environ.get("CER_WGB_CHUNK", "0"))
# blocks of a side-stream wgrad batch (0 = one per work item): a small grid
# walks its tiles persistently on a few CUs, leaving the rest to the dgrad chain
_SIDE_GRID = int(os.environ.get("CER_WGB_GRID", "0"))
# adaptive split (deferred_wgrad(side_frac=f)): the first f of a step's layers
# (by the previous step's count) go to the side stream as one batch on
# SPLIT_GRID blocks; the rest launch at the end as usual
_SPLIT_GRID = int(os.environ.get("CER_WGB_SPLIT_GRID", "96"))
_DEFER = 0
_HELD = []          # operands of queued wgrads (alive until the flush)
_NQ = 0             # layers queued since the last flush
_NSTEP = 0          # layers queued in the current deferred block
_LAST = {}          # ... in the previous block of the same key
_CUR = (0, 0)       # (chunk, grid) in force for the current block
_SPANS = []         # grad pointers of the layers queued since the last flush
_HOOK = None        # deferred_wgrad(hook=...): pre() before / after(ptrs) behind a side batch


def batching():
    """True while wgrads are being queued (inside ``deferred_wgrad``)."""
    return _DEFER > 0


def hold(*tensors, grad_ptr=None):
    """Keep a queued layer's operands alive until its batch is launched; with
    ``CER_WGB_CHUNK`` every n-th layer launches the batch on the side stream.
    ``grad_ptr``: where the layer's gradient lands (handed to the hook)."""
    global _NQ, _NSTEP, _CUR
    _HELD.extend(t for t in tensors if t is not None)
    if grad_ptr is not None:
        _SPANS.append(grad_ptr)
    _NQ += 1
    _NSTEP += 1
    chunk = _CUR[0] if _DEFER else _CHUNK
    if chunk > 0 and _NQ >= chunk and torch.cuda.is_available():
        flush_wgrad(side=True)
        if _DEFER and len(_CUR) > 2:           # adaptive split: one side batch per step
            _CUR = (0, 0)


_ROWS = [None]


def set_batch_rows(rows):
    """Rows of the reduction per split for the next queued fp32/bf16 wgrads
    (0: the library default, CER_WGB_ROWS or 1024)."""
    if _ROWS[0] != rows:
        from . import _hip
        _hip.lib().cer_wgrad_batch_set_rows(int(rows))
        _ROWS[0] = rows


def set_chunk(n, grid=None):
    """Side-stream wgrad batches every ``n`` layers (0: off); ``grid`` caps
    their blocks (None: keep, 0: one block per work item)."""
    global _CHUNK, _SIDE_GRID
    _CHUNK = int(n)
    if grid is not None:
        _SIDE_GRID = int(grid)


def set_batch_variant(v):
    global _BATCH_VARIANT
    _BATCH_VARIANT = int(v)


@contextlib.contextmanager
def deferred_wgrad(enabled=True, side_frac=0.0, key=None, hook=None):
    """Queue HIP weight gradients issued inside the block; flush them on exit.

    ``side_frac`` > 0 (and no ``CER_WGB_CHUNK`` override): once that fraction
    of the previous block's layer count (same ``key``) is queued, the batch so
    far launches ONCE on the side stream on a capped grid
    (``CER_WGB_SPLIT_GRID`` blocks) and overlaps the rest of backward; the
    remaining layers launch at the end as usual, with the full grid
    (profiles/r2_ab_wgrad_chunk.md: +2 % with 8 packed configs, slower with 1;
    a capped grid for the tail batch, or more side batches, lose 10-25 %).

    ``hook`` (adaptive split only): ``hook.pre()`` runs on the current stream
    just before the fork and ``hook.after(grad_ptrs)`` on the side stream right
    behind the side batch (the runtime starts the optimizer update of the
    layers whose gradients are final there, runtime/group.py)."""
    global _DEFER, _CUR, _NSTEP, _HOOK
    on = enabled and _BATCH
    if on:
        if _DEFER == 0:
            if _CHUNK > 0:
                _CUR = (_CHUNK, _SIDE_GRID)
            elif side_frac > 0 and _LAST.get(key, 0) > 1:
                # ONE side batch of the first ceil(frac * n) layers; the rest
                # launches at the end on the current stream with the full grid
                _CUR = (-(-int(round(side_frac * 1000)) * _LAST[key] // 1000), _SPLIT_GRID, 1)
            else:
                _CUR = (0, 0)
            _NSTEP = 0
            _HOOK = hook if len(_CUR) > 2 else None
            del _SPANS[:]
        _DEFER += 1
    try:
        yield
    finally:
        if on:
            _DEFER -= 1
            if _DEFER == 0:
                flush_wgrad()
                _LAST[key] = _NSTEP
                _CUR = (0, 0)
                _HOOK = None


def flush_wgrad(discard=False, side=False, grid=None):
    global _NQ
    if not _HELD:
        return
    from . import _hip
    _NQ = 0
    spans = list(_SPANS)
    del _SPANS[:]
    if side and not discard:
        cur = torch.cuda.current_stream()
        dev = cur.device.index
        st = _side(dev)
        hook = _HOOK if _DEFER else None
        if hook is not None:
            hook.pre()
        st.wait_stream(cur)              # the fork: every queued dy is issued by now
        L = _hip.lib()
        if grid is None:
            grid = _CUR[1] if _DEFER else _SIDE_GRID
        if grid:
            L.cer_wgrad_batch_set_grid(grid)
        try:
            rc = L.cer_wgrad_batch_flush(_BATCH_VARIANT, 0, _hip.c_p(st.cuda_stream))
        finally:
            if grid:
                L.cer_wgrad_batch_set_grid(0)
        if hook is not None:
            with torch.cuda.stream(st):
                hook.after(spans)
        for t in _HELD:
            t.record_stream(st)
        _PENDING.add(dev)
    else:
        rc = _hip.lib().cer_wgrad_batch_flush(_BATCH_VARIANT, 1 if discard else 0, _hip._stream())
    del _HELD[:]
    _hip._check(rc, "cer_wgrad_batch_flush")


def enabled():
    return _ON


def set_enabled(on):
    global _ON
    join()
    _ON = bool(on)


def _side(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = torch.cuda.Stream(device=dev)
        _SIDE[dev] = s
    return s


def run_side(fn, *tensors):
    """Run ``fn`` (kernel launches on the current stream) on the side stream,
    ordered after all work already issued on the current stream."""
    if not _ON:
        return fn()
    cur = torch.cuda.current_stream()
    dev = cur.device.index
    side = _side(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        out = fn()
    for t in tensors:
        if t is not None:
            t.record_stream(side)
    _PENDING.add(dev)
    return out


def join():
    """Launch queued wgrads; current stream waits for every side-stream launch."""
    if _HELD and not _DEFER:
        flush_wgrad()
    if not _PENDING:
        return
    cur = torch.cuda.current_stream()
    for dev in list(_PENDING):
        if dev == cur.device.index:
            cur.wait_stream(_SIDE[dev])
            _PENDING.discard(dev)
