"""Weight-gradient overlap: wgrad kernels on a side HIP stream.

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

Tensors read by a side-stream launch are ``record_stream``-ed so the caching
allocator does not hand their memory to the main stream while the wgrad may
still read it.  ``CER_WGRAD_STREAM=0`` keeps everything on one stream.
"""

import os

import torch

_ON = os.environ.get("CER_WGRAD_STREAM", "0") == "1"
_SIDE = {}
_PENDING = set()


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
    """Current stream waits for every side-stream launch issued so far."""
    if not _PENDING:
        return
    cur = torch.cuda.current_stream()
    for dev in list(_PENDING):
        if dev == cur.device.index:
            cur.wait_stream(_SIDE[dev])
            _PENDING.discard(dev)
