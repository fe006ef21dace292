"""Fused multi-config Adam / SGD over the flat arena.

One launch updates every parameter of all G packed configurations: per-row
learning rate / lambda from device tensors, bias correction from the per-row
step counter (also on device, so the update is CUDA-graph capturable), and the
compute-dtype shadow ``work`` refreshed in the same pass.

Semantics = ``torch.optim.Adam(lr, weight_decay=lambda)`` (the reference's
PyTorch trainer, ``cerebro_gpdb/run_pytorchddp.py:288-292``): coupled L2,
``p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)``.
"""

import torch

from . import streams
from .backend import use_hip

BETA1, BETA2, EPS = 0.9, 0.999, 1e-8


def _aux(cursor, zero):
    """Side jobs of the HIP optimizer launch (adam.hip cer_adam_set_aux):
    advance the data ``cursor`` (int32 device scalar) and zero ``zero`` (an
    fp32 buffer, the step's BN statistics arena) -- two small launches less
    per step.  Returns True when the HIP launch will do them."""
    from . import _hip
    if cursor is None and zero is None:
        return False
    if zero is not None and zero.numel() % 4:
        zero.zero_()        # the kernel zeroes float4s only: clear it here, same stream point
        zero = None
    _hip.lib().cer_adam_set_aux(_hip._ptr(cursor), _hip._ptr(zero),
                                _hip.c_i64(zero.numel() if zero is not None else 0))
    return True


def adam_step(arena, beta1=BETA1, beta2=BETA2, eps=EPS, l2=True, cursor=None, zero=None):
    """``cursor`` / ``zero`` (HIP path only): see ``_aux``; returns True when
    they were handled (else the caller advances the cursor itself)."""
    streams.join()
    if use_hip("adam", arena.state):
        from . import _hip
        done = _aux(cursor, zero)
        _hip.adam_step(arena, beta1, beta2, eps, l2)
        return done
    with torch.no_grad():
        arena.step.add_(1.0)
        t = arena.step                                                 # [G, 1]
        p, g, m, v = arena.params, arena.grad, arena.m, arena.v
        if l2:
            g = g + arena.wd.unsqueeze(1) * p
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        bc1 = 1 - torch.pow(torch.full_like(t, beta1), t)
        bc2 = 1 - torch.pow(torch.full_like(t, beta2), t)
        denom = v.sqrt() / bc2.sqrt() + eps
        p.sub_((arena.lr.unsqueeze(1) / bc1) * m / denom)
        arena.sync_work()
        if arena.grad_clean:
            arena.grad.zero_()
    return False


SGD_MOMENTUM = 0.9


def sgd_step(arena, momentum=SGD_MOMENTUM, l2=True, cursor=None, zero=None):
    """``torch.optim.SGD(lr, momentum, weight_decay=lambda)``; the momentum
    buffer lives in the arena's first-moment slot."""
    streams.join()
    if use_hip("adam", arena.state):
        from . import _hip
        done = _aux(cursor, zero)
        _hip.sgd_step(arena, momentum, l2)
        return done
    with torch.no_grad():
        arena.step.add_(1.0)
        p, g, m = arena.params, arena.grad, arena.m
        if l2:
            g = g + arena.wd.unsqueeze(1) * p
        first = (arena.step <= 1.0).float()                               # [G, 1]
        if momentum:
            m.copy_(first * g + (1 - first) * (momentum * m + g))
            upd = m
        else:
            upd = g
        p.sub_(arena.lr.unsqueeze(1) * upd)
        arena.sync_work()
        if arena.grad_clean:
            arena.grad.zero_()
    return False


def optimizer_step(arena, name="adam", l2=True, cursor=None, zero=None):
    """Returns True when the HIP launch also advanced ``cursor`` / zeroed
    ``zero`` (``_aux``)."""
    streams.join()          # side-stream weight gradients (ops.streams) land first
    if name == "sgd":
        return sgd_step(arena, l2=l2, cursor=cursor, zero=zero)
    return adam_step(arena, l2=l2, cursor=cursor, zero=zero)
