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


def adam_step(arena, beta1=BETA1, beta2=BETA2, eps=EPS, l2=True):
    streams.join()
    if use_hip("adam", arena.state):
        from . import _hip
        _hip.adam_step(arena, beta1, beta2, eps, l2)
        return
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


SGD_MOMENTUM = 0.9


def sgd_step(arena, momentum=SGD_MOMENTUM, l2=True):
    """``torch.optim.SGD(lr, momentum, weight_decay=lambda)``; the momentum
    buffer lives in the arena's first-moment slot."""
    streams.join()
    if use_hip("adam", arena.state):
        from . import _hip
        _hip.sgd_step(arena, momentum, l2)
        return
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


def optimizer_step(arena, name="adam", l2=True):
    streams.join()          # side-stream weight gradients (ops.streams) land first
    if name == "sgd":
        return sgd_step(arena, l2=l2)
    return adam_step(arena, l2=l2)
