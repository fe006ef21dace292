"""Kernel backend selection.

``hip``   — our hand-written CDNA4 kernels (``csrc/hip``, loaded by
            ``ops._hip``); the production path on MI355X.
``torch`` — plain PyTorch implementations of the same ops; the numerical
            oracle in tests and the path on CPU (gloo plumbing tests).

``auto`` picks ``hip`` when a GPU is present.  If ``hip`` is requested on a
GPU and the extension cannot be loaded, it fails loudly: there is no silent
fallback on a GPU box.  Individual ops can be forced to the oracle with
``CEREBRO_TORCH_OPS=conv,bn,...`` (used by A/B tests and bring-up).
"""

import os

import torch

_STATE = {"backend": None}
_FORCED_TORCH = set(filter(None, os.environ.get("CEREBRO_TORCH_OPS", "").split(",")))


def set_backend(name):
    if name == "auto":
        name = "hip" if torch.cuda.is_available() else "torch"
    if name not in ("hip", "torch"):
        raise ValueError(name)
    if name == "hip":
        from . import _hip
        _hip.lib()  # raises if the extension is missing / broken
    _STATE["backend"] = name
    return name


def get_backend():
    if _STATE["backend"] is None:
        set_backend(os.environ.get("CEREBRO_BACKEND", "auto"))
    return _STATE["backend"]


def use_hip(op, *tensors):
    if get_backend() != "hip" or op in _FORCED_TORCH:
        return False
    from . import _hip
    if op not in _hip.IMPLEMENTED:
        return False
    for t in tensors:
        if isinstance(t, torch.Tensor):
            if not t.is_cuda:
                return False
            # activation kernels exist for bf16 (compute mode) and fp32
            # (reference precision, 3-pass split-bf16 MFMA convolutions)
            if t.is_floating_point() and t.dtype not in (torch.bfloat16, torch.float32):
                return False
    return True


# Ops that ran their PyTorch path on a GPU tensor while the HIP backend is
# active (a shape no HIP kernel covers, or an op without one).  The runtime
# captures a training step in a HIP graph only if the step made none: the
# MIOpen-backed torch convolutions / pools are not stream-capture safe on this
# stack (replays diverge from eager; scripts/debug/nasnet_capture.py), while
# elementwise torch glue is.
_FALLBACKS = set()


def hip_gate(op, shape_ok, *tensors):
    """use_hip(op) and the HIP kernel covers this shape; records a fallback
    when the HIP backend is active but the shape is not covered."""
    if not use_hip(op, *tensors):
        return False
    if not shape_ok:
        _FALLBACKS.add(op)
        return False
    return True


def note_fallback(op):
    _FALLBACKS.add(op)


def take_fallbacks():
    """Fallbacks recorded since the last call (and reset)."""
    out = set(_FALLBACKS)
    _FALLBACKS.clear()
    return out


def force_torch_ops(ops):
    _FORCED_TORCH.clear()
    _FORCED_TORCH.update(ops)
