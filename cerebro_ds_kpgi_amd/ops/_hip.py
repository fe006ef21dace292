"""ctypes bindings of ``libcerebro_hip.so`` (csrc/hip/*.hip, gfx950).

The library is loaded after torch so it binds to the HIP runtime torch has
already loaded (both carry SONAME libamdhip64.so.7).  Every call launches on
torch's *current* stream, so kernels order with torch ops and are captured by
``torch.cuda.graph``.  A missing / unloadable library raises — there is no
silent fallback on a GPU.

``IMPLEMENTED`` lists the ops with a native path; ``ops.backend.use_hip``
routes only those here.
"""

import ctypes
import os

import torch

_LIB = None
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_lib", "libcerebro_hip.so")

IMPLEMENTED = {"adam", "loss", "gather"}

c_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i = ctypes.c_int
c_f = ctypes.c_float

_SIGS = {
    "cer_adam_step": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p,
                      c_i, c_f, c_f, c_f, c_i, c_p],
    "cer_softmax_ce": [c_p, c_i, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p],
    "cer_gather_images": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p, c_p, c_p],
}


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("HIP kernel library missing: {} (run __graft_entry__.build())"
                               .format(LIB_PATH))
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = c_i
        _LIB = L
    return _LIB


def _stream():
    return c_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return c_p(t.data_ptr()) if t is not None else c_p(0)


def _check(rc, name):
    if rc != 0:
        raise RuntimeError("{} failed with hipError {}".format(name, rc))


# ---------------------------------------------------------------------------
def adam_step(arena, beta1, beta2, eps, l2):
    L = arena.layout
    st = arena.state
    work = arena.work if arena.work is not arena.params else None
    rc = lib().cer_adam_step(
        _ptr(st), st.stride(0), L.n_train, L.off_m, L.off_v, L.off_step,
        _ptr(arena.grad), arena.grad.stride(0),
        _ptr(work), work.stride(0) if work is not None else 0,
        _ptr(arena.lr), _ptr(arena.wd), arena.G, beta1, beta2, eps, int(bool(l2)), _stream())
    _check(rc, "cer_adam_step")


def softmax_ce_fwd(logits, labels, acc, G, need_grad=True):
    logits = logits.contiguous()
    B, GN = logits.shape
    N = GN // G
    loss = torch.empty(G, dtype=torch.float32, device=logits.device)
    d = torch.empty((B, GN), dtype=torch.bfloat16, device=logits.device) if need_grad else None
    is_bf16 = 1 if logits.dtype == torch.bfloat16 else 0
    if not is_bf16 and logits.dtype != torch.float32:
        logits = logits.float()
    rc = lib().cer_softmax_ce(_ptr(logits), is_bf16, _ptr(labels.contiguous()), _ptr(acc),
                              _ptr(loss), _ptr(d), B, G, N, _stream())
    _check(rc, "cer_softmax_ce")
    return loss, d


_NORM = {}


def _norm(device):
    t = _NORM.get(device)
    if t is None:
        from ..config import catalog as cat
        mean = [m * 255.0 for m in cat.IMAGENET_MEAN]
        inv = [1.0 / (s * 255.0) for s in cat.IMAGENET_STD]
        t = ((ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*inv))
        _NORM[device] = t
    return t


def gather_images(X, Y, perm, part_of_row, cursor, B, x_out, y_out):
    assert x_out.dtype == torch.bfloat16 and x_out.is_contiguous()
    P, n, H, W, C = X.shape
    assert C == 3 and perm.shape == (P, n)
    G = part_of_row.shape[0]
    assert x_out.shape == (B, H, W, G * 3)
    mean, inv = _norm(X.device)
    rc = lib().cer_gather_images(_ptr(X), _ptr(Y), _ptr(perm), _ptr(part_of_row), _ptr(cursor),
                                 _ptr(x_out), _ptr(y_out), n, H * W, G, B,
                                 ctypes.cast(mean, c_p), ctypes.cast(inv, c_p), _stream())
    _check(rc, "cer_gather_images")
