"""ctypes bindings of ``libcerebro_hip.so`` (csrc/hip/*.hip, gfx950).

The library is loaded after torch so it binds to the HIP runtime torch has
already loaded (both carry SONAME libamdhip64.so.7).  Every call launches on
torch's *current* stream, so kernels order with torch ops and are captured by
``torch.cuda.graph``.  A missing / unloadable library raises — there is no
silent fallback on a GPU.

``IMPLEMENTED`` lists the ops with a native path; ``ops.backend.use_hip``
routes only those here.

Every activation op exists in two storage dtypes: the bf16 compute mode and
the reference-precision fp32 mode (entry point suffix ``_f32``; convolutions
run as 3-pass split-bf16 MFMA GEMMs with fp32 accumulation, csrc/hip/conv.hip).
``_fn(name, t)`` picks the entry point matching tensor ``t``'s dtype.
"""

import contextlib
import ctypes
import os

import torch

from . import streams

_LIB = None
_HERE = os.path.dirname(os.path.abspath(__file__))
# CER_HIP_LIB: an A/B twin built by ``tools.build --variant`` (file name in _lib/)
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_lib",
                        os.environ.get("CER_HIP_LIB", "libcerebro_hip.so"))

IMPLEMENTED = {"adam", "loss", "gather"}

# BN partials of a conv epilogue go into STAT_SLABS slabs by exact fp64
# atomics (conv.hip cer_conv_set_stat_slabs), so every BN apply folds its
# finalize (0: one fp32 slab per M tile, plain stores, a separate finalize
# launch for layers with many tiles).  Buffers come zeroed from the step's
# stats arena.  Every BN apply block re-reads the slabs before its rows, one
# memory round trip per slab, so fewer slabs are faster despite the denser
# atomics: 2 vs 8 is +2.2 % at 8 ResNet-50 configs, +5.2 % at one, +3.3 %
# on MobileNetV2 (profiles/r4_bn_slabs.md).
STAT_SLABS = int(os.environ.get("CER_BN_ATOMIC_SLABS", "2"))
SLAB_F64 = 1 << 24     # conv.hip: a returned slab count with this flag is fp64 slabs
_RET_I64 = {"cer_bn_part_floats", "cer_conv_stats_floats", "cer_stem_wpk_elems",
            "cer_bn_bwd_f64_floats"}

c_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i = ctypes.c_int
c_f = ctypes.c_float

_SIGS = {
    "cer_adam_step": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i, c_p, c_i64, c_p,
                      c_p, c_i, c_f, c_f, c_f, c_i, c_p],
    "cer_sgd_step": [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i, c_p, c_i64, c_p, c_p, c_i,
                     c_f, c_i, c_p],
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
            for nm in (name, name + "_f32"):
                if nm != name and not hasattr(L, nm):
                    continue
                fn = getattr(L, nm)
                fn.argtypes = args
                fn.restype = c_i64 if name in _RET_I64 else c_i
        _LIB = L
        if hasattr(L, "cer_conv_set_stat_slabs"):
            L.cer_conv_set_stat_slabs.argtypes = [c_i]
            L.cer_conv_set_stat_slabs(STAT_SLABS)
    return _LIB


def _fn(name, t):
    """Entry point ``name`` for the storage dtype of tensor ``t``."""
    if t.dtype == torch.float32:
        return getattr(lib(), name + "_f32")
    assert t.dtype == torch.bfloat16, t.dtype
    return getattr(lib(), name)


def _stream():
    return c_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return c_p(t.data_ptr()) if t is not None else c_p(0)


def _check(rc, name):
    if rc != 0:
        raise RuntimeError("{} failed with hipError {}".format(name, rc))


# ---------------------------------------------------------------------------
def _opt_hl(arena):
    """The optimizer launch also writes the arena's HL weight image."""
    if arena.whl is not None:
        lib().cer_adam_set_hl(_ptr(arena.whl), arena.whl.stride(0))


def hl_image(src, dst):
    """dst = HL image of the rows of ``src`` (fp32 [G, n], n % 8 == 0)."""
    assert src.dtype == dst.dtype == torch.float32 and src.shape == dst.shape
    rc = lib().cer_hl_image(_ptr(src), src.stride(0), _ptr(dst), dst.stride(0), src.shape[1],
                            src.shape[0], _stream())
    _check(rc, "cer_hl_image")


def adam_step(arena, beta1, beta2, eps, l2):
    L = arena.layout
    st = arena.state
    work = arena.work if arena.work is not arena.params else None
    _opt_hl(arena)
    rc = lib().cer_adam_step(
        _ptr(st), st.stride(0), L.n_train, L.off_m, L.off_v, L.off_step,
        _ptr(arena.grad), arena.grad.stride(0), int(bool(arena.grad_clean)),
        _ptr(work), work.stride(0) if work is not None else 0,
        _ptr(arena.lr), _ptr(arena.wd), arena.G, beta1, beta2, eps, int(bool(l2)), _stream())
    _check(rc, "cer_adam_step")


def sgd_step(arena, momentum, l2):
    L = arena.layout
    st = arena.state
    work = arena.work if arena.work is not arena.params else None
    _opt_hl(arena)
    rc = lib().cer_sgd_step(
        _ptr(st), st.stride(0), L.n_train, L.off_m, L.off_step,
        _ptr(arena.grad), arena.grad.stride(0), int(bool(arena.grad_clean)),
        _ptr(work), work.stride(0) if work is not None else 0,
        _ptr(arena.lr), _ptr(arena.wd), arena.G, float(momentum), int(bool(l2)), _stream())
    _check(rc, "cer_sgd_step")


def softmax_ce_fwd(logits, labels, acc, G, need_grad=True):
    logits = logits.contiguous()
    B, GN = logits.shape
    N = GN // G
    loss = torch.empty(G, dtype=torch.float32, device=logits.device)
    if logits.dtype == torch.float32:
        # reference-precision mode: fp32 dlogits
        d = torch.empty((B, GN), dtype=torch.float32, device=logits.device) if need_grad else None
        rc = lib().cer_softmax_ce_f32(_ptr(logits), _ptr(labels.contiguous()), _ptr(acc),
                                      _ptr(loss), _ptr(d), B, G, N, _stream())
        _check(rc, "cer_softmax_ce_f32")
        return loss, d
    d = torch.empty((B, GN), dtype=torch.bfloat16, device=logits.device) if need_grad else None
    is_bf16 = 1 if logits.dtype == torch.bfloat16 else 0
    if not is_bf16 and logits.dtype != torch.float32:
        logits = logits.float()
    rc = lib().cer_softmax_ce(_ptr(logits), is_bf16, _ptr(labels.contiguous()), _ptr(acc),
                              _ptr(loss), _ptr(d), B, G, N, _stream())
    _check(rc, "cer_softmax_ce")
    return loss, d


def softmax_ce_train(logits, labels, acc, G, head_bias=None):
    """Training-step form (fp32): dlogits + metric accumulators, no loss
    output (its gradient is a unit seed, ops/loss.py); with ``head_bias``
    (the ParamRef of the act-free Dense that made the logits) its bias
    gradient is accumulated here (cer_softmax_ce_f32_head)."""
    logits = logits.contiguous()
    B, GN = logits.shape
    N = GN // G
    d = torch.empty((B, GN), dtype=torch.float32, device=logits.device)
    if head_bias is not None and not head_bias.arena.grad_clean:
        head_bias.grad().zero_()      # the kernel accumulates into it
    gp, gs = head_bias.grad_ptr() if head_bias is not None else (0, 0)
    rc = lib().cer_softmax_ce_f32_head(_ptr(logits), _ptr(labels.contiguous()), _ptr(acc),
                                       _ptr(d), c_p(gp), gs, B, G, N, _stream())
    _check(rc, "cer_softmax_ce_f32_head")
    return d


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
    assert x_out.dtype in (torch.bfloat16, torch.float32) and x_out.is_contiguous()
    P, n, H, W, C = X.shape
    assert C == 3 and perm.shape == (P, n)
    G = part_of_row.shape[0]
    assert x_out.shape == (B, H, W, G * 3)
    mean, inv = _norm(X.device)
    rc = _fn("cer_gather_images", x_out)(_ptr(X), _ptr(Y), _ptr(perm), _ptr(part_of_row), _ptr(cursor),
                                 _ptr(x_out), _ptr(y_out), n, H * W, G, B,
                                 ctypes.cast(mean, c_p), ctypes.cast(inv, c_p), _stream())
    _check(rc, "cer_gather_images")


# ---------------------------------------------------------------------------
# zeroed BN-statistics buffers (atomic slabs)
# ---------------------------------------------------------------------------
class _StatsArena(object):
    """One zeroed fp32 buffer per training working set, handed out in call
    order during a step and zeroed ONCE at the step's start (one fill kernel,
    captured with the step's HIP graph) instead of a fill per layer.  Its
    size settles in the first (eager) step; a buffer it outgrows is kept
    alive (earlier graphs may hold it)."""

    def __init__(self, device):
        self.device = device
        self.buf = None
        self.off = 0
        self.keep = []

    def begin(self):
        self.off = 0
        # eager steps zero here; a captured step relies on the previous
        # step's optimizer launch, which zeroes the arena at its end
        # (runtime/group.py, ops.optim._aux) -- one fill kernel less
        if self.buf is not None and not torch.cuda.is_current_stream_capturing():
            self.buf.zero_()

    def take(self, n):
        n_al = (n + 63) // 64 * 64
        if self.buf is None or self.off + n_al > self.buf.numel():
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("BN stats arena grew during graph capture")
            size = max(self.off + n_al, 2 * (self.buf.numel() if self.buf is not None else 0),
                       1 << 16)
            if self.buf is not None:
                self.keep.append(self.buf)
            self.buf = torch.zeros(size, dtype=torch.float32, device=self.device)
        t = self.buf[self.off:self.off + n]
        self.off += n_al
        return t


_ARENA = [None]


def stats_step(arena):
    """Make ``arena`` (a ``_StatsArena`` or None) the current one and zero it
    (runtime/group.py, at the start of every training step)."""
    _ARENA[0] = arena
    if arena is not None:
        arena.begin()


def new_stats_arena(device):
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:   # "cuda" -> "cuda:<current>": the
        d = torch.device("cuda", torch.cuda.current_device())   # per-launch device check
    return _StatsArena(d)


def _stats_buffer(M, C, device):
    """Zeroed buffer for a conv epilogue's BN partials of an [M, C] output."""
    if STAT_SLABS > 0:          # [slabs][2][C] doubles (conv.hip SLAB_F64)
        n = min(STAT_SLABS, (M + 63) // 64) * 2 * C * 2
    else:
        n = int(lib().cer_conv_stats_floats(M, C))
    a = _ARENA[0]
    if a is None or a.device != torch.device(device) or not STAT_SLABS:
        return torch.zeros(n, dtype=torch.float32, device=device)
    return a.take(n)


# ---------------------------------------------------------------------------
# convolution / linear (csrc/hip/conv.hip)
# ---------------------------------------------------------------------------
_SIGS.update({
    "cer_conv_fwd": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_i, c_i, c_i, c_p,
                     c_i, c_i, c_p, c_i64, c_i, c_p],
    "cer_conv_dgrad": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_p, c_i, c_i, c_i, c_i, c_i,
                       c_p, c_i, c_i, c_p, c_p],
    "cer_conv_wgrad": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i,
                       c_p, c_i64, c_i, c_p],
    "cer_wgrad_splits": [c_i, c_i, c_i, c_i],
    "cer_conv_set_variant": [c_i, c_i],
    "cer_conv_set_addend_grid": [c_i],
    "cer_conv_set_addend_mask": [c_p],
    "cer_bn_set_dres_skip": [c_i],
    "cer_stem_set_wgrad_scratch": [c_p],
    "cer_stem_set_wgrad_zeroed": [c_i],
    "cer_bn_set_bwd_f64": [c_i],
    "cer_bn_bwd_f64_floats": [c_i64, c_i, c_i, c_i],
    "cer_conv_set_splitk": [c_p, c_i64, c_p, c_i],
    "cer_conv_dgrad_bnbwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_i, c_i, c_p],
    "cer_conv_dgrad_babwd": [c_p, c_i64, c_p, c_i, c_p],
    "cer_bn_bwd_part": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p,
                        c_p, c_p, c_p, c_i, c_i64, c_i, c_i, c_i, c_p],
    "cer_wgrad_batch_add": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i,
                            c_p, c_i64],
    "cer_wgrad_batch_flush": [c_i, c_i, c_p],
    "cer_wgrad_batch_set_grid": [c_i],
    "cer_wgrad_batch_set_rows": [c_i],
    "cer_wgrad_batch_set_narrow": [c_i],
    "cer_wgrad_batch_pending": [],
    "cer_bn_set_zmask": [c_i],
    "cer_bn_set_hl_out": [c_i],
    "cer_bn_set_mask_out": [c_p],
    "cer_bn_set_mask_in": [c_i],
    "cer_conv_set_hl": [c_i, c_i],
    "cer_bn_set_fold": [c_i],
    "cer_bn_part_floats": [c_i64, c_i],
    "cer_conv_fwd_stats": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_i, c_i, c_i,
                           c_p, c_i, c_i, c_p, c_p, c_p],
    "cer_conv_stats_floats": [c_i64, c_i],
    "cer_stem_ok": [c_i, c_i, c_i, c_i, c_i],
    "cer_bn_apply_fwd": [c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_i64, c_i, c_i, c_i, c_p],
    "cer_stem_wpk_elems": [c_i, c_i, c_i, c_i, c_i],
    "cer_stem_cp": [c_i],
    "cer_stem_fwd": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_i, c_i, c_i, c_p, c_p,
                     c_p, c_i, c_i, c_p, c_p, c_p, c_i64, c_i, c_p],
    "cer_stem_wgrad": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p,
                       c_p, c_i64, c_p],
    "cer_bn_fwd_train_part": [c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p,
                              c_p, c_p, c_i, c_i64, c_i, c_i, c_f, c_f, c_i, c_p],
    "cer_bn_fwd_train": [c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p,
                         c_p, c_i64, c_i, c_i, c_f, c_f, c_i, c_p],
    "cer_bn_fwd_eval": [c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i, c_i,
                        c_f, c_i, c_p],
    "cer_bn_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p,
                   c_p, c_p,
                   c_i64, c_i, c_i, c_i, c_p],
    "cer_maxpool_fwd": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p],
    "cer_maxpool_bwd_relu_bias": [c_p, c_p, c_p, c_p, c_i64, c_i, c_i, c_i, c_i, c_i, c_i, c_i,
                                  c_i, c_i, c_i, c_p],
    "cer_maxpool_bwd": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p],
    "cer_gavgpool_fwd": [c_p, c_p, c_i, c_i, c_i, c_p],
    "cer_gavgpool_bwd": [c_p, c_p, c_i, c_i, c_i, c_p],
    "cer_bias_act_fwd": [c_p, c_p, c_i64, c_p, c_i64, c_i, c_i, c_i, c_p],
    "cer_bias_act_bwd": [c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_i, c_i, c_i, c_p],
    "cer_softmax_ce_f32": [c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_p],
    "cer_softmax_ce_f32_head": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i, c_i, c_i, c_p],
    "cer_adam_set_aux": [c_p, c_p, c_i64],
    "cer_adam_set_hl": [c_p, c_i64],
    "cer_hl_image": [c_p, c_i64, c_p, c_i64, c_i64, c_i, c_p],
    "cer_conv_set_whl": [c_p, c_i64],
    "cer_conv_set_uk": [c_i],
    "cer_conv_dgrad_bnbwd_f32": None,
})
_SIGS.pop("cer_conv_dgrad_bnbwd_f32")
IMPLEMENTED |= {"conv", "bn", "pool", "bias", "linear"}

_SIGS2 = {
    "cer_dwconv_fwd": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_i, c_i, c_i, c_i,
                       c_p, c_p],
    "cer_dwconv_bwd": [c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_p, c_i64, c_i, c_i, c_i,
                       c_i, c_i, c_i, c_p, c_p],
    "cer_dwconv_fwd_stats": [c_p, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_i, c_i, c_i,
                             c_i, c_p, c_p, c_i, c_p],
    "cer_dwconv_bwd_bn": [c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_p,
                          c_i64, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_i, c_p],
    "cer_avgpool_fwd": [c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p],
    "cer_avgpool_bwd": [c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p],
    "cer_embbag_fwd": [c_p, c_i, c_i, c_i, c_p, c_i64, c_p, c_i64, c_i, c_i, c_p, c_p],
    "cer_embbag_bwd": [c_p, c_p, c_p, c_i, c_i, c_i, c_p, c_i64, c_p, c_i64, c_i, c_i, c_p],
}
_SIGS.update(_SIGS2)
IMPLEMENTED |= {"dwconv", "embbag"}


def _act_code(a):
    if a == 6:
        return 6
    return 1 if a else 0


def _act(t, hl_ok=False):
    """Activation operand: bf16 (compute mode) or fp32 (reference precision).
    An HL-format tensor (``is_hl``) is only handed as-is to the conv entry
    points that read HL (``hl_ok``); anything else gets its fp32 value back
    (hi + lo, what the conv kernels would have used)."""
    assert t.dtype in (torch.bfloat16, torch.float32), t.dtype
    if not hl_ok and is_hl(t):
        return hl_to_fp32(t)
    return t.contiguous()


# ---------------------------------------------------------------------------
# HL operand format (csrc/hip/common.h st8_hl, conv.hip take_hi_lo): an fp32
# tensor whose only consumers are fp32 3-pass conv operand loads is written
# by its producer (the BN apply forward, the BN backward) as
# [8 x bf16 hi | 8 x bf16 lo] per 8 channels -- the exact split the conv
# kernels would compute from the fp32 value, in the same 32 bytes -- so the
# consumer convs skip the split VALU and see bit-identical operands.
# CER_HL=0 turns it off.
# ---------------------------------------------------------------------------
HL_ENABLED = os.environ.get("CER_HL", "1") != "0"
HL_COUNTS = {"x": 0, "dy": 0, "out": 0}     # launches that read / wrote HL (tests, logs)


def is_hl(t):
    return getattr(t, "_cer_hl", False)


def hl_to_fp32(t):
    """fp32 value (hi + lo) of an HL-format tensor."""
    C = t.shape[-1]
    u = t.contiguous().view(torch.int32).view(-1, C // 8, 2, 4)
    hi, lo = u[:, :, 0], u[:, :, 1]

    def unpack(w):                       # 4 words = 8 bf16 -> 8 fp32 (low half first)
        a = (w << 16).view(torch.float32)
        b = (w & -65536).view(torch.float32)
        return torch.stack((a, b), dim=-1).reshape(w.shape[0], w.shape[1], 8)
    return (unpack(hi) + unpack(lo)).reshape(t.shape)


def hl_ok(t, C=None):
    """``t`` (fp32, channels % 8) may be produced in HL format for conv consumers."""
    return (HL_ENABLED and t.dtype == torch.float32 and t.is_cuda
            and (t.shape[-1] if C is None else C) % 8 == 0)


@contextlib.contextmanager
def _hl_operands(x_hl, dy_hl):
    """The next conv launches read x (fwd A / wgrad B) and/or dy (dgrad /
    wgrad A) in HL format (conv.hip cer_conv_set_hl)."""
    x_hl, dy_hl = int(bool(x_hl)), int(bool(dy_hl))
    if not (x_hl or dy_hl):
        yield
        return
    HL_COUNTS["x"] += x_hl
    HL_COUNTS["dy"] += dy_hl
    lib().cer_conv_set_hl(x_hl, dy_hl)
    try:
        yield
    finally:
        lib().cer_conv_set_hl(0, 0)


@contextlib.contextmanager
def _hl_out(on):
    """The next BN apply launches write their output (y / dx) in HL format."""
    if not on:
        yield
        return
    HL_COUNTS["out"] += 1
    lib().cer_bn_set_hl_out(1)
    try:
        yield
    finally:
        lib().cer_bn_set_hl_out(0)


# Residual-join activation masks as bits (bn.hip YM_M): the forward apply of
# a BN with a residual writes its ReLU mask as [M][C / 8] bytes next to y,
# and the backward -- the BN apply / partials and the BN-link statistics in
# the consumer's dgrad epilogue -- reads 1 bit instead of the fp32 y per
# element (fp32, 8-aligned widths).  CER_BN_BITMASK=0 reads y.
BITMASK_ENABLED = os.environ.get("CER_BN_BITMASK", "1") != "0"


def mask_ok(t, act, residual):
    return (BITMASK_ENABLED and residual is not None and act in (1, 6)
            and t.dtype == torch.float32 and t.is_cuda and t.shape[-1] % 8 == 0)


def new_mask(t):
    C = t.shape[-1]
    return torch.empty((t.numel() // C, C // 8), dtype=torch.uint8, device=t.device)


@contextlib.contextmanager
def _mask_out(mask):
    if mask is None:
        yield
        return
    lib().cer_bn_set_mask_out(_ptr(mask))
    try:
        yield
    finally:
        lib().cer_bn_set_mask_out(None)


@contextlib.contextmanager
def mask_in(on):
    """Backward launches inside read residual-join masks as bits (their y
    argument is the mask)."""
    if not on:
        yield
        return
    lib().cer_bn_set_mask_in(1)
    try:
        yield
    finally:
        lib().cer_bn_set_mask_in(0)


def _same(t, ref):
    """Operand that must share ``ref``'s storage dtype."""
    assert t.dtype == ref.dtype, (t.dtype, ref.dtype)
    return t.contiguous()


# Kernel-variant autotuning (the MIOpen "find" step, done by the framework):
# every conv problem is timed once under each of the 12 kernel variants
# ({register-staged, LDS-DMA ring} x {one block per tile, split-K} x
# {64x64, 128x128, 128x64} tiles; split-K applies to fwd / dgrad GEMMs whose
# tile count cannot fill the chip) on its first eager call and the fastest is
# pinned for all later calls, including HIP-graph capture.  CER_CONV_TUNE=0
# keeps the built-in heuristic.
NVARIANTS = 12
SPLITK_FLOATS = 1 << 24      # 64 MB of fp32 split-K partial slots per device
_SPLITK = {}
_TUNED = {}
_TUNE_T = {}     # (op, problem key) -> {variant: best ms over reps} (tune logs)
_PINNED = {}


def _tune_enabled():
    return os.environ.get("CER_CONV_TUNE", "1") != "0"


_LANE = [0]


def set_lane(lane):
    """Concurrency lane of the pack group whose steps run / are captured next
    (runtime/group.py): groups on different lanes replay their graphs at the
    same time on different streams (async_mop._run_batch), so each lane has
    its own split-K workspace."""
    _LANE[0] = int(lane)


def _splitk_ready(device):
    """Register the persistent split-K workspace of this device with the
    library: one for a model's branch stream (ops.streams.branch_stream),
    one for everything else -- kernels of the two may run at once, so each
    has its own partial slots and arrival counters (the pointers are baked
    into captured graphs) -- per concurrency lane (``set_lane``)."""
    key = (str(device), streams.on_branch(device), _LANE[0])
    if _SPLITK.get("_current") == key:
        return
    ws = _SPLITK.get(key)
    if ws is None:
        ws = (torch.empty(SPLITK_FLOATS, dtype=torch.float32, device=device),
              torch.zeros(1 << 16, dtype=torch.int32, device=device))
        _SPLITK[key] = ws
    lib().cer_conv_set_splitk(_ptr(ws[0]), ws[0].numel(), _ptr(ws[1]), ws[1].numel())
    _SPLITK["_current"] = key


# fp32 variants per op: the forward also has the LDS-DMA ring kernels
# (conv.hip pipe_nt32: 3-5, split-K 9-11); dgrad / wgrad register-staged only
# (CER_FP32_RING=0 leaves the ring kernels out of the forward autotune).
# 12-23 are the 32x32x16-MFMA ("wide") twins of ids 0-11 of every op
# (CER_FP32_WIDE=0 leaves them out).
_FWD32 = tuple(range(12)) if os.environ.get("CER_FP32_RING", "1") != "0" else (0, 1, 2, 6, 7, 8)
_REG32 = (0, 1, 2, 6, 7, 8)
FP32_VARIANTS = {0: _FWD32, 1: _REG32, 2: (0, 1, 2)}
if os.environ.get("CER_FP32_WIDE", "1") != "0":
    FP32_VARIANTS = {op: vs + tuple(12 + v for v in vs) for op, vs in FP32_VARIANTS.items()}
# 24-35: intra-block K-split twins (512-thread blocks, two wave groups on the
# halves of the K range; conv.hip group_range) of the register-staged 64x64
# and 128x64 fwd / dgrad kernels, with and without split-K
# (CER_FP32_KSPLIT=0 leaves them out).
_KSPLIT32 = (24, 26, 30, 32)
if os.environ.get("CER_FP32_KSPLIT", "1") != "0":
    FP32_VARIANTS = {op: vs + (_KSPLIT32 if op < 2 else ()) for op, vs in FP32_VARIANTS.items()}
# (ids 36-47, the wave-specialised twins, and the LDS-DMA wgrad ring were
# measured slower -- profiles/r4_ws.md, r5_wgring.md -- and removed in
# round 6; their A/B evidence stays in those profiles and in git history)


def _select(op, key, launch, dtype, after_tune=None):
    """Pin the kernel variant of conv problem ``key`` (tuned once per problem
    and storage dtype)."""
    if op in _PINNED:
        lib().cer_conv_set_variant(op, _PINNED[op])
        return
    key = (str(dtype),) + tuple(key)
    v = _TUNED.get((op, key))
    if v is None:
        v = -1
        if _tune_enabled() and not torch.cuda.is_current_stream_capturing():
            cands = FP32_VARIANTS[op] if dtype == torch.float32 else range(NVARIANTS)
            times = {}
            v = _autotune(op, launch, after=after_tune, variants=cands, times=times)
            _TUNE_T[(op, key)] = times
        _TUNED[(op, key)] = v
    lib().cer_conv_set_variant(op, v)


# interleaved timing passes per variant (4 picked the same kernels as 2:
# r2_ab_kernel_knobs.md)
TUNE_PASSES = 2


def _autotune(op, launch, reps=3, passes=None, after=None, variants=None, times=None):
    """Time every variant (``reps`` back-to-back launches after a warm one)
    over ``passes`` interleaved passes and keep each variant's best pass:
    one noisy measurement no longer pins a slow kernel for the whole run."""
    L = lib()
    if passes is None:
        passes = TUNE_PASSES
    variants = list(range(NVARIANTS) if variants is None else variants)
    best_t = dict.fromkeys(variants)
    for _ in range(max(1, passes)):
        for v in variants:
            L.cer_conv_set_variant(op, v)
            launch()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                launch()
            e.record()
            e.synchronize()
            t = s.elapsed_time(e)
            if best_t[v] is None or t < best_t[v]:
                best_t[v] = t
    best_v = min(variants, key=lambda v: best_t[v])
    if times is not None:
        times.update({v: t / reps for v, t in best_t.items()})
    if after is not None:
        after()
    return best_v


def tuned_variants():
    """{(op, problem key): variant} chosen so far (for logs / profiles)."""
    return dict(_TUNED)


def tune_times():
    """{(op, problem key): {variant: ms per launch}} measured by the autotune."""
    return {k: dict(v) for k, v in _TUNE_T.items()}


def _with_whl(wref, fn):
    """Run ``fn()`` with ``wref``'s HL weight image registered for the fp32
    GEMM it launches (conv.hip cer_conv_set_whl; the uniform-K kernels read
    it instead of splitting the weights; nothing when the arena has none)."""
    h, hs = wref.whl_ptr() if wref is not None else (0, 0)
    if not h:
        return fn()
    L = lib()
    L.cer_conv_set_whl(c_p(h), hs)
    try:
        return fn()
    finally:
        L.cer_conv_set_whl(None, 0)


def _conv_fwd_launch(x, B, H, W, cin, G, wp, ws, cout, kh, kw, stride, pad, y, Ho, Wo, bp, bs,
                     act, wref=None):
    _splitk_ready(x.device)
    def launch():
        rc = _with_whl(wref, lambda: _fn("cer_conv_fwd", x)(
            _ptr(x), B, H, W, cin, G, c_p(wp), ws, cout, kh, kw, stride, pad, _ptr(y), Ho, Wo,
            c_p(bp), bs, _act_code(act), _stream()))
        _check(rc, "cer_conv_fwd")
    _select(0, (B, H, W, cin, cout, kh, kw, stride, pad, G, Ho, Wo), launch, x.dtype)
    launch()


def conv2d_fwd(x, wref, stride, pad, bref=None, act=0):
    """y = act(conv(x, W) + b): bias and activation fused in the GEMM epilogue."""
    x = _act(x)
    B, H, W, GC = x.shape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    assert GC == G * cin, (x.shape, wref.spec.shape, G)
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    if stem_ok(x, wref, stride, pad):
        # narrow-input stem (ResNet's 7x7/2 on RGB in validation, VGG's
        # 3x3/1): the repacked MFMA path instead of the element-gather fallback
        return stem_fwd_stats(x, wref, stride, pad, bref, act, stats=False)[0]
    y = torch.empty((B, Ho, Wo, G * cout), dtype=x.dtype, device=x.device)
    wp, ws = wref.work_ptr()
    bp, bs = bref.work_ptr() if bref is not None else (0, 0)
    _conv_fwd_launch(x, B, H, W, cin, G, wp, ws, cout, kh, kw, stride, pad, y, Ho, Wo, bp, bs, act,
                     wref=wref)
    return y


def conv2d_fwd_stats(x, wref, stride, pad):
    """z = conv(x, W) plus the BN (sum, sum^2) per-slab partials of z, computed
    in the GEMM epilogue.  Returns (z, part, nslab)."""
    x = _act(x)
    B, H, W, GC = x.shape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    assert GC == G * cin, (x.shape, wref.spec.shape, G)
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    z = torch.empty((B, Ho, Wo, G * cout), dtype=x.dtype, device=x.device)
    C = G * cout
    M = B * Ho * Wo
    part = _stats_buffer(M, C, x.device)
    nslab = ctypes.c_int(0)
    wp, ws = wref.work_ptr()
    _splitk_ready(x.device)

    def launch():
        rc = _with_whl(wref, lambda: _fn("cer_conv_fwd_stats", x)(
            _ptr(x), B, H, W, cin, G, c_p(wp), ws, cout, kh, kw, stride, pad, _ptr(z), Ho, Wo,
            _ptr(part), ctypes.byref(nslab), _stream()))
        _check(rc, "cer_conv_fwd_stats")
    # the autotune's timing launches accumulate into the (atomic) slabs
    _select(0, ("stats", B, H, W, cin, cout, kh, kw, stride, pad, G, Ho, Wo), launch, x.dtype,
            after_tune=part.zero_)
    launch()
    return z, part, nslab.value


def _bn_from_part(z, part, nslab, residual, gref, bref, rmref, rvref, act, momentum, eps,
                  hl_out=False):
    mask = new_mask(z) if mask_ok(z, _act_code(act), residual) else None
    y, mean, invstd = bn_act_fwd_train_part(z, residual, gref, bref, rmref, rvref, act, momentum,
                                            eps, part, nslab, hl_out=hl_out, mask=mask)
    if mask is not None:
        y._cer_mask = mask
    return y, z, mean, invstd


def conv_bn_fwd_train(x, wref, gref, bref, rmref, rvref, residual, act, momentum, eps,
                      stride, pad, stem=False, hl_out=False):
    """Fused training unit: conv (+ BN statistics into the fp64 slabs in the
    GEMM epilogue) then one BN-apply pass that folds the finalize.
    Returns (y, z, mean, invstd, x4) — z the conv output (BN input), x4
    the repacked stem input (stem path) or None.  ``x`` may be HL (read as
    such); ``hl_out``: write y in HL format (its only consumer is a conv;
    taken only without a residual and for act none / ReLU, the cases whose
    BN backward never reads y)."""
    x_hl = is_hl(x)
    with _hl_operands(x_hl, 0):
        return _conv_bn_fwd_train(x, wref, gref, bref, rmref, rvref, residual, act, momentum,
                                  eps, stride, pad, stem, x_hl,
                                  hl_out and residual is None and _act_code(act) in (0, 1))


def _conv_bn_fwd_train(x, wref, gref, bref, rmref, rvref, residual, act, momentum, eps,
                       stride, pad, stem, x_hl=False, hl_out=False):
    x = _act(x, hl_ok=x_hl)
    B, H, W, GC = x.shape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    C, M = G * cout, B * Ho * Wo
    dev = x.device
    L = lib()
    _splitk_ready(dev)
    z = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=dev)
    part = _stats_buffer(M, C, dev)
    wp, wstr = wref.work_ptr()
    nslab = ctypes.c_int(0)
    if stem:
        mode = stem_mode(x, wref, stride, pad)
        x4 = torch.empty((G, B, H, W, int(L.cer_stem_cp(mode))), dtype=x.dtype, device=dev)
        wpk = torch.empty(int(L.cer_stem_wpk_elems(G, cout, kh, kw, mode)), dtype=x.dtype,
                          device=dev)
        x4._cer_dwp = _stem_dwp(G, cout, kh, kw, mode, dev)

        def launch():        # conv + BN statistics partials (no running-stat side effects)
            L.cer_stem_set_wgrad_scratch(_ptr(x4._cer_dwp))
            _check(_fn("cer_stem_fwd", x)(_ptr(x), B, H, W, cin, G, c_p(wp), wstr, cout, kh, kw,
                                      stride, pad, _ptr(x4), _ptr(wpk), _ptr(z), Ho, Wo,
                                      _ptr(part), ctypes.byref(nslab), None, 0, 0, _stream()),
                   "cer_stem_fwd")
        _select(0, ("stem", B, H, W, cin, cout, kh, kw, stride, pad, G), launch, x.dtype,
                after_tune=part.zero_)
        launch()
        return _bn_from_part(z, part, nslab.value, residual, gref, bref, rmref, rvref, act,
                             momentum, eps) + (x4,)

    def launch():
        rc = _with_whl(wref, lambda: _fn("cer_conv_fwd_stats", x)(
            _ptr(x), B, H, W, cin, G, c_p(wp), wstr, cout, kh, kw, stride, pad, _ptr(z), Ho, Wo,
            _ptr(part), ctypes.byref(nslab), _stream()))
        _check(rc, "cer_conv_fwd_stats")
    _select(0, ("stats", B, H, W, cin, cout, kh, kw, stride, pad, G, Ho, Wo) + (("hl",) * x_hl),
            launch, x.dtype, after_tune=part.zero_)
    launch()
    return _bn_from_part(z, part, nslab.value, residual, gref, bref, rmref, rvref, act,
                         momentum, eps, hl_out=hl_out and hl_ok(z)) + (None,)


def _stem_dwp(G, cout, kh, kw, mode, device):
    """fp32 split-K scratch of the stem wgrad (packed layout), zeroed by the
    stem forward's prep launch (conv.hip cer_stem_set_wgrad_scratch)."""
    return torch.empty(int(lib().cer_stem_wpk_elems(G, cout, kh, kw, mode)), dtype=torch.float32,
                       device=device)


def stem_mode(x, wref, stride, pad):
    """conv.hip STEM_*: 2 = pixel pairs (Cin <= 4, stride 2), 1 = channels
    padded to 8 (Cin < 8, stride 1), 0 = not a narrow-input stem."""
    cout, kh, kw, cin = wref.spec.shape
    return int(lib().cer_stem_ok(cin, x.shape[2], kw, stride, pad))


def stem_ok(x, wref, stride, pad):
    """Narrow-input first layer eligible for the repacked stem path (cer_stem_fwd)."""
    return stem_mode(x, wref, stride, pad) != 0


def stem_fwd_stats(x, wref, stride, pad, bref=None, act=0, stats=True):
    """Stem conv via the repacked geometry (pixel pairs or 8-channel pixels),
    with BN partials (``stats``) or bias + activation in the epilogue.
    Returns (z, part, nslab, x4) — x4 (the repacked input) feeds the wgrad."""
    x = _act(x)
    B, H, W, GC = x.shape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    mode = stem_mode(x, wref, stride, pad)
    z = torch.empty((B, Ho, Wo, G * cout), dtype=x.dtype, device=x.device)
    L = lib()
    x4 = torch.empty((G, B, H, W, int(L.cer_stem_cp(mode))), dtype=x.dtype, device=x.device)
    wpk = torch.empty(int(L.cer_stem_wpk_elems(G, cout, kh, kw, mode)), dtype=x.dtype,
                      device=x.device)
    part = _stats_buffer(B * Ho * Wo, G * cout, x.device) if stats else None
    nslab = ctypes.c_int(0)
    wp, ws = wref.work_ptr()
    bp, bs = bref.work_ptr() if bref is not None else (0, 0)
    dwp = _stem_dwp(G, cout, kh, kw, mode, x.device) if torch.is_grad_enabled() else None
    if dwp is not None:
        x4._cer_dwp = dwp

    def launch():
        L.cer_stem_set_wgrad_scratch(_ptr(dwp))
        rc = _fn("cer_stem_fwd", x)(_ptr(x), B, H, W, cin, G, c_p(wp), ws, cout, kh, kw, stride, pad,
                                _ptr(x4), _ptr(wpk), _ptr(z), Ho, Wo, _ptr(part),
                                ctypes.byref(nslab), c_p(bp), bs, _act_code(act), _stream())
        _check(rc, "cer_stem_fwd")
    _select(0, ("stem", B, H, W, cin, cout, kh, kw, stride, pad, G, stats, bref is not None,
                _act_code(act)), launch, x.dtype,
            after_tune=part.zero_ if part is not None else None)
    launch()
    return z, part, nslab.value, x4


def stem_wgrad(x4, dy, wref, pad, stride=2):
    dy = _same(dy, x4)
    G, B, H, W, _ = x4.shape
    _, Ho, Wo, _ = dy.shape
    cout, kh, kw, cin = wref.spec.shape
    L = lib()
    mode = int(L.cer_stem_ok(cin, W, kw, stride, pad))
    # the forward's prep launch zeroed this step's scratch (cer_stem_set_wgrad_scratch)
    dwp = getattr(x4, "_cer_dwp", None)
    zeroed = dwp is not None
    if dwp is None:
        dwp = torch.empty(int(L.cer_stem_wpk_elems(G, cout, kh, kw, mode)), dtype=torch.float32,
                          device=dy.device)
    gp, gs = wref.grad_ptr()

    def launch():
        L.cer_stem_set_wgrad_zeroed(int(zeroed))
        rc = _fn("cer_stem_wgrad", x4)(_ptr(x4), B, H, W, cin, G, _ptr(dy), Ho, Wo, cout, kh, kw,
                                  stride, pad, _ptr(dwp), c_p(gp), gs, _stream())
        _check(rc, "cer_stem_wgrad")
    # (the timing launches of a first call accumulate into the scratch: re-zeroed after)
    _select(2, ("stem", B, H, W, cin, cout, kh, kw, stride, pad, G), launch, dy.dtype,
            after_tune=dwp.zero_ if zeroed else None)
    launch()


def _conv_dgrad_launch(dy, B, Ho, Wo, cout, G, wp, ws, cin, kh, kw, stride, pad, dx, H, W,
                       addend=None, bnstats=False, wref=None, after_tune=None, dy_hl=False):
    _splitk_ready(dy.device)
    # transposed-weight scratch only for the unaligned fallback (NN kernel reads W in place)
    n_wt = G * cout * kh * kw * cin if (cout % 8 or cin % 8) else 1
    wt = torch.empty(n_wt, dtype=dy.dtype, device=dy.device)

    def launch(out=dx):
        rc = _with_whl(wref, lambda: _fn("cer_conv_dgrad", dy)(
            _ptr(dy), B, Ho, Wo, cout, G, c_p(wp), ws, _ptr(wt), cin, kh, kw, stride, pad,
            _ptr(out), H, W, _ptr(addend), _stream()))
        _check(rc, "cer_conv_dgrad")
    # an in-place accumulation (dx IS the addend) must not be repeated by the
    # autotune's timing launches: they run in place too, on one scratch copy
    # of the addend made once here (timing the same work as the real launch:
    # a scratch dx != addend would add a full-tensor copy to every timing)
    inplace = addend is not None and addend.data_ptr() == dx.data_ptr()
    tune = launch
    if inplace:
        scratch = [None]

        def tune():
            if scratch[0] is None:
                scratch[0] = addend.clone()
            _check(_with_whl(wref, lambda: _fn("cer_conv_dgrad", dy)(
                _ptr(dy), B, Ho, Wo, cout, G, c_p(wp), ws, _ptr(wt), cin, kh, kw, stride, pad,
                _ptr(scratch[0]), H, W, _ptr(scratch[0]), _stream())), "cer_conv_dgrad")
    _select(1, (B, Ho, Wo, cout, cin, kh, kw, stride, pad, G, H, W, addend is not None, bnstats)
            + (("hl",) * bool(dy_hl)), tune, dy.dtype, after_tune=after_tune)
    launch()


def conv2d_dgrad(dy, wref, xshape, stride, pad, addend=None, bnlink=None, consume_addend=False,
                 balink=None):
    """dx of the conv; ``addend`` (same shape and dtype as dx) is added in the
    GEMM epilogue (the other consumer's gradient of a shared input).
    ``consume_addend=True`` (only ops.nn's GradJoin passes it: it owns the
    addend and uses it nowhere else) lets a strided 1x1 conv accumulate dx
    into the addend's storage; otherwise the addend is never written.
    ``bnlink`` = (link, y): dx is the input gradient of the BatchNorm whose
    output y this conv consumed — the epilogue also computes that BN's
    backward partials into ``link.part`` / ``link.nslab`` (ops.nn.BNLink).
    ``balink`` (ops.nn.BiasActLink): dx is the output gradient of a conv +
    bias + activation layer (its output y is this conv's input); if the
    epilogue can apply it (fp32, aligned, stride 1, no addend) dx comes back
    as dz = act'(y) * dx with the bias gradient accumulated, and
    ``balink.done`` is set.  ``dy`` may be HL (read as such)."""
    dy_hl = is_hl(dy)
    if addend is not None and getattr(addend, "masked_grad", False):
        # a residual gradient never stored: dres = mask * dy (ops.nn.MaskedGrad)
        # joins in the epilogue through the bit mask where the launch can
        # apply it, else it is materialised here
        strided1 = wref.spec.shape[1] == 1 and wref.spec.shape[2] == 1 and pad == 0 and stride > 1
        cout, cin = wref.spec.shape[0], wref.spec.shape[3]
        if (strided1 or cout % 8 or cin % 8 or addend.dy.dtype != torch.float32
                or is_hl(addend.dy) or addend.dy.numel() * 4 >= (1 << 31)):
            addend = addend.materialize()
        else:
            L = lib()
            L.cer_conv_set_addend_mask(_ptr(addend.mask))
            try:
                with _hl_operands(0, dy_hl):
                    return _conv2d_dgrad(_act(dy, hl_ok=dy_hl), wref, xshape, stride, pad,
                                         addend.dy, bnlink, False, dy_hl)
            finally:
                L.cer_conv_set_addend_mask(None)
    with _hl_operands(0, dy_hl):
        if balink is not None and addend is None and bnlink is None:
            return _conv2d_dgrad_balink(_act(dy, hl_ok=dy_hl), wref, xshape, stride, pad, balink,
                                        dy_hl)
        return _conv2d_dgrad(_act(dy, hl_ok=dy_hl), wref, xshape, stride, pad, addend, bnlink,
                             consume_addend, dy_hl)


def _conv2d_dgrad_balink(dy, wref, xshape, stride, pad, balink, dy_hl):
    B, Ho, Wo, _ = dy.shape
    _, H, W, _ = xshape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    wp, ws = wref.work_ptr()
    link, y = balink
    bref = link.bref
    link.done = False
    if y.dtype != torch.float32 or is_hl(y):
        return _conv2d_dgrad(dy, wref, xshape, stride, pad, None, None, False, dy_hl)
    dx = torch.empty((B, H, W, G * cin), dtype=dy.dtype, device=dy.device)
    if not bref.arena.grad_clean:
        bref.grad().zero_()           # the epilogue accumulates into it
    gp, gs = bref.grad_ptr()
    done = ctypes.c_int(0)
    L = lib()
    L.cer_conv_dgrad_babwd(c_p(gp), gs, _ptr(_same(y, dy)), _act_code(link.act),
                           ctypes.byref(done))
    try:
        # the timing launches of the autotune add into the bias gradient too
        _conv_dgrad_launch(dy, B, Ho, Wo, cout, G, wp, ws, cin, kh, kw, stride, pad, dx, H, W,
                           None, bnstats="bias", wref=wref, after_tune=bref.grad().zero_,
                           dy_hl=dy_hl)
    finally:
        L.cer_conv_dgrad_babwd(None, 0, None, 0, None)
    link.done = done.value > 0
    return dx


def _conv2d_dgrad(dy, wref, xshape, stride, pad, addend, bnlink, consume_addend, dy_hl):
    B, Ho, Wo, _ = dy.shape
    _, H, W, _ = xshape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    wp, ws = wref.work_ptr()
    if addend is not None:
        addend = _same(addend, dy)
        assert addend.shape == (B, H, W, G * cin)
    # strided 1x1 dgrad with an addend (the second input gradient of a ResNet
    # stage's first block): accumulate in place into the addend, which is the
    # other consumer's freshly computed dx parked in a GradJoin and used
    # nowhere else -- the kernel then only touches the 1/4 of the pixels it
    # computes, instead of first copying the whole addend into a new dx
    strided1 = kh == 1 and kw == 1 and pad == 0 and stride > 1
    if consume_addend and addend is not None and strided1 and addend.is_contiguous():
        dx = addend
    else:
        dx = torch.empty((B, H, W, G * cin), dtype=dy.dtype, device=dy.device)
    if bnlink is None:
        _conv_dgrad_launch(dy, B, Ho, Wo, cout, G, wp, ws, cin, kh, kw, stride, pad, dx, H, W,
                           addend, wref=wref, dy_hl=dy_hl)
        if strided1 and addend is None:
            # zero off the stride grid: a later strided 1x1 dgrad that adds it
            # can compute a BN link's statistics (conv.hip g_addend_grid)
            dx._cer_grid_st = stride
        return dx
    link, ybn = bnlink
    L = lib()
    M, C = B * H * W, G * cin
    part = _stats_buffer(M, C, dy.device)
    nslab = ctypes.c_int(0)
    gp, gs = link.gref.work_ptr()
    bp, bs = link.bref.work_ptr()
    lmask = getattr(link, "mask", None)
    use_mask = lmask is not None and link.has_res and _act_code(link.act) in (1, 6)
    with mask_in(use_mask):          # the epilogue's mask mode is fixed here
        L.cer_conv_dgrad_bnbwd(_ptr(part), _ptr(link.z),
                               _ptr(lmask) if use_mask else _ptr(_same(ybn, dy)),
                               _ptr(link.mean), _ptr(link.invstd), c_p(gp), gs, c_p(bp), bs,
                               _act_code(link.act), 1 if link.has_res else 0, ctypes.byref(nslab))
    # the addend (the other consumer's parked dx) is zero off this conv's
    # stride grid: the epilogue sees every nonzero pixel, so it can compute
    # the statistics (a ResNet stage transition: c1 and the shortcut)
    grid = (BNLINK_GRID and addend is not None and strided1
            and getattr(addend, "_cer_grid_st", 0) == stride)
    if grid:
        L.cer_conv_set_addend_grid(stride)
    try:
        _conv_dgrad_launch(dy, B, Ho, Wo, cout, G, wp, ws, cin, kh, kw, stride, pad, dx, H, W,
                           addend, bnstats=True, wref=wref, after_tune=part.zero_, dy_hl=dy_hl)
    finally:
        L.cer_conv_dgrad_bnbwd(None, None, None, None, None, None, 0, None, 0, 0, 0, None)
        if grid:
            L.cer_conv_set_addend_grid(0)
    if nslab.value > 0:
        link.part, link.nslab = part, nslab.value
    return dx


def conv_set_variant(op, v):
    """Pin a conv kernel variant (tuning): op 0 fwd / 1 dgrad / 2 wgrad; v -1 = unpin."""
    if v < 0:
        _PINNED.pop(int(op), None)
    else:
        _PINNED[int(op)] = int(v)
    lib().cer_conv_set_variant(int(op), int(v))


def _conv_wgrad_launch(x, B, H, W, cin, G, dy, Ho, Wo, cout, kh, kw, stride, pad, wref,
                       hl=(False, False)):
    gp, gs = wref.grad_ptr()
    if streams.batching():
        splits = _fn("cer_wgrad_batch_add", x)(_ptr(x), B, H, W, cin, G, _ptr(dy), Ho, Wo, cout, kh,
                                           kw, stride, pad, c_p(gp), gs)
        if splits > 0:
            if splits > 1 and not wref.arena.grad_clean:
                wref.grad().zero_()
            streams.hold(x, dy, grad_ptr=gp)
            return

    def launch():
        L = lib()
        splits = L.cer_wgrad_splits(B * Ho * Wo, cout, kh * kw * cin, G)
        if splits > 1 and not wref.arena.grad_clean:
            wref.grad().zero_()
        rc = _fn("cer_conv_wgrad", x)(_ptr(x), B, H, W, cin, G, _ptr(dy), Ho, Wo, cout, kh, kw, stride,
                              pad, c_p(gp), gs, splits, _stream())
        _check(rc, "cer_conv_wgrad")
    # timing runs of split-K variants accumulate into the gradient: clear it
    # before the real launch
    _select(2, (B, H, W, cin, cout, kh, kw, stride, pad, G, Ho, Wo)
            + (("hl", bool(hl[0]), bool(hl[1])),) * any(hl), launch, x.dtype,
            after_tune=lambda: wref.grad().zero_())
    launch()


# ---- grouped convolutions (ResNeXt cardinality; conv.hip cer_conv_grouped_*) ----
_SIGS.update({
    "cer_conv_grouped_fwd": [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_i, c_i,
                             c_i, c_p, c_i, c_i, c_p],
    "cer_conv_grouped_dgrad": [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_i64, c_p, c_i, c_i,
                               c_i, c_i, c_i, c_p, c_i, c_i, c_p],
    "cer_conv_grouped_wgrad": [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i, c_i,
                               c_i, c_i, c_p, c_i64, c_i, c_p],
    "cer_wgrad_batch_add_grouped": [c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_i, c_i, c_i, c_i,
                                    c_i, c_i, c_i, c_p, c_i64],
})


def grouped_ok(wref, groups, stride, pad):
    cout, kh, kw, cin_g = wref.spec.shape
    return (groups >= 1 and cout % groups == 0 and
            not (kh == 1 and kw == 1 and pad == 0 and stride > 1))


def grouped_conv_fwd(x, wref, stride, pad, groups):
    """y of a conv with ``groups`` channel groups inside each packed config;
    weights per config [cout, kh, kw, cin / groups] (ops.nn.PackedGroupedConv2d)."""
    x = _act(x)
    B, H, W, GC = x.shape
    G = wref.G
    cout, kh, kw, cin_g = wref.spec.shape
    cin = cin_g * groups
    assert GC == G * cin, (x.shape, wref.spec.shape, G, groups)
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    y = torch.empty((B, Ho, Wo, G * cout), dtype=x.dtype, device=x.device)
    wp, ws = wref.work_ptr()
    _splitk_ready(x.device)

    def launch():
        _check(_fn("cer_conv_grouped_fwd", x)(_ptr(x), B, H, W, cin, G, groups, c_p(wp), ws, cout,
                                              kh, kw, stride, pad, _ptr(y), Ho, Wo, _stream()),
               "cer_conv_grouped_fwd")
    _select(0, ("grouped", B, H, W, cin, cout, kh, kw, stride, pad, G, groups), launch, x.dtype)
    launch()
    return y


def grouped_conv_dgrad(dy, wref, xshape, stride, pad, groups):
    dy = _act(dy)
    B, Ho, Wo, _ = dy.shape
    _, H, W, _ = xshape
    G = wref.G
    cout, kh, kw, cin_g = wref.spec.shape
    cin = cin_g * groups
    dx = torch.empty((B, H, W, G * cin), dtype=dy.dtype, device=dy.device)
    wp, ws = wref.work_ptr()
    n_wt = cout * kh * kw * cin_g if ((cout // groups) % 8 or cin_g % 8) else 1
    wt = torch.empty(n_wt, dtype=dy.dtype, device=dy.device)
    _splitk_ready(dy.device)

    def launch():
        _check(_fn("cer_conv_grouped_dgrad", dy)(_ptr(dy), B, Ho, Wo, cout, G, groups, c_p(wp), ws,
                                                 _ptr(wt), cin, kh, kw, stride, pad, _ptr(dx), H,
                                                 W, _stream()), "cer_conv_grouped_dgrad")
    _select(1, ("grouped", B, Ho, Wo, cout, cin, kh, kw, stride, pad, G, groups), launch,
            dy.dtype)
    launch()
    return dx


def grouped_conv_wgrad(x, dy, wref, stride, pad, groups):
    x = _act(x)
    dy = _act(dy)
    B, H, W, _ = x.shape
    _, Ho, Wo, _ = dy.shape
    G = wref.G
    cout, kh, kw, cin_g = wref.spec.shape
    cin = cin_g * groups
    gp, gs = wref.grad_ptr()
    if streams.batching():
        splits = _fn("cer_wgrad_batch_add_grouped", x)(_ptr(x), B, H, W, cin, G, groups, _ptr(dy),
                                                       Ho, Wo, cout, kh, kw, stride, pad,
                                                       c_p(gp), gs)
        if splits > 0:
            if splits > 1 and not wref.arena.grad_clean:
                wref.grad().zero_()
            streams.hold(x, dy, grad_ptr=gp)
            return

    def launch():
        splits = lib().cer_wgrad_splits(B * Ho * Wo, cout // groups, kh * kw * cin_g, groups)
        if splits > 1 and not wref.arena.grad_clean:
            wref.grad().zero_()
        _check(_fn("cer_conv_grouped_wgrad", x)(_ptr(x), B, H, W, cin, G, groups, _ptr(dy), Ho,
                                                Wo, cout, kh, kw, stride, pad, c_p(gp), gs,
                                                splits, _stream()), "cer_conv_grouped_wgrad")
    _select(2, ("grouped", B, H, W, cin, cout, kh, kw, stride, pad, G, groups, Ho, Wo), launch,
            x.dtype, after_tune=lambda: wref.grad().zero_())
    launch()


def conv2d_wgrad(x, dy, wref, stride, pad):
    """dW of the conv; ``x`` and / or ``dy`` may be HL (read as such; a
    batched launch captures the format at queue time)."""
    x_hl, dy_hl = is_hl(x), is_hl(dy)
    x = _act(x, hl_ok=x_hl)
    dy = _act(dy, hl_ok=dy_hl)
    B, H, W, _ = x.shape
    _, Ho, Wo, _ = dy.shape
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    with _hl_operands(x_hl, dy_hl):
        _conv_wgrad_launch(x, B, H, W, cin, G, dy, Ho, Wo, cout, kh, kw, stride, pad, wref,
                           hl=(x_hl, dy_hl))


# ---------------------------------------------------------------------------
# batch norm (csrc/hip/bn.hip)
# ---------------------------------------------------------------------------
def _bn_part(M, C, device):
    return torch.empty(int(lib().cer_bn_part_floats(M, C)), dtype=torch.float32, device=device)


def bn_act_fwd_train(x, residual, gref, bref, rmref, rvref, act, momentum, eps):
    x = _act(x)
    C = x.shape[-1]
    M = x.numel() // C
    Cper = gref.spec.shape[0]
    y = torch.empty_like(x)
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    invstd = torch.empty(C, dtype=torch.float32, device=x.device)
    ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    part = _bn_part(M, C, x.device)
    gp, gs = gref.work_ptr()
    bp, bs = bref.work_ptr()
    rmp, rs = rmref.master_ptr()
    rvp, _ = rvref.master_ptr()
    res = _same(residual, x) if residual is not None else None
    rc = _fn("cer_bn_fwd_train", x)(_ptr(x), _ptr(res), _ptr(y), c_p(gp), gs, c_p(bp), bs,
                                c_p(rmp), c_p(rvp), rs, _ptr(mean), _ptr(invstd), _ptr(ws),
                                _ptr(part), M, C, Cper, eps, momentum, _act_code(act), _stream())
    _check(rc, "cer_bn_fwd_train")
    return y, mean, invstd


def bn_act_fwd_train_part(x, residual, gref, bref, rmref, rvref, act, momentum, eps, part,
                          nslab, hl_out=False, mask=None):
    """BN forward from conv-epilogue partials (cer_conv_fwd_stats);
    ``hl_out``: y in HL format (tagged ``_cer_hl``); ``mask``: also write
    the activation mask as bits (``mask_ok`` / ``new_mask``)."""
    x = _act(x)
    C = x.shape[-1]
    M = x.numel() // C
    Cper = gref.spec.shape[0]
    y = torch.empty_like(x)
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    invstd = torch.empty(C, dtype=torch.float32, device=x.device)
    ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    gp, gs = gref.work_ptr()
    bp, bs = bref.work_ptr()
    rmp, rs = rmref.master_ptr()
    rvp, _ = rvref.master_ptr()
    res = _same(residual, x) if residual is not None else None
    with _hl_out(hl_out), _mask_out(mask):
        rc = _fn("cer_bn_fwd_train_part", x)(_ptr(x), _ptr(res), _ptr(y), c_p(gp), gs, c_p(bp),
                                         bs, c_p(rmp), c_p(rvp), rs, _ptr(mean), _ptr(invstd),
                                         _ptr(ws), _ptr(part), int(nslab), M, C, Cper, eps,
                                         momentum, _act_code(act), _stream())
    _check(rc, "cer_bn_fwd_train_part")
    if hl_out:
        y._cer_hl = True
    return y, mean, invstd


def bn_act_fwd_eval(x, residual, gref, bref, rmref, rvref, act, eps):
    x = _act(x)
    C = x.shape[-1]
    M = x.numel() // C
    Cper = gref.spec.shape[0]
    y = torch.empty_like(x)
    gp, gs = gref.work_ptr()
    bp, bs = bref.work_ptr()
    rmp, rs = rmref.master_ptr()
    rvp, _ = rvref.master_ptr()
    res = _same(residual, x) if residual is not None else None
    rc = _fn("cer_bn_fwd_eval", x)(_ptr(x), _ptr(res), _ptr(y), c_p(gp), gs, c_p(bp), bs, c_p(rmp),
                               c_p(rvp), rs, M, C, Cper, eps, _act_code(act), _stream())
    _check(rc, "cer_bn_fwd_eval")
    return y


@contextlib.contextmanager
def _dres_skip(on):
    if not on:
        yield
        return
    L = lib()
    L.cer_bn_set_dres_skip(1)
    try:
        yield
    finally:
        L.cer_bn_set_dres_skip(0)


def dres_skip_ok(x, gref, act, has_res, mask):
    """The residual gradient of this BN backward can stay unwritten (the
    consumer recomputes it as mask * dy, ops.nn.MaskedGrad): fp32, aligned,
    a ReLU residual join whose forward stored its mask as bits."""
    return (has_res and mask is not None and _act_code(act) == 1 and x.dtype == torch.float32
            and x.shape[-1] % 8 == 0 and gref.spec.shape[0] % 8 == 0)


def bn_act_bwd(dy, x, y, mean, invstd, gref, bref, act, has_res, part=None, nslab=0,
               hl_out=False, mask=None, skip_dres=False):
    """BN backward; ``part`` / ``nslab``: the (sum dz, sum dz*xhat) partials
    already computed by the dgrad epilogue that produced dy.  ``hl_out``: dx
    (the conv-output gradient) in HL format for the conv's dgrad / wgrad
    (tagged ``_cer_hl``); the residual gradient stays fp32.  ``mask``: the
    forward's activation bits of a residual join, read instead of y.
    ``skip_dres`` (``dres_skip_ok``): the residual gradient is not written
    (returned as None; bn.hip cer_bn_set_dres_skip)."""
    use_mask = mask is not None and has_res and _act_code(act) in (1, 6)
    if use_mask:
        y = mask
    dy = _act(dy)
    hl_out = hl_out and hl_ok(x)
    C = x.shape[-1]
    M = x.numel() // C
    Cper = gref.spec.shape[0]
    dx = torch.empty_like(x)
    skip_dres = skip_dres and use_mask
    dres = torch.empty_like(x) if has_res and not skip_dres else None
    ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    gp, gs = gref.work_ptr()
    bp, bs = bref.work_ptr()
    dgp, dgs = gref.grad_ptr()
    dbp, _ = bref.grad_ptr()
    if hl_out:
        dx._cer_hl = True
    with _hl_out(hl_out), mask_in(use_mask), _dres_skip(skip_dres):
        if part is not None and nslab > 0:
            rc = _fn("cer_bn_bwd_part", dy)(_ptr(dy), _ptr(x), _ptr(y), _ptr(mean), _ptr(invstd),
                                       c_p(gp), gs, c_p(bp), bs, c_p(dgp), c_p(dbp), dgs,
                                       _ptr(dx), _ptr(dres), _ptr(ws), _ptr(part), int(nslab),
                                       M, C, Cper, _act_code(act), _stream())
            _check(rc, "cer_bn_bwd_part")
            return dx, dres
        # a layer with many row slabs: its partials go into STAT_SLABS fp64
        # slabs of a zeroed buffer (fp64 atomics), so the apply folds the
        # finalize as after a dgrad-epilogue link -- one launch less (+0.2 %
        # at 8 configs, +0.6 % at one: profiles/r5_final.md)
        L = lib()
        nf = int(L.cer_bn_bwd_f64_floats(M, C, Cper, STAT_SLABS)) if STAT_SLABS > 0 else 0
        if nf:
            a = _ARENA[0]
            part = (a.take(nf) if a is not None and torch.device(a.device) == x.device
                    else torch.zeros(nf, dtype=torch.float32, device=x.device))
        else:
            part = _bn_part(M, C, x.device)
        L.cer_bn_set_bwd_f64(STAT_SLABS if nf else 0)
        try:
            rc = _fn("cer_bn_bwd", dy)(_ptr(dy), _ptr(x), _ptr(y), _ptr(mean), _ptr(invstd),
                                  c_p(gp), gs, c_p(bp), bs, c_p(dgp), c_p(dbp), dgs, _ptr(dx),
                                  _ptr(dres), _ptr(ws), _ptr(part), M, C, Cper, _act_code(act),
                                  _stream())
        finally:
            L.cer_bn_set_bwd_f64(0)
    _check(rc, "cer_bn_bwd")
    return dx, dres


# ---------------------------------------------------------------------------
# pooling / bias+act (csrc/hip/pool.hip)
# ---------------------------------------------------------------------------
def maxpool_fwd(x, k, s, p, relu_bit=False):
    """``relu_bit``: also mark in each argmax byte whether the window max is
    > 0 (for maxpool_bwd_relu_bias; C % 8 == 0, k*k <= 128)."""
    x = _act(x)
    B, H, W, C = x.shape
    Ho = (H + 2 * p - k) // s + 1
    Wo = (W + 2 * p - k) // s + 1
    y = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=x.device)
    arg = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device=x.device)
    rc = _fn("cer_maxpool_fwd", x)(_ptr(x), _ptr(y), _ptr(arg), B, H, W, C, Ho, Wo, k, s, p,
                               1 if relu_bit else 0, _stream())
    _check(rc, "cer_maxpool_fwd")
    return y, (arg, k, s, p)


def maxpool_bwd(dy, saved, xshape):
    arg, k, s, p = saved
    B, H, W, C = xshape
    _, Ho, Wo, _ = dy.shape
    dx = torch.empty((B, H, W, C), dtype=dy.dtype, device=dy.device)
    rc = _fn("cer_maxpool_bwd", dy)(_ptr(_act(dy)), _ptr(arg), _ptr(dx), B, H, W, C, Ho, Wo, k, s, p,
                               _stream())
    _check(rc, "cer_maxpool_bwd")
    return dx


def maxpool_relu_bias_ok(x, k, bref, act):
    """The pool's input is a ReLU conv + bias output this pass can finish."""
    return (x.dtype == torch.float32 and x.shape[-1] % 8 == 0 and bref.spec.shape[0] % 8 == 0
            and k * k <= 128 and _act_code(act) == 1 and not is_hl(x))


def maxpool_bwd_relu_bias(dy, saved, xshape, bref):
    """dz of the ReLU conv + bias layer under the pool (its ReLU' applied) and
    that layer's bias gradient, in one pass (pool.hip
    maxpool_bwd_relu_bias_kernel; the forward ran with relu_bit)."""
    arg, k, s, p = saved
    B, H, W, C = xshape
    _, Ho, Wo, _ = dy.shape
    dx = torch.empty((B, H, W, C), dtype=dy.dtype, device=dy.device)
    if not bref.arena.grad_clean:
        bref.grad().zero_()
    gp, gs = bref.grad_ptr()
    rc = _fn("cer_maxpool_bwd_relu_bias", dy)(_ptr(_act(dy)), _ptr(arg), _ptr(dx), c_p(gp), gs,
                                              bref.spec.shape[0], B, H, W, C, Ho, Wo, k, s, p,
                                              _stream())
    _check(rc, "cer_maxpool_bwd_relu_bias")
    return dx


def gavgpool_fwd(x):
    x = _act(x)
    B, H, W, C = x.shape
    y = torch.empty((B, C), dtype=x.dtype, device=x.device)
    rc = _fn("cer_gavgpool_fwd", x)(_ptr(x), _ptr(y), B, H * W, C, _stream())
    _check(rc, "cer_gavgpool_fwd")
    return y


def gavgpool_bwd(dy, xshape):
    B, H, W, C = xshape
    dx = torch.empty(xshape, dtype=dy.dtype, device=dy.device)
    rc = _fn("cer_gavgpool_bwd", dy)(_ptr(_act(dy)), _ptr(dx), B, H * W, C, _stream())
    _check(rc, "cer_gavgpool_bwd")
    return (dx,)


def bias_act_fwd(x, bref, act, out=None):
    x = _act(x)
    C = x.shape[-1]
    M = x.numel() // C
    y = torch.empty_like(x) if out is None else out
    bp, bs = bref.work_ptr()
    rc = _fn("cer_bias_act_fwd", x)(_ptr(x), c_p(bp), bs, _ptr(y), M, C, bref.spec.shape[0],
                                _act_code(act), _stream())
    _check(rc, "cer_bias_act_fwd")
    return y


def bias_act_bwd(dy, y, bref, act):
    dy = _act(dy)
    C = y.shape[-1]
    M = y.numel() // C
    dx = torch.empty_like(dy)
    ws = torch.empty(C, dtype=torch.float32, device=dy.device)
    gp, gs = bref.grad_ptr()
    rc = _fn("cer_bias_act_bwd", dy)(_ptr(dy), _ptr(y), _ptr(dx), c_p(gp), gs, _ptr(ws), M, C,
                                bref.spec.shape[0], _act_code(act), _stream())
    _check(rc, "cer_bias_act_bwd")
    return dx


# ---------------------------------------------------------------------------
# grouped linear = 1x1 conv on a 1x1 image (+ bias/act kernel)
# ---------------------------------------------------------------------------
def linear_fwd(x, wref, bref, act):
    x = _act(x)
    B = x.shape[0]
    G = wref.G
    N, K = wref.spec.shape
    y = torch.empty((B, G * N), dtype=x.dtype, device=x.device)
    wp, ws = wref.work_ptr()
    bp, bs = bref.work_ptr() if bref is not None else (0, 0)
    _conv_fwd_launch(x, B, 1, 1, K, G, wp, ws, N, 1, 1, 1, 0, y, 1, 1, bp, bs, act, wref=wref)
    return y


def linear_bwd(dy, x, y, wref, bref, act, need_dx, bias_done=False):
    """``bias_done``: the bias gradient was accumulated by the loss that
    consumed this act-free head (softmax_ce_train) -- no bias pass."""
    G = wref.G
    N, K = wref.spec.shape
    B = x.shape[0]
    if bref is not None and not (bias_done and not act):
        dz = bias_act_bwd(dy, y, bref, act)
    else:
        dz = _act(dy)
    xb = _act(x)
    _conv_wgrad_launch(xb, B, 1, 1, K, G, dz, 1, 1, N, 1, 1, 1, 0, wref)
    if not need_dx:
        return None
    dx = torch.empty((B, G * K), dtype=dy.dtype, device=dy.device)
    wp, ws = wref.work_ptr()
    _conv_dgrad_launch(dz, B, 1, 1, N, G, wp, ws, K, 1, 1, 1, 0, dx, 1, 1, wref=wref)
    return dx



# ---------------------------------------------------------------------------
# depthwise conv (csrc/hip/dwconv.hip) and embedding bag (csrc/hip/embbag.hip)
# ---------------------------------------------------------------------------
def _pad4(pad):
    """int (symmetric) or (top, bottom, left, right)."""
    if isinstance(pad, int):
        return pad, pad, pad, pad
    return tuple(int(p) for p in pad)


def dw_out_hw(H, W, k, stride, pad):
    pt, pb, pl, pr = _pad4(pad)
    return (H + pt + pb - k) // stride + 1, (W + pl + pr - k) // stride + 1


def dwconv_fwd(x, wref, stride, pad):
    x = _act(x)
    B, H, W, GC = x.shape
    G = wref.G
    C, kh, kw = wref.spec.shape
    Ho, Wo = dw_out_hw(H, W, kh, stride, pad)
    pt, _, pl, _ = _pad4(pad)
    y = torch.empty((B, Ho, Wo, GC), dtype=x.dtype, device=x.device)
    wp, ws = wref.work_ptr()
    rc = _fn("cer_dwconv_fwd", x)(_ptr(x), B, H, W, C, G, c_p(wp), ws, kh, stride, pt, pl, Ho, Wo,
                              _ptr(y), _stream())
    _check(rc, "cer_dwconv_fwd")
    return y


# smallest output (elements) that takes the fused depthwise forward + BN
# statistics.  A sweep (0 / 4M / 16M, profiles/r3_secondary_published.md)
# showed no size at which the plain forward + BN statistics pass wins, so 0.
DW_STATS_MIN = int(os.environ.get("CER_DW_STATS_MIN", "0"))


# a strided 1x1 dgrad whose GradJoin addend is zero off its stride grid (the
# other strided 1x1 consumer's dx) computes the BN link's partials
# (conv.hip g_addend_grid; 0 = the BN runs its own partials pass there)
BNLINK_GRID = os.environ.get("CER_BN_LINK_GRID", "1") != "0"


# stride-2 depthwise dgrads also compute the producing BN's backward partials
DW_BNLINK_S2 = os.environ.get("CER_DW_BNLINK_S2", "1") != "0"


def dwconv_stats_ok(x, wref, stride, pad):
    """The fused 3x3 forward + BN statistics (cer_dwconv_fwd_stats) applies."""
    C, kh, kw = wref.spec.shape
    if not (STAT_SLABS > 0 and kh == 3 and C % 8 == 0 and x.shape[-1] % 8 == 0):
        return False
    Ho, Wo = dw_out_hw(x.shape[1], x.shape[2], kh, stride, pad)
    return x.shape[0] * Ho * Wo * x.shape[-1] >= DW_STATS_MIN


def dwconv_fwd_stats(x, wref, stride, pad):
    """y = dwconv(x) plus the BN (sum, sum^2) partials of y in the conv
    epilogue's fp64 slab format; returns (y, part, nslab) for
    ``bn_act_fwd_train_part`` (the BN then skips its statistics pass)."""
    x = _act(x)
    B, H, W, GC = x.shape
    G = wref.G
    C, kh, kw = wref.spec.shape
    Ho, Wo = dw_out_hw(H, W, kh, stride, pad)
    pt, _, pl, _ = _pad4(pad)
    M = B * Ho * Wo
    y = torch.empty((B, Ho, Wo, GC), dtype=x.dtype, device=x.device)
    part = _stats_buffer(M, GC, x.device)
    nsl = min(STAT_SLABS, (M + 63) // 64)
    wp, ws = wref.work_ptr()
    rc = _fn("cer_dwconv_fwd_stats", x)(_ptr(x), B, H, W, C, G, c_p(wp), ws, kh, stride, pt, pl,
                                    Ho, Wo, _ptr(y), _ptr(part), nsl, _stream())
    _check(rc, "cer_dwconv_fwd_stats")
    return y, part, nsl | SLAB_F64


def dwconv_bwd(dy, x, wref, stride, pad, need_dx, bnlink=None):
    """``bnlink``: the BNLink of the BN that produced ``x`` (its output); when
    usable, dx also yields that BN's backward partials (``link.part``)."""
    dy = _act(dy)
    x = _act(x)
    B, H, W, GC = x.shape
    _, Ho, Wo, _ = dy.shape
    G = wref.G
    C, kh, kw = wref.spec.shape
    pt, _, pl, _ = _pad4(pad)
    if not wref.arena.grad_clean:
        wref.grad().zero_()
    dx = torch.empty_like(x) if need_dx else None
    wp, ws = wref.work_ptr()
    gp, gs = wref.grad_ptr()
    link = bnlink
    if (link is not None and need_dx and (stride == 1 or DW_BNLINK_S2)
            and link.z is not None and link.part is None
            and not link.has_res and _act_code(link.act) in (0, 1, 6) and STAT_SLABS > 0
            and kh == 3 and C % 8 == 0 and link.z.shape == x.shape
            and link.z.dtype == x.dtype):
        M = B * H * W
        part = _stats_buffer(M, GC, x.device)
        nsl = min(STAT_SLABS, (M + 63) // 64)
        rc = _fn("cer_dwconv_bwd_bn", dy)(_ptr(dy), _ptr(x), _ptr(link.z), _ptr(link.mean),
                                      _ptr(link.invstd), _act_code(link.act), B, H, W, C, G,
                                      c_p(wp), ws, c_p(gp), gs, kh, stride, pt, pl, Ho, Wo,
                                      _ptr(dx), _ptr(part), nsl, _stream())
        _check(rc, "cer_dwconv_bwd_bn")
        link.part, link.nslab = part, nsl | SLAB_F64
        return dx
    rc = _fn("cer_dwconv_bwd", dy)(_ptr(dy), _ptr(x), B, H, W, C, G, c_p(wp), ws, c_p(gp), gs, kh,
                              stride, pt, pl, Ho, Wo, _ptr(dx), _stream())
    _check(rc, "cer_dwconv_bwd")
    return dx


def avgpool_fwd(x, k, s, pad, count_pad):
    """k x k / s average pool; pad = int or (top, bottom, left, right) zero
    padding; count_pad: divide by k*k, else by the in-bounds tap count."""
    x = _act(x)
    B, H, W, C = x.shape
    Ho, Wo = dw_out_hw(H, W, k, s, pad)
    pt, _, pl, _ = _pad4(pad)
    y = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=x.device)
    rc = _fn("cer_avgpool_fwd", x)(_ptr(x), _ptr(y), B, H, W, C, Ho, Wo, k, s, pt, pl,
                               int(bool(count_pad)), _stream())
    _check(rc, "cer_avgpool_fwd")
    return y


def avgpool_bwd(dy, xshape, k, s, pad, count_pad):
    dy = _act(dy)
    B, H, W, C = xshape
    _, Ho, Wo, _ = dy.shape
    pt, _, pl, _ = _pad4(pad)
    dx = torch.empty(xshape, dtype=dy.dtype, device=dy.device)
    rc = _fn("cer_avgpool_bwd", dy)(_ptr(dy), _ptr(dx), B, H, W, C, Ho, Wo, k, s, pt, pl,
                               int(bool(count_pad)), _stream())
    _check(rc, "cer_avgpool_bwd")
    return dx


def embbag_fwd(idx, wref, bref, relu):
    G, B, nnz = idx.shape
    K, N = wref.spec.shape
    y = torch.empty((B, G * N), dtype=wref.arena.work.dtype, device=idx.device)
    wp, ws = wref.work_ptr()
    bp, bs = bref.work_ptr()
    rc = _fn("cer_embbag_fwd", y)(_ptr(idx.contiguous()), G, B, nnz, c_p(wp), ws, c_p(bp), bs, N,
                              1 if relu else 0, _ptr(y), _stream())
    _check(rc, "cer_embbag_fwd")
    return y


def embbag_bwd(dy, idx, y, wref, bref, relu):
    G, B, nnz = idx.shape
    K, N = wref.spec.shape
    if not wref.arena.grad_clean:
        wref.grad().zero_()
        bref.grad().zero_()
    gp, gs = wref.grad_ptr()
    bp, bs = bref.grad_ptr()
    rc = _fn("cer_embbag_bwd", dy)(_ptr(_act(dy)), _ptr(y), _ptr(idx.contiguous()), G, B, nnz,
                              c_p(gp), gs, c_p(bp), bs, N, 1 if relu else 0, _stream())
    _check(rc, "cer_embbag_bwd")
