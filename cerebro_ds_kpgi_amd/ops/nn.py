"""Packed (horizontally fused) training ops.

Activation layout is **packed NHWC**: ``[B, H, W, G*C]`` — channel block
``g`` belongs to configuration ``g`` of the G configurations trained
together on this GPU.  With that layout

* BatchNorm / ReLU / residual add / pooling over G*C channels are exactly the
  per-config ops (channels are independent), so they need no group logic,
* convolutions and linears are *grouped*: config g's weights only see
  channel block g.

Weights live in the arena (``runtime.arena``), addressed through
``ParamRef``; backward passes write weight gradients straight into the fp32
gradient arena instead of returning them to autograd.

Each op dispatches to our HIP kernel (``ops._hip``) or to the PyTorch oracle
implementation in this file (``ops.backend``).
"""

import os

import torch
import torch.nn.functional as F

from . import streams
from .backend import hip_gate, note_fallback, use_hip


def _hip():
    from . import _hip as h
    return h


def _act(z, code):
    """Activation codes: False/0 = identity, True/1 = ReLU, 6 = ReLU6."""
    if code == 6:
        return torch.clamp(z, 0.0, 6.0)
    if code:
        return torch.relu(z)
    return z


def _act_grad(dz, y, code):
    if code == 6:
        return dz * ((y > 0) & (y < 6))
    if code:
        return dz * (y > 0)
    return dz


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


# ---------------------------------------------------------------------------
# convolution
# ---------------------------------------------------------------------------

def _torch_weight(wref):
    G = wref.G
    cout, kh, kw, cin = wref.spec.shape
    return wref.work().permute(0, 1, 4, 2, 3).reshape(G * cout, cin, kh, kw)


def _conv_forward(x, wref, stride, pad):
    if use_hip("conv", x):
        return _hip().conv2d_fwd(x, wref, stride, pad)
    w = _torch_weight(wref)
    return _nhwc(F.conv2d(_nchw(x), w, None, stride, pad, 1, wref.G))


class GradJoin(object):
    """A tensor read by exactly two of our autograd Functions (a ResNet block
    input: the first conv and the shortcut).  Autograd would add the two input
    gradients in a separate elementwise kernel; instead the consumer whose
    backward runs first parks its gradient here (and returns None to
    autograd), and the second adds it — inside its dgrad GEMM epilogue when it
    is a HIP conv (``conv2d_dgrad(addend=...)``).  Correct in either order,
    and across streams: the two consumers' backwards may run on different
    streams (a ResNet shortcut on the branch stream, ops.streams), so parking
    records an event that the taking stream waits on (``take``)."""
    __slots__ = ("pending", "_ev")

    def __init__(self):
        self.pending = None
        self._ev = None

    def _park(self, g):
        self.pending = g
        self._ev = None
        if g is not None and g.is_cuda:
            self._ev = torch.cuda.Event()
            self._ev.record()

    def take(self):
        """The parked gradient (or None), ordered before the current stream's
        next work; the join is empty afterwards."""
        g, ev = self.pending, self._ev
        self.pending, self._ev = None, None
        if g is not None and ev is not None:
            cur = torch.cuda.current_stream(g.device)
            cur.wait_event(ev)
            g.record_stream(cur)
        return g

    def join(self, g):
        """First arrival: park g, return None.  Second: return the other one."""
        if self.pending is None:
            self._park(g)
            return None
        return self.take()


class MaskedGrad(object):
    """A residual join's gradient dres = mask * dy that was never stored: the
    BN backward of a ReLU(BN(z) + residual) unit skips writing it
    (``bn_act_bwd(skip_dres=True)``) and parks this in the residual's
    GradJoin; the other consumer's dgrad epilogue adds dy where the forward's
    activation bits are set (``conv2d_dgrad``, conv.hip addend_mask).  Saves a
    full-size write and keeps the read the same (dy instead of dres).
    ``materialize()`` is the fallback for any other consumer."""
    __slots__ = ("dy", "mask")
    masked_grad = True

    def __init__(self, dy, mask):
        self.dy, self.mask = dy, mask

    @property
    def is_cuda(self):
        return self.dy.is_cuda

    @property
    def device(self):
        return self.dy.device

    def record_stream(self, s):
        self.dy.record_stream(s)
        self.mask.record_stream(s)

    def materialize(self):
        C = self.dy.shape[-1]
        bits = (self.mask.view(-1, C // 8).unsqueeze(-1) >>
                torch.arange(8, device=self.mask.device, dtype=torch.uint8)) & 1
        return self.dy * bits.view(self.dy.shape).to(self.dy.dtype)


# CER_DRES_LAZY=0: residual gradients are stored by the BN backward as before
DRES_LAZY = os.environ.get("CER_DRES_LAZY", "1") != "0"


def _join_after(join, g):
    """Join a gradient computed without the fused add (torch paths)."""
    if join is None or g is None:
        return g
    other = join.join(g)
    if other is not None and getattr(other, "masked_grad", False):
        other = other.materialize()
    return None if other is None else g + other


class BNLink(object):
    """Forward-time handle from a BatchNorm output to the conv that consumes
    it (``y._cer_bnlink``).  In backward, the consumer's dgrad output IS the
    BN's input gradient dy, so its GEMM epilogue also computes the BN's
    backward partials (``conv2d_dgrad(bnlink=...)``) and the BN backward skips
    its own pass over (dy, z[, y]).  Only set by models on outputs whose whole
    gradient comes out of one dgrad — a sole conv consumer, or two consumers
    joined by a GradJoin (the second arrival holds the full gradient)."""
    __slots__ = ("z", "mean", "invstd", "gref", "bref", "act", "has_res", "part", "nslab",
                 "mask")

    def __init__(self):
        self.z = self.mean = self.invstd = self.gref = self.bref = self.mask = None
        self.act, self.has_res, self.part, self.nslab = 0, False, None, 0


# CER_BIAS_LINKS=0: every conv + bias + activation layer runs its own bias_act_bwd
BIAS_LINKS = os.environ.get("CER_BIAS_LINKS", "1") != "0"


class BiasActLink(object):
    """Forward-time handle from a conv + bias + activation output y to the
    conv that is its SOLE consumer (``y._cer_balink``; VGG's conv -> conv).
    In backward the consumer's dgrad output is y's whole gradient, so its
    epilogue applies act'(y) and accumulates the bias gradient
    (``conv2d_dgrad(balink=...)``, conv.hip YM_BIAS); ``done`` then tells the
    producer's backward to skip its bias_act_bwd pass."""
    __slots__ = ("bref", "act", "done")

    def __init__(self, bref, act):
        self.bref, self.act, self.done = bref, act, False


def _bnlink_for(ctx, x, join, addend):
    """(link, y) when this conv's dx will be the full input gradient of a linked BN."""
    link = getattr(ctx, "bnlink", None)
    if link is None or link.z is None or link.part is not None:
        return None
    if join is not None and addend is None:    # first of two consumers: partial gradient
        return None
    return link, x


class PackedConv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, wref, stride, pad):
        ctx.wref, ctx.stride, ctx.pad = wref, stride, pad
        ctx.join = None
        ctx.bnlink = getattr(x, "_cer_bnlink", None)
        ctx.balink = getattr(x, "_cer_balink", None)
        y = _conv_forward(x, wref, stride, pad)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        return PackedConv2d.backward_core(ctx, x, dy.contiguous(), ctx.needs_input_grad[0])

    @staticmethod
    def backward_core(ctx, x, dy, need_dx):
        wref, stride, pad = ctx.wref, ctx.stride, ctx.pad
        join = getattr(ctx, "join", None) if need_dx else None
        dx = None
        if use_hip("conv", x):
            h = _hip()
            if need_dx:
                # the other consumer's gradient, if it already ran, joins in the epilogue
                addend = join.take() if join is not None else None
                bnl = _bnlink_for(ctx, x, join, addend)
                if addend is not None:
                    join = None
                bal = getattr(ctx, "balink", None) if join is None and addend is None else None
                dx = h.conv2d_dgrad(dy, wref, x.shape, stride, pad, addend=addend, bnlink=bnl,
                                    consume_addend=addend is not None,
                                    balink=None if bal is None else (bal, x))
            # off the critical path: overlaps the dgrad chain below (ops.streams);
            # issued before a park, so the event the other consumer waits on
            # also orders this stream's wgrad (a branch-stream backward launched
            # without batching would otherwise race the optimizer)
            h.conv2d_wgrad(x, dy, wref, stride, pad)
            if need_dx and join is not None:   # first of the two: park dx for the other one
                dx = join.join(dx)
        else:
            G = wref.G
            cout, kh, kw, cin = wref.spec.shape
            w = _torch_weight(wref)
            xn, dyn = _nchw(x), _nchw(dy)
            if need_dx:
                dx = _nhwc(torch.nn.grad.conv2d_input(xn.shape, w, dyn, stride, pad, 1, G))
                dx = _join_after(join, dx)
            dw = torch.nn.grad.conv2d_weight(xn, w.shape, dyn, stride, pad, 1, G)
            wref.grad().copy_(dw.view(G, cout, cin, kh, kw).permute(0, 1, 3, 4, 2))
        return dx, None, None, None, None


def conv2d(x, wref, stride=1, pad=0, anchor=None):
    return PackedConv2d.apply(x, anchor, wref, stride, pad)


class PackedConvBiasAct(torch.autograd.Function):
    """y = act(conv(x) + b) — BN-free conv layers (VGG); bias + activation are
    fused into the HIP GEMM epilogue (one bf16 rounding, no extra pass)."""

    @staticmethod
    def forward(ctx, x, anchor, wref, bref, stride, pad, act, link=None):
        ctx.wref, ctx.bref, ctx.stride, ctx.pad, ctx.act = wref, bref, stride, pad, act
        ctx.join = None
        ctx.bnlink = None
        ctx.balink = getattr(x, "_cer_balink", None)    # x: a linked layer's output
        ctx.link = link                                 # this layer's own output
        ctx.x4 = None
        if use_hip("conv", x) and use_hip("bias", x):
            h = _hip()
            if not x.requires_grad and h.stem_ok(x, wref, stride, pad):
                # narrow first layer (VGG's 3x3/1 on RGB): repacked input, kept for the wgrad
                y, _, _, ctx.x4 = h.stem_fwd_stats(x, wref, stride, pad, bref, act, stats=False)
            else:
                y = h.conv2d_fwd(x, wref, stride, pad, bref, act)
        else:
            w = _torch_weight(wref)
            z = F.conv2d(_nchw(x), w, None, stride, pad, 1, wref.G)
            z = z.float() + bref.work().reshape(1, -1, 1, 1).float()
            y = _nhwc(_act(z, act).to(x.dtype))
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        link = ctx.link
        if link is not None and link.done:
            dz = dy.contiguous()           # act'(y) applied, bias gradient added by the consumer
            link.done = False
        else:
            dz = PackedBiasAct.backward_core(dy.contiguous(), y, ctx.bref, ctx.act)
        if ctx.x4 is not None:
            _hip().stem_wgrad(ctx.x4, dz, ctx.wref, ctx.pad, ctx.stride)
            ctx.x4 = None
            return None, None, None, None, None, None, None, None
        dx, _, _, _, _ = PackedConv2d.backward_core(ctx, x, dz, ctx.needs_input_grad[0])
        return dx, None, None, None, None, None, None, None


def conv2d_bias_act(x, wref, bref, stride=1, pad=0, act=1, anchor=None, link_out=False):
    """``link_out``: the output's only consumer is another conv (its whole
    gradient comes out of that conv's dgrad), which then applies this layer's
    activation derivative and bias gradient in its epilogue (BiasActLink)."""
    link = BiasActLink(bref, act) if link_out and BIAS_LINKS and act in (1, 6) else None
    y = PackedConvBiasAct.apply(x, anchor, wref, bref, stride, pad, act, link)
    if link is not None:
        y._cer_balink = link
    return y


# ---------------------------------------------------------------------------
# batch norm (+ residual add) (+ ReLU)
# ---------------------------------------------------------------------------

def _bn_hip(x, gref):
    """HIP BN kernels: 8 channels per thread when every config's channel count
    is a multiple of 8, one otherwise (ragged widths: NASNet-Mobile's 11 / 22
    / 44 filters) -- every width runs on HIP."""
    return hip_gate("bn", True, x)


def _bn_aligned(gref):
    """8-aligned widths: the conv-epilogue BN statistics and BN links apply."""
    return gref.spec.shape[0] % 8 == 0


def _flat_param(ref):
    return ref.work().reshape(-1).float() if ref.spec.kind in ("gamma", "beta") else ref.master().reshape(-1)


def _bn_forward_train(x, residual, gref, bref, rmref, rvref, relu, momentum, eps):
    C = x.shape[-1]
    part = getattr(x, "_cer_part", None)      # statistics from the producer (dwconv2d stats)
    if part is not None:
        del x._cer_part
    if _bn_hip(x, gref):
        if part is not None and _bn_aligned(gref):
            return _hip().bn_act_fwd_train_part(x, residual, gref, bref, rmref, rvref, relu,
                                                momentum, eps, part[0], part[1])
        return _hip().bn_act_fwd_train(x, residual, gref, bref, rmref, rvref, relu, momentum, eps)
    x2 = x.reshape(-1, C).float()
    n = x2.shape[0]
    mean = x2.mean(0)
    var = x2.var(0, unbiased=False)
    invstd = torch.rsqrt(var + eps)
    with torch.no_grad():
        rm, rv = rmref.master(), rvref.master()
        rm.mul_(1 - momentum).add_(mean.view(rm.shape), alpha=momentum)
        rv.mul_(1 - momentum).add_((var * n / max(n - 1, 1)).view(rv.shape), alpha=momentum)
    gamma = gref.work().reshape(-1).float()
    beta = bref.work().reshape(-1).float()
    z = (x2 - mean) * (invstd * gamma) + beta
    if residual is not None:
        z = z + residual.reshape(-1, C).float()
    z = _act(z, relu)
    return z.to(x.dtype).view(x.shape), mean, invstd


class PackedBNAct(torch.autograd.Function):
    """y = act(BN(x) + residual);  BN statistics per packed channel."""

    @staticmethod
    def forward(ctx, x, residual, gref, bref, rmref, rvref, relu, momentum, eps, link=None):
        ctx.refs = (gref, bref)
        ctx.relu = relu
        ctx.has_res = residual is not None
        y, mean, invstd = _bn_forward_train(x, residual, gref, bref, rmref, rvref, relu, momentum,
                                            eps)
        ctx.link = None
        if link is not None and _bn_hip(x, gref) and _bn_aligned(gref):
            # the consumer conv's dgrad epilogue computes this BN's backward
            # partials (BNLink; e.g. MobileNetV2's depthwise BN -> projection)
            link.z, link.mean, link.invstd = x, mean, invstd
            link.gref, link.bref, link.act, link.has_res = gref, bref, relu, ctx.has_res
            ctx.link = link
        ctx.save_for_backward(x, y, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, invstd = ctx.saved_tensors
        gref, bref = ctx.refs
        link = ctx.link
        if link is not None and link.part is not None:
            dx, dres = _hip().bn_act_bwd(dy.contiguous(), x, y, mean, invstd, gref, bref,
                                         ctx.relu, ctx.has_res, part=link.part, nslab=link.nslab)
        else:
            dx, dres = _bn_backward(ctx, dy.contiguous(), x, y, mean, invstd, gref, bref)
        if link is not None:
            link.z = link.mean = link.invstd = link.part = None
        return dx, dres, None, None, None, None, None, None, None, None


class PackedConvBNAct(torch.autograd.Function):
    """y = act(BN(conv(x)) + residual) in training mode — the ResNet unit.

    HIP path: the convolution's GEMM epilogue also emits the per-channel
    (sum, sum^2) partials of its bf16 output, so BN skips its statistics pass
    over z (finalize + apply only).  Backward = BN backward, then the conv's
    dgrad / wgrad on the BN input gradient.
    """

    @staticmethod
    def forward(ctx, x, residual, anchor, wref, gref, bref, rmref, rvref, stride, pad, relu,
                momentum, eps, join=None, res_join=None, link=None, hl_box=None):
        ctx.wref, ctx.stride, ctx.pad = wref, stride, pad
        ctx.join, ctx.res_join = join, res_join
        ctx.bnlink = getattr(x, "_cer_bnlink", None)     # x is a linked BN's output
        ctx.link = link                                  # this unit's own BN output
        ctx.refs = (gref, bref)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.x4 = None
        hip_ok = (use_hip("conv", x) and use_hip("bn", x) and wref.spec.shape[0] % 8 == 0
                  and gref.spec.shape[0] % 8 == 0)
        ctx.x_hl = False
        ctx.mask = None
        # a branch-stream unit (models/resnet.py shortcut): the stream its
        # block forked from, which consumes its input gradient in backward
        ctx.parent = streams.branch_parent(x.device) if x.is_cuda else None
        if hip_ok:
            h = _hip()
            ctx.x_hl = h.is_hl(x)        # an HL-format input (see conv_bn_act hl_out)
            # narrow first layer: pixel-pair path; its repacked input feeds the wgrad
            stem = not x.requires_grad and h.stem_ok(x, wref, stride, pad)
            y, z, mean, invstd, ctx.x4 = h.conv_bn_fwd_train(
                x, wref, gref, bref, rmref, rvref, residual, relu, momentum, eps, stride, pad,
                stem=stem, hl_out=hl_box is not None and not stem and residual is None)
            # a residual join's activation mask as bits (ops._hip mask_ok)
            ctx.mask = getattr(y, "_cer_mask", None)
            if hl_box is not None:
                hl_box[0] = h.is_hl(y)
        else:
            if getattr(x, "_cer_hl", False):
                x = _hip().hl_to_fp32(x)
            z = _conv_forward(x, wref, stride, pad)
            y, mean, invstd = _bn_forward_train(z, residual, gref, bref, rmref, rvref, relu,
                                                momentum, eps)
        if link is not None and _bn_hip(z, gref) and _bn_aligned(gref):
            link.z, link.mean, link.invstd = z, mean, invstd
            link.gref, link.bref, link.act, link.has_res = gref, bref, relu, ctx.has_res
            link.mask = ctx.mask
        ctx.save_for_backward(x, z, y, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, y, mean, invstd = ctx.saved_tensors
        gref, bref = ctx.refs
        dy = dy.contiguous()
        if ctx.parent is not None:
            # dy was made on the parent stream: keep its memory from being
            # reused there while this stream still reads it
            dy.record_stream(torch.cuda.current_stream(dy.device))
        if ctx.x_hl:
            x._cer_hl = True             # the saved input's format tag
        # the BN input gradient's only consumers are this conv's dgrad and
        # wgrad: HL format when both read it (aligned HIP fp32 path, not the stem)
        wref = ctx.wref
        hl_bwd = (ctx.x4 is None and use_hip("conv", x) and _bn_hip(z, gref)
                  and wref.spec.shape[0] % 8 == 0 and wref.spec.shape[3] % 8 == 0)
        link = ctx.link
        # first arrival at the residual's join: park dres = mask * dy unstored
        lazy = (DRES_LAZY and ctx.res_join is not None and ctx.needs_input_grad[1]
                and ctx.res_join.pending is None and _bn_hip(z, gref)
                and _hip().dres_skip_ok(z, gref, ctx.relu, ctx.has_res, ctx.mask))
        mask = ctx.mask
        if link is not None and link.part is not None:
            # partials from the consumer's dgrad epilogue
            dz, dres = _hip().bn_act_bwd(dy, z, y, mean, invstd, gref, bref, ctx.relu,
                                         ctx.has_res, part=link.part, nslab=link.nslab,
                                         hl_out=hl_bwd, mask=ctx.mask, skip_dres=lazy)
            link.part = None
        else:
            dz, dres = _bn_backward(ctx, dy, z, y, mean, invstd, gref, bref, hl_out=hl_bwd,
                                    mask=ctx.mask, skip_dres=lazy)
        if link is not None:
            link.z = link.mean = link.invstd = link.mask = None
        ctx.mask = None
        if lazy and dres is None:
            ctx.res_join.join(MaskedGrad(dy, mask))
        elif ctx.res_join is not None and ctx.needs_input_grad[1]:
            dres = _join_after(ctx.res_join, dres)
        if ctx.x4 is not None:
            x4, wref, pad = ctx.x4, ctx.wref, ctx.pad
            _hip().stem_wgrad(x4, dz, wref, pad, ctx.stride)
            ctx.x4 = None
            dx = None
        else:
            dx, _, _, _, _ = PackedConv2d.backward_core(ctx, x, dz, ctx.needs_input_grad[0])
        if ctx.parent is not None and dx is not None:
            dx.record_stream(ctx.parent)      # consumed on the parent stream
        return (dx, dres, None, None, None, None, None, None, None, None, None, None, None, None,
                None, None, None)


def _bn_backward(ctx, dy, x, y, mean, invstd, gref, bref, hl_out=False, mask=None,
                 skip_dres=False):
    if _bn_hip(x, gref):
        return _hip().bn_act_bwd(dy, x, y, mean, invstd, gref, bref, ctx.relu, ctx.has_res,
                                 hl_out=hl_out, mask=mask, skip_dres=skip_dres)
    C = x.shape[-1]
    dz = _act_grad(dy.reshape(-1, C).float(), y.reshape(-1, C), ctx.relu)
    n = dz.shape[0]
    xhat = (x.reshape(-1, C).float() - mean) * invstd
    dbeta = dz.sum(0)
    dgamma = (dz * xhat).sum(0)
    gamma = gref.work().reshape(-1).float()
    dx = (gamma * invstd / n) * (n * dz - dbeta - xhat * dgamma)
    dx = dx.to(x.dtype).view(x.shape)
    gref.grad().copy_(dgamma.view(gref.grad().shape))
    bref.grad().copy_(dbeta.view(bref.grad().shape))
    dres = dz.to(x.dtype).view(x.shape) if ctx.has_res else None
    return dx, dres


def conv_bn_act(x, wref, gref, bref, rmref, rvref, stride=1, pad=0, relu=True, residual=None,
                momentum=0.1, eps=1e-5, anchor=None, join=None, res_join=None, link_out=False,
                hl_out=False):
    """``join``: GradJoin shared with the other consumer of ``x``;
    ``res_join``: GradJoin shared with the other consumer of ``residual``;
    ``link_out``: the output's whole gradient comes out of one consumer dgrad
    (see BNLink) — its BN backward partials are computed there;
    ``hl_out``: the output's ONLY consumer is another conv_bn_act (HIP fp32):
    it is written in HL format (``_hip.is_hl``: the pre-split operand of the
    consumer's 3-pass kernels, bit-identical operands, no split VALU there).
    (Folding the BN apply into the consumer conv's operand loads was measured
    slower at 1, 2 and 8 configs and removed: profiles/r3_resnet50_1cfg_fp32.md.)"""
    link = BNLink() if link_out else None
    box = [False] if hl_out else None
    y = PackedConvBNAct.apply(x, residual, anchor, wref, gref, bref, rmref, rvref, stride, pad,
                              relu, momentum, eps, join, res_join, link, box)
    if link is not None:
        y._cer_bnlink = link
    if box is not None and box[0]:
        y._cer_hl = True
    return y


def bn_act_eval(x, residual, gref, bref, rmref, rvref, relu, eps):
    C = x.shape[-1]
    if _bn_hip(x, gref):
        return _hip().bn_act_fwd_eval(x, residual, gref, bref, rmref, rvref, relu, eps)
    rm = rmref.master().reshape(-1)
    rv = rvref.master().reshape(-1)
    scale = gref.work().reshape(-1).float() * torch.rsqrt(rv + eps)
    shift = bref.work().reshape(-1).float() - rm * scale
    z = x.reshape(-1, C).float() * scale + shift
    if residual is not None:
        z = z + residual.reshape(-1, C).float()
    return _act(z, relu).to(x.dtype).view(x.shape)


def bn_act(x, gref, bref, rmref, rvref, training, relu=True, residual=None,
           momentum=0.1, eps=1e-5, link_out=False):
    """``link_out`` (training): the output's whole gradient comes out of one
    consumer conv's dgrad (see BNLink), which computes the BN backward partials."""
    if training:
        link = BNLink() if link_out else None
        y = PackedBNAct.apply(x, residual, gref, bref, rmref, rvref, relu, momentum, eps, link)
        if link is not None:
            y._cer_bnlink = link
        return y
    return bn_act_eval(x, residual, gref, bref, rmref, rvref, relu, eps)


# ---------------------------------------------------------------------------
# bias + activation (conv nets without BN, e.g. VGG)
# ---------------------------------------------------------------------------

class PackedBiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bref, relu):
        C = x.shape[-1]
        ctx.bref, ctx.relu = bref, relu
        if use_hip("bias", x):
            y = _hip().bias_act_fwd(x, bref, relu)
        else:
            z = x.reshape(-1, C).float() + bref.work().reshape(-1).float()
            if relu:
                z = torch.relu(z)
            y = z.to(x.dtype).view(x.shape)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, = ctx.saved_tensors
        return PackedBiasAct.backward_core(dy.contiguous(), y, ctx.bref, ctx.relu), None, None

    @staticmethod
    def backward_core(dy, y, bref, act):
        """dz = act'(y) * dy; dbias = sum_rows dz written into the arena."""
        if use_hip("bias", y):
            return _hip().bias_act_bwd(dy, y, bref, act)
        C = y.shape[-1]
        dz = _act_grad(dy.reshape(-1, C).float(), y.reshape(-1, C), act)
        bref.grad().copy_(dz.sum(0).view(bref.grad().shape))
        return dz.to(dy.dtype).view(dy.shape)


def bias_act(x, bref, relu=True):
    return PackedBiasAct.apply(x, bref, relu)


# ---------------------------------------------------------------------------
# pooling
# ---------------------------------------------------------------------------

class MaxPoolHip(torch.autograd.Function):
    """``x`` may be a linked conv + bias + ReLU output (BiasActLink, set by
    the model when the pool is its sole consumer): the backward then returns
    that layer's dz (ReLU' applied) and writes its bias gradient in the same
    pass (pool.hip maxpool_bwd_relu_bias_kernel)."""

    @staticmethod
    def forward(ctx, x, k, s, p):
        link = getattr(x, "_cer_balink", None)
        h = _hip()
        if link is not None and not h.maxpool_relu_bias_ok(x, k, link.bref, link.act):
            link = None
        ctx.link = link
        y, saved = h.maxpool_fwd(x, k, s, p, relu_bit=link is not None)
        ctx.save_for_backward(saved[0])
        ctx.geom = saved[1:]
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        arg, = ctx.saved_tensors
        link = ctx.link
        if link is not None:
            dx = _hip().maxpool_bwd_relu_bias(dy.contiguous(), (arg,) + ctx.geom, ctx.xshape,
                                              link.bref)
            link.done = True
        else:
            dx = _hip().maxpool_bwd(dy.contiguous(), (arg,) + ctx.geom, ctx.xshape)
        return dx, None, None, None


def maxpool2d(x, k, s, p=0):
    if hip_gate("pool", True, x):
        return MaxPoolHip.apply(x, k, s, p)
    return _nhwc(F.max_pool2d(_nchw(x), k, s, p))


class GlobalAvgPoolHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.xshape = x.shape
        return _hip().gavgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _hip().gavgpool_bwd(dy.contiguous(), ctx.xshape)[0]


def global_avgpool(x):
    """[B, H, W, C] -> [B, C]."""
    if hip_gate("pool", True, x):
        return GlobalAvgPoolHip.apply(x)
    return x.float().mean(dim=(1, 2)).to(x.dtype)


# ---------------------------------------------------------------------------
# grouped linear (+bias) (+relu)
# ---------------------------------------------------------------------------

class PackedLinear(torch.autograd.Function):
    """x [B, G*K] -> y [B, G*N];  config g: y_g = act(x_g W_g^T + b_g)."""

    @staticmethod
    def forward(ctx, x, anchor, wref, bref, relu):
        ctx.wref, ctx.bref, ctx.relu = wref, bref, relu
        # set by a loss that accumulated this layer's bias gradient itself
        # (ops.loss.softmax_ce(head=y._cer_head))
        ctx.head_box = [False]
        G = wref.G
        N, K = wref.spec.shape
        B = x.shape[0]
        if use_hip("linear", x):
            y = _hip().linear_fwd(x, wref, bref, relu)
            if bref is not None and not relu:
                y._cer_head = (bref, ctx.head_box)
        else:
            xg = x.view(B, G, K).transpose(0, 1)                       # [G, B, K]
            w = wref.work()                                             # [G, N, K]
            z = torch.bmm(xg.float(), w.float().transpose(1, 2))        # [G, B, N]
            if bref is not None:
                z = z + bref.work().float().unsqueeze(1)
            if relu:
                z = torch.relu(z)
            y = z.transpose(0, 1).reshape(B, G * N).to(x.dtype)
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        wref, bref, relu = ctx.wref, ctx.bref, ctx.relu
        dy = dy.contiguous()
        if use_hip("linear", x):
            dx = _hip().linear_bwd(dy, x, y, wref, bref, relu, ctx.needs_input_grad[0],
                                   bias_done=ctx.head_box[0])
            return dx, None, None, None, None
        G = wref.G
        N, K = wref.spec.shape
        B = x.shape[0]
        dz = dy.view(B, G, N).float()
        if relu:
            dz = dz * (y.view(B, G, N) > 0)
        dzg = dz.transpose(0, 1)                                        # [G, B, N]
        xg = x.view(B, G, K).transpose(0, 1).float()                    # [G, B, K]
        wref.grad().copy_(torch.bmm(dzg.transpose(1, 2), xg))           # [G, N, K]
        if bref is not None:
            bref.grad().copy_(dzg.sum(1))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.bmm(dzg, wref.work().float())                    # [G, B, K]
            dx = dx.transpose(0, 1).reshape(B, G * K).to(x.dtype)
        return dx, None, None, None, None


def linear(x, wref, bref=None, relu=False, anchor=None):
    return PackedLinear.apply(x, anchor, wref, bref, relu)


# ---------------------------------------------------------------------------
# sparse-input first layer (Criteo confA): embedding-bag over one-hot indices
# ---------------------------------------------------------------------------

class PackedEmbeddingBag(torch.autograd.Function):
    """One-hot input with ``nnz`` active columns per row == sum of W columns.

    idx [G, B, nnz] int32 (column ids into the K-wide input; -1 = padding for
    rows with fewer active features), W_g [N, K]:
    y[b, g*N:(g+1)*N] = act(sum_j W_g[idx[g,b,j], :] + b_g).
    Weight layout is [K, N] (input-major), which is the Keras ``Dense``
    kernel layout, so the flat checkpoint blob matches a Dense(7306 -> N)
    layer and each active input column is one contiguous N-row to gather.
    """

    @staticmethod
    def forward(ctx, idx, anchor, wref, bref, relu):
        ctx.wref, ctx.bref, ctx.relu = wref, bref, relu
        G = wref.G
        K, N = wref.spec.shape
        Gi, B, nnz = idx.shape
        ctx.hip = hip_gate("embbag", N % 8 == 0, idx)
        if ctx.hip:
            y = _hip().embbag_fwd(idx, wref, bref, relu)
        else:
            w = wref.work().float()                                     # [G, K, N]
            valid = (idx >= 0).unsqueeze(-1).float()                    # -1 = padding
            rows = torch.stack([w[g][idx[g].long().clamp(min=0)] for g in range(G)])
            z = (rows * valid).sum(2) + bref.work().float().unsqueeze(1)
            if relu:
                z = torch.relu(z)
            y = z.transpose(0, 1).reshape(B, G * N).to(wref.arena.compute_dtype)
        ctx.save_for_backward(idx, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, y = ctx.saved_tensors
        wref, bref, relu = ctx.wref, ctx.bref, ctx.relu
        dy = dy.contiguous()
        if ctx.hip:
            _hip().embbag_bwd(dy, idx, y, wref, bref, relu)
            return None, None, None, None, None
        G = wref.G
        K, N = wref.spec.shape
        B = dy.shape[0]
        dz = dy.view(B, G, N).float()
        if relu:
            dz = dz * (y.view(B, G, N) > 0)
        dzg = dz.transpose(0, 1)                                        # [G, B, N]
        gw = wref.grad()
        gw.zero_()
        for g in range(G):
            flat = idx[g].long().reshape(-1)
            keep = flat >= 0                                            # -1 = padding
            gw[g].index_add_(0, flat[keep], dzg[g].repeat_interleave(idx.shape[2], 0)[keep])
        bref.grad().copy_(dzg.sum(1))
        return None, None, None, None, None


def embedding_bag(idx, wref, bref, relu=True, anchor=None):
    return PackedEmbeddingBag.apply(idx, anchor, wref, bref, relu)


# ---------------------------------------------------------------------------
# depthwise conv (MobileNetV2) — packed channels, one filter per channel
# ---------------------------------------------------------------------------

def _pad4(pad):
    if isinstance(pad, int):
        return pad, pad, pad, pad
    return tuple(int(p) for p in pad)


def _zero_pad(x, pad):
    """Explicit zero padding of packed NHWC; pad = (top, bottom, left, right)."""
    pt, pb, pl, pr = pad
    return F.pad(x, (0, 0, pl, pr, pt, pb))


# CER_DW_STATS=0: the BN after a depthwise conv computes its own statistics
_DW_STATS = os.environ.get("CER_DW_STATS", "1") != "0"
# CER_DW_BNLINK=0: the BN before a depthwise conv runs its own backward pass
_DW_BNLINK = os.environ.get("CER_DW_BNLINK", "1") != "0"


class PackedDWConv2d(torch.autograd.Function):
    """Depthwise k x k conv (k in {3, 5, 7}), stride 1/2; ``pad`` is an int or
    (top, bottom, left, right) — Keras stride-2 ``correct_pad`` is asymmetric."""

    @staticmethod
    def forward(ctx, x, anchor, wref, stride, pad, stats=False):
        ctx.wref, ctx.stride, ctx.pad = wref, stride, pad
        # x is a linked BN's output: dgrad computes that BN's backward partials
        ctx.bnlink = getattr(x, "_cer_bnlink", None) if _DW_BNLINK else None
        C, kh, kw = wref.spec.shape
        ctx.hip = hip_gate("dwconv", kh == kw and kh in (3, 5, 7)
                           and stride in (1, 2) and max(_pad4(pad)) < kh, x)
        if ctx.hip and stats and _DW_STATS and _hip().dwconv_stats_ok(x, wref, stride, pad):
            # BN (sum, sum^2) partials of y for the BN that consumes it
            # (_bn_forward_train takes them instead of a statistics pass)
            y, part, nslab = _hip().dwconv_fwd_stats(x, wref, stride, pad)
            y._cer_part = (part, nslab)
        elif ctx.hip:
            y = _hip().dwconv_fwd(x, wref, stride, pad)
        else:
            w = wref.work().reshape(wref.G * C, 1, kh, kw)
            y = _nhwc(F.conv2d(_nchw(_zero_pad(x, _pad4(pad))), w, None, stride, 0, 1,
                               wref.G * C))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        wref, stride, pad = ctx.wref, ctx.stride, ctx.pad
        dy = dy.contiguous()
        if ctx.hip:
            dx = _hip().dwconv_bwd(dy, x, wref, stride, pad, ctx.needs_input_grad[0],
                                   bnlink=ctx.bnlink)
            return dx, None, None, None, None, None
        C, kh, kw = wref.spec.shape
        GC = wref.G * C
        w = wref.work().reshape(GC, 1, kh, kw)
        pt, pb, pl, pr = _pad4(pad)
        xp = _nchw(_zero_pad(x, (pt, pb, pl, pr)))
        dyn = _nchw(dy)
        dx = None
        if ctx.needs_input_grad[0]:
            dxp = torch.nn.grad.conv2d_input(xp.shape, w, dyn, stride, 0, 1, GC)
            dx = _nhwc(dxp[:, :, pt:pt + x.shape[1], pl:pl + x.shape[2]])
        dw = torch.nn.grad.conv2d_weight(xp, w.shape, dyn, stride, 0, 1, GC)
        wref.grad().copy_(dw.view(wref.G, C, kh, kw))
        return dx, None, None, None, None, None


def dwconv2d(x, wref, stride=1, pad=1, anchor=None, stats=False):
    """``stats``: the output's consumer is a training-mode BN (``bn_act``);
    the HIP 3x3 path then also emits its batch statistics."""
    return PackedDWConv2d.apply(x, anchor, wref, stride, pad, stats)


# ---------------------------------------------------------------------------
# grouped convolution inside each configuration (ResNeXt cardinality; HIP),
# average pooling and per-config channel concat (DenseNet)
# ---------------------------------------------------------------------------

class PackedGroupedConv2d(torch.autograd.Function):
    """conv with ``groups`` channel groups per configuration.

    W_g [cout, kh, kw, cin / groups].  HIP: the packed implicit-GEMM kernels
    run once per config over its ``groups`` sub-configs (conv.hip
    ``cer_conv_grouped_*``; weight gradients join the deferred batch).
    PyTorch oracle: one torch grouped conv with G * groups groups.
    """

    @staticmethod
    def forward(ctx, x, anchor, wref, stride, pad, groups):
        ctx.wref, ctx.stride, ctx.pad, ctx.groups = wref, stride, pad, groups
        ctx.hip = use_hip("conv", x) and _hip().grouped_ok(wref, groups, stride, pad)
        if ctx.hip:
            y = _hip().grouped_conv_fwd(x, wref, stride, pad, groups)
        else:
            if use_hip("conv", x):
                note_fallback("grouped_conv")
            w = _torch_weight(wref)
            y = _nhwc(F.conv2d(_nchw(x), w, None, stride, pad, 1, wref.G * groups))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        wref, stride, pad, groups = ctx.wref, ctx.stride, ctx.pad, ctx.groups
        dy = dy.contiguous()
        dx = None
        if ctx.hip:
            h = _hip()
            if ctx.needs_input_grad[0]:
                dx = h.grouped_conv_dgrad(dy, wref, x.shape, stride, pad, groups)
            h.grouped_conv_wgrad(x, dy, wref, stride, pad, groups)
            return dx, None, None, None, None, None
        G = wref.G
        cout, kh, kw, cin_g = wref.spec.shape
        w = _torch_weight(wref)
        xn, dyn = _nchw(x), _nchw(dy)
        if ctx.needs_input_grad[0]:
            dx = _nhwc(torch.nn.grad.conv2d_input(xn.shape, w, dyn, stride, pad, 1, G * groups))
        dw = torch.nn.grad.conv2d_weight(xn, w.shape, dyn, stride, pad, 1, G * groups)
        wref.grad().copy_(dw.view(G, cout, cin_g, kh, kw).permute(0, 1, 3, 4, 2))
        return dx, None, None, None, None, None


def grouped_conv2d(x, wref, stride=1, pad=0, groups=1, anchor=None):
    if groups == 1:
        return conv2d(x, wref, stride, pad, anchor)
    return PackedGroupedConv2d.apply(x, anchor, wref, stride, pad, groups)


class AvgPoolHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, count_pad):
        ctx.geom = (x.shape, k, s, p, count_pad)
        return _hip().avgpool_fwd(x, k, s, p, count_pad)

    @staticmethod
    def backward(ctx, dy):
        xshape, k, s, p, count_pad = ctx.geom
        dx = _hip().avgpool_bwd(dy.contiguous(), xshape, k, s, p, count_pad)
        return dx, None, None, None, None


def avgpool2d(x, k, s, p=0, count_include_pad=False):
    """Per-channel k x k / s average pooling with symmetric zero padding ``p``;
    count_include_pad=False divides by the in-bounds taps (Keras/TF 'same')."""
    if hip_gate("pool", p < k, x):
        return AvgPoolHip.apply(x, k, s, p, count_include_pad)
    # contiguous NCHW: PyTorch-ROCm's avg_pool2d backward on a channels-last
    # view with padding and count_include_pad=False returns wrong gradients
    # (rel. error ~1.0; scripts/debug/avgpool_check.py)
    return _nhwc(F.avg_pool2d(_nchw(x).contiguous(), k, s, p,
                              count_include_pad=count_include_pad))


def cat_packed(xs, G):
    """Channel concat per configuration of packed [B, H, W, G*C_i] tensors."""
    B, H, W = xs[0].shape[:3]
    parts = [t.reshape(B, H, W, G, t.shape[-1] // G) for t in xs]
    return torch.cat(parts, dim=-1).reshape(B, H, W, -1)


class ReluAdd(torch.autograd.Function):
    """y = relu(a + b) in fp32 with one rounding; backward da = db = dy * (y > 0)
    (one saved tensor, no fp32 temporaries kept for autograd)."""

    @staticmethod
    def forward(ctx, a, b):
        y = torch.relu(a.float() + b.float()).to(a.dtype)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, = ctx.saved_tensors
        g = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
        return g, g.clone()


def relu_add(a, b):
    """relu(a + b) in fp32 with one rounding (BN-free residual join)."""
    return ReluAdd.apply(a, b)


class _GradMark(torch.autograd.Function):
    """Identity whose backward calls ``fn`` first: by then every layer above
    this point has issued its backward (their parameter gradients are final
    once the queued weight-gradient kernels are flushed).  Used for the
    bucketed DDP all-reduce overlapped with backward (runtime.baselines)."""

    @staticmethod
    def forward(ctx, x, fn):
        ctx.fn = fn
        y = x.view_as(x)
        link = getattr(x, "_cer_bnlink", None)
        if link is not None:           # keep the BN-link handoff to the consumer conv
            y._cer_bnlink = link
        return y

    @staticmethod
    def backward(ctx, dy):
        ctx.fn()
        return dy, None


def grad_mark(x, fn):
    return _GradMark.apply(x, fn)
