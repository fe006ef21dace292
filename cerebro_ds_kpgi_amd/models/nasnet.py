"""NASNet-Mobile, packed over G configurations.

``keras.applications.NASNetMobile(weights=None)`` as the reference builds it
(``cerebro_gpdb/in_rdbms_helper.py:390-396``); it is the slow model of the
heterogeneous-workload grid (``cerebro_gpdb/imagenetcat.py:50-60``, 10 x
NASNetMobile bs4 next to 38 x MobileNetV2 bs128).  NASNet-A with
penultimate_filters 1056, num_blocks 4, stem_block_filters 32,
filter_multiplier 2, skip_reduction False; at 112x112x3:

    stem conv3x3/2 valid (32) + BN                        112 -> 55
    reduction cells stem_1 (f=11), stem_2 (f=22)          55 -> 28 -> 14
    normal cells 0-3 (f=44)                               14
    reduction reduce_4 (f=88), normal cells 5-8          14 -> 7
    reduction reduce_8 (f=176), normal cells 9-12         7 -> 4
    ReLU -> global average pool -> Dense(1000)

* separable block = ReLU -> depthwise k x k -> pointwise 1x1 -> BN -> ReLU
  -> depthwise k x k -> pointwise -> BN (k in {3, 5, 7}); its stride-2
  padding is Keras ``correct_pad`` (one less at top/left on even inputs),
  which the HIP depthwise kernel takes directly (``ops.nn.dwconv2d``),
* adjust block for the previous cell's input ``p``: spatial mismatch ->
  ReLU, 1x1 convs (f/2 each) of the even and the odd-shifted stride-2
  subsamples, concat, BN; channel mismatch -> ReLU, 1x1 projection, BN,
* a cell returns (output, its own input): the input becomes the next
  cell's ``p``,
* BN momentum 0.9997 / eps 1e-3 (Keras NASNet's values).

Parameters: 5 289 978 trainable + 36 738 moving statistics = 5 326 716, the
Keras NASNetMobile count for 1000 classes.
"""

import os

import torch

from .common import BN, Conv, Dense, PackedNet
from ..ops import nn as P
from ..runtime.arena import ParamSpec


# the cells' branch additions folded into the last BN of a separable block
# as its residual (CER_NASNET_FUSED_ADD=0: BN, then an add kernel)
_FUSED_ADD = os.environ.get("CER_NASNET_FUSED_ADD", "1") != "0"


def correct_pad(n, k):
    """Keras ``imagenet_utils.correct_pad`` for a stride-2 k-window over n: (before, after)."""
    return (k // 2 - (1 - n % 2), k // 2)


class _PW(object):
    """1x1 convolution (pointwise half of SeparableConv2D, adjust / cell-input convs)."""
    k, stride, pad = 1, 1, 0

    def __init__(self, net, name, cin, cout):
        self.w = net.spec(ParamSpec(name, (cout, 1, 1, cin), "weight", fan_in=cin))


class _SepBlock(object):
    """Keras ``_separable_conv_block``: two SeparableConv2D(use_bias=False) + BN."""

    def __init__(self, net, block_id, cin, f, k, stride):
        self.k, self.stride = k, stride
        n1, n2 = "separable_conv_1_" + block_id, "separable_conv_2_" + block_id
        self.dw1 = net.spec(ParamSpec(n1 + "/depthwise_kernel", (cin, k, k), "weight",
                                      fan_in=k * k))
        self.pw1 = _PW(net, n1 + "/pointwise_kernel", cin, f)
        self.bn1 = BN(net, "separable_conv_1_bn_" + block_id, f)
        self.dw2 = net.spec(ParamSpec(n2 + "/depthwise_kernel", (f, k, k), "weight",
                                      fan_in=k * k))
        self.pw2 = _PW(net, n2 + "/pointwise_kernel", f, f)
        self.bn2 = BN(net, "separable_conv_2_bn_" + block_id, f)


class _Adjust(object):
    """Keras ``_adjust_block``: brings ``p`` to the cell's resolution and width."""

    def __init__(self, net, block_id, cp, hp, h, f, first=False):
        self.kind = None
        self.cout = cp
        if first:                             # p is None: p = ip, unchanged
            return
        if hp != h:
            self.kind = "reduce"
            half = f // 2
            self.c1 = _PW(net, "adjust_conv_1_{}/kernel".format(block_id), cp, half)
            self.c2 = _PW(net, "adjust_conv_2_{}/kernel".format(block_id), cp, half)
            self.bn = BN(net, "adjust_bn_" + block_id, 2 * half)
            self.cout = 2 * half
        elif cp != f:
            self.kind = "project"
            self.c = _PW(net, "adjust_conv_projection_{}/kernel".format(block_id), cp, f)
            self.bn = BN(net, "adjust_bn_" + block_id, f)
            self.cout = f


class _Cell(object):
    def __init__(self, net, kind, block_id, c_in, h_in, c_p, h_p, f):
        self.kind = kind
        first = c_p is None                   # first cell: p = ip
        if first:
            c_p, h_p = c_in, h_in
        self.adj = _Adjust(net, block_id, c_p, h_p, h_in, f, first)
        pc = self.adj.cout
        pre = "normal" if kind == "normal" else "reduction"
        self.h = _PW(net, "{}_conv_1_{}/kernel".format(pre, block_id), c_in, f)
        self.hbn = BN(net, "{}_bn_1_{}".format(pre, block_id), f)
        b = "_" + block_id
        if kind == "normal":
            self.l1 = _SepBlock(net, "normal_left1" + b, f, f, 5, 1)
            self.r1 = _SepBlock(net, "normal_right1" + b, pc, f, 3, 1)
            self.l2 = _SepBlock(net, "normal_left2" + b, pc, f, 5, 1)
            self.r2 = _SepBlock(net, "normal_right2" + b, pc, f, 3, 1)
            self.l5 = _SepBlock(net, "normal_left5" + b, f, f, 3, 1)
            self.cout, self.hout = pc + 5 * f, h_in
        else:
            self.l1 = _SepBlock(net, "reduction_left1" + b, f, f, 5, 2)
            self.r1 = _SepBlock(net, "reduction_right1" + b, pc, f, 7, 2)
            self.r2 = _SepBlock(net, "reduction_right2" + b, pc, f, 7, 2)
            self.r3 = _SepBlock(net, "reduction_right3" + b, pc, f, 5, 2)
            self.l4 = _SepBlock(net, "reduction_left4" + b, f, f, 3, 1)
            self.cout, self.hout = 4 * f, (h_in + 1) // 2


class PackedNASNetMobile(PackedNet):
    def __init__(self, num_classes=1000, input_hw=112, penultimate_filters=1056, num_blocks=4,
                 stem_filters=32, multiplier=2):
        super(PackedNASNetMobile, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.bn_momentum = 1.0 - 0.9997
        self.bn_eps = 1e-3
        f = penultimate_filters // 24
        self.stem = Conv(self, "stem_conv1", 3, stem_filters, 3, 2, 0)
        self.stem_bn = BN(self, "stem_bn1", stem_filters)
        plan = [("reduction", "stem_1", f // multiplier ** 2),
                ("reduction", "stem_2", f // multiplier)]
        plan += [("normal", str(i), f) for i in range(num_blocks)]
        plan += [("reduction", "reduce_{}".format(num_blocks), f * multiplier)]
        plan += [("normal", str(num_blocks + i + 1), f * multiplier) for i in range(num_blocks)]
        plan += [("reduction", "reduce_{}".format(2 * num_blocks), f * multiplier ** 2)]
        plan += [("normal", str(2 * num_blocks + i + 1), f * multiplier ** 2)
                 for i in range(num_blocks)]
        c_in, h_in = stem_filters, (input_hw - 3) // 2 + 1
        c_p = h_p = None
        self.cells = []
        for kind, bid, filt in plan:
            cell = _Cell(self, kind, bid, c_in, h_in, c_p, h_p, filt)
            self.cells.append(cell)
            c_p, h_p = c_in, h_in
            c_in, h_in = cell.cout, cell.hout
        self.fc = Dense(self, "predictions", c_in, num_classes)
        self.build_layout()

    # ------------------------------------------------------------------
    def _sep(self, x, blk, training, plus=None):
        """The separable block; ``plus``: the cell branch it is added to,
        folded into the block's last BN as its residual (one BN apply
        instead of BN + an add kernel; the residual gradient comes out of
        the BN backward)"""
        k = blk.k
        x = torch.relu(x)
        if blk.stride == 2:
            pad = correct_pad(x.shape[1], k) + correct_pad(x.shape[2], k)
        else:
            pad = k // 2
        x = P.dwconv2d(x, self.ref(blk.dw1), blk.stride, pad)
        x = self.conv_bn(x, blk.pw1, blk.bn1, training, relu=True)
        x = P.dwconv2d(x, self.ref(blk.dw2), 1, k // 2)
        if plus is not None and not _FUSED_ADD:
            return self.conv_bn(x, blk.pw2, blk.bn2, training, relu=False) + plus
        return self.conv_bn(x, blk.pw2, blk.bn2, training, relu=False, residual=plus)

    def _adjust(self, p, adj, training):
        if adj.kind == "reduce":
            p = torch.relu(p)
            p1 = p[:, ::2, ::2, :].contiguous()
            # ZeroPadding((0,1),(0,1)) + Cropping((1,0),(1,0)) = shift by one pixel
            p2 = P._zero_pad(p, (0, 1, 0, 1))[:, 1::2, 1::2, :].contiguous()
            p = P.cat_packed([self.conv(p1, adj.c1), self.conv(p2, adj.c2)], self.G)
            return self.bn(p, adj.bn, training, relu=False)
        if adj.kind == "project":
            return self.conv_bn(torch.relu(p), adj.c, adj.bn, training, relu=False)
        return p

    def _cell(self, ip, p, cell, training):
        p = self._adjust(ip if p is None else p, cell.adj, training)
        h = self.conv_bn(torch.relu(ip), cell.h, cell.hbn, training, relu=False)
        if cell.kind == "normal":
            x1 = self._sep(h, cell.l1, training, plus=self._sep(p, cell.r1, training))
            x2 = self._sep(p, cell.l2, training, plus=self._sep(p, cell.r2, training))
            x3 = P.avgpool2d(h, 3, 1, 1) + p
            x4 = 2.0 * P.avgpool2d(p, 3, 1, 1)     # Keras left4 + right4: the same pool twice
            x5 = self._sep(h, cell.l5, training, plus=h)
            return P.cat_packed([p, x1, x2, x3, x4, x5], self.G), ip
        h3 = P._zero_pad(h, correct_pad(h.shape[1], 3) + correct_pad(h.shape[2], 3))
        x1 = self._sep(h, cell.l1, training, plus=self._sep(p, cell.r1, training))
        mx = P.maxpool2d(h3, 3, 2, 0)              # reduction_left2 == reduction_right5
        x2 = self._sep(p, cell.r2, training, plus=mx)
        x3 = self._sep(p, cell.r3, training, plus=P.avgpool2d(h3, 3, 2, 0))
        x4 = P.avgpool2d(x1, 3, 1, 1) + x2
        x5 = self._sep(x1, cell.l4, training, plus=mx)
        return P.cat_packed([x2, x3, x4, x5], self.G), ip

    def forward(self, x, training):
        x = self.conv_bn(x, self.stem, self.stem_bn, training, relu=False, anchor=True)
        p = None
        for cell in self.cells:
            x, p = self._cell(x, p, cell, training)
        x = P.global_avgpool(torch.relu(x))
        return self.dense(x, self.fc)
