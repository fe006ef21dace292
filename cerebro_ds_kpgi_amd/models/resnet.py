"""ResNet-18/34/50/101/152 for ImageNet-112, packed over G configurations.

Architecture = ``keras.applications`` ResNet50 as used by the reference
(``cerebro_gpdb/resnet50tfk_default.py:161-314``; conv table SURVEY.md §2.8
K1): ZeroPad(3) -> conv7x7/2 valid -> BN -> ReLU -> ZeroPad(1) ->
MaxPool3x3/2 valid, bottleneck stages [3, 4, 6, 3] with the stride on the
block's first 1x1 conv and a 1x1 projection shortcut in each stage's first
block, global average pool, Dense(1000).  At 112x112 the stage resolutions
are 28 / 14 / 7 / 4.

Differences (documented, deliberate): convolutions carry no bias — a bias
followed by BatchNorm is exactly cancelled by the batch-mean subtraction and
its gradient is identically zero; BN momentum/eps follow the reference's
PyTorch trainer (0.1 / 1e-5).  Trainable parameters: 25 557 032 (= the
torchvision count); Keras reports 25 583 592 trainable + 53 120 moving
statistics = 25 636 712, the difference being the 26 560 conv biases.
Serialised blobs (checkpoints, MA states) are nevertheless in the Keras
``get_weights()`` layout: HWIO kernels, the dropped biases as zeros right
after their kernels (a non-zero bias read from a Keras blob folds into the
BN moving mean), and Keras's layer order, in which a projection block lists
``..._branch2c, ..._branch1`` kernels before ``bn..._branch2c, bn..._branch1``
(``runtime.arena.KerasBias``, ``runtime.serialize``).

ResNet-18/34 (hyperopt grid, ``cerebro_gpdb/imagenetcat.py:100-105``) use
basic blocks with the same stem; 101/152 bottleneck depths [3,4,23,3] /
[3,8,36,3] (model-size drill-down).
"""

import os

import torch

from .common import BN, Conv, Dense, PackedNet
from ..ops import nn as P
from ..ops import streams
from ..ops.backend import get_backend

# projection shortcuts on the branch stream (CER_SC_BRANCH=1): the shortcut
# conv + BN of a stage's first block runs concurrently with the main path's
# c1 / c2 in forward and, being created after c1, its backward runs ahead of
# c1's (autograd's order) on the branch stream, beside c2 / c1's backward
_SC_BRANCH = os.environ.get("CER_SC_BRANCH", "1") == "1"

_BOTTLENECK = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}
_BASIC = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3]}


class PackedResNet(PackedNet):
    def __init__(self, depth=50, num_classes=1000, input_hw=112):
        super(PackedResNet, self).__init__()
        self.depth = depth
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.bottleneck = depth in _BOTTLENECK
        # stem: ZeroPad(3) + conv7x7/2 valid == conv7x7/2 pad 3
        self.conv1 = Conv(self, "conv1", 3, 64, 7, 2, 3)
        self.bn1 = BN(self, "bn_conv1", 64)
        self.blocks = []
        cin = 64
        stages = _BOTTLENECK[depth] if self.bottleneck else _BASIC[depth]
        widths = [64, 128, 256, 512]
        for si, (n, w) in enumerate(zip(stages, widths)):
            for bi in range(n):
                stride = 2 if (si > 0 and bi == 0) else 1
                name = "res{}{}".format(si + 2, chr(ord("a") + bi) if bi < 26 else "z{}".format(bi))
                blk = {}
                if self.bottleneck:
                    cout = 4 * w
                    blk["c1"] = Conv(self, name + "_branch2a", cin, w, 1, stride, 0)
                    blk["b1"] = BN(self, name.replace("res", "bn") + "_branch2a", w)
                    blk["c2"] = Conv(self, name + "_branch2b", w, w, 3, 1, 1)
                    blk["b2"] = BN(self, name.replace("res", "bn") + "_branch2b", w)
                    blk["c3"] = Conv(self, name + "_branch2c", w, cout, 1, 1, 0)
                    blk["b3"] = BN(self, name.replace("res", "bn") + "_branch2c", cout)
                else:
                    cout = w
                    blk["c1"] = Conv(self, name + "_branch2a", cin, w, 3, stride, 1)
                    blk["b1"] = BN(self, name.replace("res", "bn") + "_branch2a", w)
                    blk["c2"] = Conv(self, name + "_branch2b", w, w, 3, 1, 1)
                    blk["b2"] = BN(self, name.replace("res", "bn") + "_branch2b", w)
                if bi == 0 and (stride != 1 or cin != cout):
                    blk["cs"] = Conv(self, name + "_branch1", cin, cout, 1, stride, 0)
                    blk["bs"] = BN(self, name.replace("res", "bn") + "_branch1", cout)
                for c, b in (("c1", "b1"), ("c2", "b2"), ("c3", "b3"), ("cs", "bs")):
                    if c in blk:
                        self.drop_bias(blk[c], blk[b])
                self.blocks.append(blk)
                cin = cout
        self.feat = cin
        self.fc = Dense(self, "fc1000", cin, num_classes)
        self.drop_bias(self.conv1, self.bn1)
        self.keras_order = self._keras_layer_order()
        self.build_layout()

    def _keras_layer_order(self):
        """Keras lists layers by graph depth: in a projection block the two
        convs feeding the add (last main-path conv, shortcut conv) come
        before their two BatchNorms."""
        def bn(b):
            return [b.g.name, b.b.name, b.rm.name, b.rv.name]
        order = [self.conv1.w.name] + bn(self.bn1)
        last = "c3" if self.bottleneck else "c2"
        lastb = "b3" if self.bottleneck else "b2"
        for blk in self.blocks:
            for c, b in (("c1", "b1"), ("c2", "b2"), ("c3", "b3")):
                if c in blk and c != last:
                    order += [blk[c].w.name] + bn(blk[b])
            if "cs" in blk:
                order += [blk[last].w.name, blk["cs"].w.name] + bn(blk[lastb]) + bn(blk["bs"])
            else:
                order += [blk[last].w.name] + bn(blk[lastb])
        return order + [self.fc.w.name, self.fc.b.name]

    def forward(self, x, training):
        x = self.conv_bn(x, self.conv1, self.bn1, training, anchor=True)
        x = P.maxpool2d(x, 3, 2, 1)  # ZeroPad(1) + MaxPool 3x3/2 valid (inputs >= 0 post-ReLU)
        nb = len(self.blocks)
        for bi, blk in enumerate(self.blocks):
            # x has two consumers (c1 and the shortcut): their input gradients
            # meet in a GradJoin instead of an autograd add kernel
            j = P.GradJoin() if training else None
            # (not under DDP's gradient buckets: a graph segment may end
            # between the branch's backward and its join; fp32 only: in the
            # bf16 diagnostic mode replays drift from eager by 1e-3 - 8e-3
            # with the branch (tests/test_graph_gpu.py) -- most likely the
            # split-K fp32 atomics' order, which overlapping kernels vary,
            # flipping bf16 roundings of activations; fp32 replays stay at
            # the 1e-4 noise floor)
            branch = ("cs" in blk and training and _SC_BRANCH and x.is_cuda
                      and x.dtype == torch.float32 and get_backend() == "hip"
                      and self.grad_buckets is None)
            if branch:
                cur = torch.cuda.current_stream(x.device)
                fork = torch.cuda.Event()
                fork.record(cur)
            elif "cs" in blk:
                sc = self.conv_bn(x, blk["cs"], blk["bs"], training, relu=False, join=j)
            rj = None if "cs" in blk else j
            if "cs" not in blk:
                sc = x
            # every BN output inside the block has one conv consumer, and the
            # block output's two consumers are joined: all link (BNLink), except
            # the last block's output (global average pool)
            link_blk = j is not None and bi + 1 < nb
            # b1 / b2 outputs feed only the next conv_bn: HL operand format
            h = self.conv_bn(x, blk["c1"], blk["b1"], training, join=j, link_out=True,
                             hl_out=True)
            if branch:
                bs = streams.branch_stream(x.device.index)
                bs.wait_event(fork)
                x.record_stream(bs)
                streams.set_branch_parent(x.device.index, cur)
                try:
                    with torch.cuda.stream(bs):
                        sc = self.conv_bn(x, blk["cs"], blk["bs"], training, relu=False,
                                          join=j)
                finally:
                    streams.set_branch_parent(x.device.index, None)
            if self.bottleneck:
                h = self.conv_bn(h, blk["c2"], blk["b2"], training, link_out=True, hl_out=True)
            if branch:
                cur.wait_stream(bs)
                sc.record_stream(cur)
            if self.bottleneck:
                h = self.conv_bn(h, blk["c3"], blk["b3"], training, relu=True, residual=sc,
                                 res_join=rj, link_out=link_blk)
            else:
                h = self.conv_bn(h, blk["c2"], blk["b2"], training, relu=True, residual=sc,
                                 res_join=rj, link_out=link_blk)
            x = h
            if bi + 1 < nb:
                x = self.bucket_mark(x, self.blocks[bi + 1]["c1"].w)
            else:
                x = self.bucket_mark(x, self.fc.w)
        x = P.global_avgpool(x)
        return self.dense(x, self.fc)
