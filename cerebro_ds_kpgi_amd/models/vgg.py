"""VGG-16 / VGG-19 for ImageNet-112, packed over G configurations.

``keras.applications`` VGG16 as used by the reference
(``cerebro_gpdb/vgg16tfk_default.py:49-263``; shapes SURVEY.md §2.8 K2):
13 conv3x3 (+bias, ReLU) in 5 blocks, MaxPool 2x2/2 valid after each block
(112 -> 56 -> 28 -> 14 -> 7 -> 3), Flatten (h, w, c order) 4608 ->
Dense 4096 ReLU -> Dense 4096 ReLU -> Dense 1000.  54.47 M parameters.
"""

import torch

from .common import Conv, Dense, PackedNet
from ..ops import nn as P
from ..runtime.arena import ParamSpec

_CFGS = {16: [(64, 2), (128, 2), (256, 3), (512, 3), (512, 3)],
         19: [(64, 2), (128, 2), (256, 4), (512, 4), (512, 4)]}


class PackedVGG16(PackedNet):
    depth = 16

    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedVGG16, self).__init__()
        _CFG = _CFGS[self.depth]
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.convs = []
        cin = 3
        hw = input_hw
        for bi, (c, n) in enumerate(_CFG):
            blk = []
            for li in range(n):
                name = "block{}_conv{}".format(bi + 1, li + 1)
                conv = Conv(self, name, cin, c, 3, 1, 1)
                bias = self.spec(ParamSpec(name + "/bias", (c,), "bias"))
                blk.append((conv, bias))
                cin = c
            self.convs.append(blk)
            hw = hw // 2
        self.flat = hw * hw * cin
        self.fc1 = Dense(self, "fc1", self.flat, 4096)
        self.fc2 = Dense(self, "fc2", 4096, 4096)
        self.fc3 = Dense(self, "predictions", 4096, num_classes)
        self.build_layout()

    def forward(self, x, training):
        first = True
        for blk in self.convs:
            for conv, bias in blk:
                x = P.conv2d_bias_act(x, self.ref(conv.w), self.ref(bias), conv.stride, conv.pad,
                                      act=1, anchor=self.anchor if first else None)
                first = False
            x = P.maxpool2d(x, 2, 2, 0)
            nxt = self.convs.index(blk) + 1
            x = self.bucket_mark(x, self.convs[nxt][0][0].w if nxt < len(self.convs)
                                 else self.fc1.w)
        B, H, W, GC = x.shape
        G = self.G
        C = GC // G
        # per-config flatten in (h, w, c) order: [B,H,W,G,C] -> [B,G,H,W,C]
        x = x.view(B, H, W, G, C).permute(0, 3, 1, 2, 4).reshape(B, G * H * W * C)
        x = self.dense(x, self.fc1, relu=True)
        x = self.bucket_mark(x, self.fc2.w)
        x = self.dense(x, self.fc2, relu=True)
        x = self.bucket_mark(x, self.fc3.w)
        return self.dense(x, self.fc3)


class PackedVGG19(PackedVGG16):
    """VGG-19: blocks of 2, 2, 4, 4, 4 convs (``keras.applications.VGG19``)."""
    depth = 19
