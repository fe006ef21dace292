"""Small CNNs: the 32x32 tiny CNN (BASELINE config 1 plumbing model) and
MobileNetV2 (hetero / model-size drill-downs, reference
``cerebro_gpdb/imagenetcat.py:50-60,68-99``).

MobileNetV2 follows ``keras.applications`` (alpha 1.0): conv3x3/2 32 ->
17 inverted-residual blocks (expand 1x1 + BN + ReLU6, depthwise 3x3 + BN +
ReLU6, project 1x1 + BN, residual when stride 1 and widths match) -> conv1x1
1280 + BN + ReLU6 -> GAP -> Dense.
"""

from .common import BN, Conv, Dense, PackedNet
from ..ops import nn as P
from ..runtime.arena import ParamSpec


class PackedTinyCNN(PackedNet):
    def __init__(self, num_classes=10, input_hw=32):
        super(PackedTinyCNN, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.c1 = Conv(self, "conv1", 3, 16, 3, 1, 1)
        self.b1 = BN(self, "bn1", 16)
        self.c2 = Conv(self, "conv2", 16, 32, 3, 1, 1)
        self.b2 = BN(self, "bn2", 32)
        self.fc = Dense(self, "fc", 32, num_classes)
        self.build_layout()

    def forward(self, x, training):
        x = self.conv_bn(x, self.c1, self.b1, training, anchor=True)
        x = P.maxpool2d(x, 2, 2, 0)
        x = self.conv_bn(x, self.c2, self.b2, training)
        x = P.global_avgpool(x)
        return self.dense(x, self.fc)


# (expansion t, channels c, repeats n, stride s)
_MBV2 = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2),
         (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]


class PackedMobileNetV2(PackedNet):
    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedMobileNetV2, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.stem = Conv(self, "Conv1", 3, 32, 3, 2, 1)
        self.stem_bn = BN(self, "bn_Conv1", 32)
        self.blocks = []
        cin = 32
        bid = 0
        for t, c, n, s in _MBV2:
            for i in range(n):
                stride = s if i == 0 else 1
                name = "block_{}".format(bid)
                blk = {"stride": stride, "res": stride == 1 and cin == c}
                hidden = cin * t
                if t != 1:
                    blk["exp"] = Conv(self, name + "_expand", cin, hidden, 1, 1, 0)
                    blk["exp_bn"] = BN(self, name + "_expand_BN", hidden)
                blk["dw"] = self.spec(ParamSpec(name + "_depthwise/depthwise_kernel",
                                                (hidden, 3, 3), "weight", fan_in=9))
                blk["dw_bn"] = BN(self, name + "_depthwise_BN", hidden)
                blk["proj"] = Conv(self, name + "_project", hidden, c, 1, 1, 0)
                blk["proj_bn"] = BN(self, name + "_project_BN", c)
                self.blocks.append(blk)
                cin = c
                bid += 1
        self.head = Conv(self, "Conv_1", cin, 1280, 1, 1, 0)
        self.head_bn = BN(self, "Conv_1_bn", 1280)
        self.fc = Dense(self, "Logits", 1280, num_classes)
        self.build_layout()

    def forward(self, x, training):
        # the first block has no expansion: its depthwise dgrad then computes
        # the stem BN's backward partials (BN link)
        b0 = self.blocks[0]
        x = self.conv_bn(x, self.stem, self.stem_bn, training, relu=6, anchor=True,
                         link_out="exp" not in b0 and not b0["res"])
        for blk in self.blocks:
            h = x
            if "exp" in blk:
                h = self.conv_bn(h, blk["exp"], blk["exp_bn"], training, relu=6,
                                 link_out=True)     # its sole consumer: the depthwise dgrad
            h = P.dwconv2d(h, self.ref(blk["dw"]), blk["stride"], 1, stats=training)
            h = self.bn(h, blk["dw_bn"], training, relu=6, link_out=True)
            h = self.conv_bn(h, blk["proj"], blk["proj_bn"], training, relu=False,
                             residual=x if blk["res"] else None)
            x = h
        x = self.conv_bn(x, self.head, self.head_bn, training, relu=6)
        x = P.global_avgpool(x)
        return self.dense(x, self.fc)
