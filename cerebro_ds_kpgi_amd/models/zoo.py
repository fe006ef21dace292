"""The rest of the reference's model factory,
packed over G configurations.

* ``mobilenetv1`` — ``keras.applications.MobileNet`` (alpha 1.0): conv3x3/2
  32 + 13 depthwise-separable blocks (dw3x3 + BN + ReLU6, pw1x1 + BN +
  ReLU6), GAP, Dense.
* ``densenet121`` / ``densenet201`` — ``keras.applications.DenseNet``:
  growth 32, blocks [6,12,24,16] / [6,12,48,32]; layer = BN-ReLU-conv1x1(4k)-
  BN-ReLU-conv3x3(k), concatenated; transition = BN-ReLU-conv1x1(c/2)-
  AvgPool2x2/2; final BN-ReLU, GAP, Dense.
* ``resnext101`` — ``classification_models`` ResNeXt-101 32x4d (reference
  ``in_rdbms_helper.py:300-313``): ResNet stem, bottlenecks [3,4,23,3] with a
  32-group 3x3 conv of width 128/256/512/1024.
* ``resnet50_nobn`` — the BN-free Keras ResNet-50 of the Spark paths
  (``cerebro_gpdb/resnet50tfk.py:45-319``): conv 7x7/2 *valid*, biases
  everywhere, no BatchNorm, TruncatedNormal(0, 0.01) init for kernels and
  biases, MaxPool 3x3/2 SAME, AvgPool 7x7 SAME -> 2048 -> Dense.
"""

from .common import BN, Conv, Dense, PackedNet
from ..ops import nn as P
from ..runtime.arena import ParamSpec

_MBV1 = [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2), (512, 1), (512, 1),
         (512, 1), (512, 1), (512, 1), (1024, 2), (1024, 1)]


class PackedMobileNetV1(PackedNet):
    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedMobileNetV1, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.stem = Conv(self, "conv1", 3, 32, 3, 2, 1)
        self.stem_bn = BN(self, "conv1_bn", 32)
        self.blocks = []
        cin = 32
        for i, (c, s) in enumerate(_MBV1):
            n = i + 1
            blk = {"stride": s,
                   "dw": self.spec(ParamSpec("conv_dw_{}/depthwise_kernel".format(n), (cin, 3, 3),
                                             "weight", fan_in=9)),
                   "dw_bn": BN(self, "conv_dw_{}_bn".format(n), cin),
                   "pw": Conv(self, "conv_pw_{}".format(n), cin, c, 1, 1, 0),
                   "pw_bn": BN(self, "conv_pw_{}_bn".format(n), c)}
            self.blocks.append(blk)
            cin = c
        self.fc = Dense(self, "conv_preds", cin, num_classes)
        self.build_layout()

    def forward(self, x, training):
        # every pointwise BN output but the last feeds only the next depthwise
        # conv, whose dgrad computes its backward partials (BN link)
        x = self.conv_bn(x, self.stem, self.stem_bn, training, relu=6, anchor=True,
                         link_out=True)
        last = len(self.blocks) - 1
        for i, blk in enumerate(self.blocks):
            x = P.dwconv2d(x, self.ref(blk["dw"]), blk["stride"], 1, stats=training)
            x = self.bn(x, blk["dw_bn"], training, relu=6, link_out=True)
            x = self.conv_bn(x, blk["pw"], blk["pw_bn"], training, relu=6, link_out=i < last)
        x = P.global_avgpool(x)
        return self.dense(x, self.fc)


_DENSE = {121: [6, 12, 24, 16], 169: [6, 12, 32, 32], 201: [6, 12, 48, 32]}


class PackedDenseNet(PackedNet):
    growth = 32

    def __init__(self, depth=121, num_classes=1000, input_hw=112):
        super(PackedDenseNet, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        k = self.growth
        self.stem = Conv(self, "conv1/conv", 3, 64, 7, 2, 3)
        self.stem_bn = BN(self, "conv1/bn", 64)
        self.stages = []
        c = 64
        blocks = _DENSE[depth]
        for bi, n in enumerate(blocks):
            layers = []
            for li in range(n):
                name = "conv{}_block{}".format(bi + 2, li + 1)
                layers.append({"bn1": BN(self, name + "_0_bn", c),
                               "c1": Conv(self, name + "_1_conv", c, 4 * k, 1, 1, 0),
                               "bn2": BN(self, name + "_1_bn", 4 * k),
                               "c2": Conv(self, name + "_2_conv", 4 * k, k, 3, 1, 1)})
                c += k
            trans = None
            if bi < len(blocks) - 1:
                name = "pool{}".format(bi + 2)
                trans = {"bn": BN(self, name + "_bn", c),
                         "conv": Conv(self, name + "_conv", c, c // 2, 1, 1, 0)}
                c = c // 2
            self.stages.append((layers, trans))
        self.final_bn = BN(self, "bn", c)
        self.fc = Dense(self, "fc1000", c, num_classes)
        self.build_layout()

    def forward(self, x, training):
        x = self.conv_bn(x, self.stem, self.stem_bn, training, anchor=True)
        x = P.maxpool2d(x, 3, 2, 1)
        G = self.G
        for layers, trans in self.stages:
            for L in layers:
                h = self.bn(x, L["bn1"], training)
                h = self.conv_bn(h, L["c1"], L["bn2"], training)
                h = self.conv(h, L["c2"])
                x = P.cat_packed([x, h], G)
            if trans is not None:
                x = self.bn(x, trans["bn"], training)
                x = self.conv(x, trans["conv"])
                x = P.avgpool2d(x, 2, 2)
        x = self.bn(x, self.final_bn, training)
        x = P.global_avgpool(x)
        return self.dense(x, self.fc)


class PackedResNeXt(PackedNet):
    cardinality = 32

    def __init__(self, depth=101, num_classes=1000, input_hw=112):
        super(PackedResNeXt, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        stages = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3]}[depth]
        self.conv1 = Conv(self, "conv0", 3, 64, 7, 2, 3)
        self.bn1 = BN(self, "bn0", 64)
        self.blocks = []
        cin = 64
        for si, n in enumerate(stages):
            width = 128 * 2 ** si
            cout = 256 * 2 ** si
            for bi in range(n):
                stride = 2 if (si > 0 and bi == 0) else 1
                name = "stage{}_unit{}".format(si + 1, bi + 1)
                blk = {"stride": stride,
                       "c1": Conv(self, name + "_conv1", cin, width, 1, 1, 0),
                       "b1": BN(self, name + "_bn1", width),
                       "c2": self.spec(ParamSpec(name + "_conv2/kernel",
                                                 (width, 3, 3, width // self.cardinality),
                                                 "weight",
                                                 fan_in=9 * width // self.cardinality)),
                       "b2": BN(self, name + "_bn2", width),
                       "c3": Conv(self, name + "_conv3", width, cout, 1, 1, 0),
                       "b3": BN(self, name + "_bn3", cout)}
                if bi == 0:
                    blk["cs"] = Conv(self, name + "_sc", cin, cout, 1, stride, 0)
                    blk["bs"] = BN(self, name + "_sc_bn", cout)
                self.blocks.append(blk)
                cin = cout
        self.fc = Dense(self, "fc1", cin, num_classes)
        self.build_layout()

    def forward(self, x, training):
        x = self.conv_bn(x, self.conv1, self.bn1, training, anchor=True)
        x = P.maxpool2d(x, 3, 2, 1)
        for blk in self.blocks:
            sc = (self.conv_bn(x, blk["cs"], blk["bs"], training, relu=False)
                  if "cs" in blk else x)
            h = self.conv_bn(x, blk["c1"], blk["b1"], training)
            h = P.grouped_conv2d(h, self.ref(blk["c2"]), blk["stride"], 1, self.cardinality)
            h = self.bn(h, blk["b2"], training)
            x = self.conv_bn(h, blk["c3"], blk["b3"], training, relu=True, residual=sc)
        x = P.global_avgpool(x)
        return self.dense(x, self.fc)


class PackedResNet50NoBN(PackedNet):
    KI = "tn0.01"

    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedResNet50NoBN, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.conv1 = self._conv("conv1", 3, 64, 7, 2, 0)
        self.blocks = []
        cin = 64
        for si, (n, w) in enumerate(zip([3, 4, 6, 3], [64, 128, 256, 512])):
            for bi in range(n):
                stride = 2 if (si > 0 and bi == 0) else 1
                name = "res{}{}".format(si + 2, chr(ord("a") + bi))
                blk = {"c1": self._conv(name + "_branch2a", cin, w, 1, stride, 0),
                       "c2": self._conv(name + "_branch2b", w, w, 3, 1, 1),
                       "c3": self._conv(name + "_branch2c", w, 4 * w, 1, 1, 0)}
                if bi == 0:
                    blk["cs"] = self._conv(name + "_branch1", cin, 4 * w, 1, stride, 0)
                self.blocks.append(blk)
                cin = 4 * w
        self.fc = Dense(self, "fc1000", cin, num_classes, init=self.KI)
        self.fc.b.init = self.KI
        self.build_layout()

    def _conv(self, name, cin, cout, k, s, p):
        c = Conv(self, name, cin, cout, k, s, p)
        c.w.init = self.KI
        c.bias = self.spec(ParamSpec(name + "/bias", (cout,), "bias", init=self.KI))
        return c

    def _cba(self, x, c, act, anchor=False):
        return P.conv2d_bias_act(x, self.ref(c.w), self.ref(c.bias), c.stride, c.pad, act=act,
                                 anchor=self.anchor if anchor else None)

    def forward(self, x, training):
        x = self._cba(x, self.conv1, 1, anchor=True)          # 112 -> 53 (valid)
        x = P.maxpool2d(x, 3, 2, 1)                             # SAME: 53 -> 27
        for blk in self.blocks:
            sc = self._cba(x, blk["cs"], 0) if "cs" in blk else x
            h = self._cba(x, blk["c1"], 1)
            h = self._cba(h, blk["c2"], 1)
            h = self._cba(h, blk["c3"], 0)
            x = P.relu_add(h, sc)
        x = P.global_avgpool(x)                                 # AvgPool 7x7 SAME on 4x4
        return self.dense(x, self.fc)
