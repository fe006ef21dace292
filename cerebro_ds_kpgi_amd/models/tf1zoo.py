"""The reference's raw-TF1 model zoo, packed over G
configurations: the two architectures of it that the Keras factory does not
already cover.  (``models/cnn/tf/{resnet50,resnet18,vgg16}.py`` are the
BN-free ResNet-50 = ``resnet50_nobn``, ResNet-18 and VGG-16 of the factory.)

* ``squeezenet`` — ``cerebro_gpdb/models/cnn/tf/squeezenet.py:5-107``:
  conv3x3/2 SAME (64) + bias + ReLU, MaxPool 3x3/2 VALID, fire modules
  (squeeze 1x1 + bias + ReLU -> [expand 1x1 + bias | expand 3x3 + bias] ->
  ReLU, with the input added before the ReLU in fire3/5/7/9), MaxPool after
  fire3 and fire5, conv10 1x1 (1000, N(0, 0.01)) + bias + ReLU, global
  average pool = logits.  Xavier kernels, biases constant 0.1.
* ``densenet_tf1`` — ``cerebro_gpdb/models/cnn/tf/densenet.py:6-77``:
  growth 24, no BatchNorm, conv7x7/2 SAME (48); dense blocks of 6/12/48/32
  bottlenecks (ReLU-conv1x1(96)-ReLU-conv3x3(24), concatenated); transitions
  ReLU-conv1x1(24)-AvgPool 2x2/2 VALID; ReLU, global average pool, Dense.
  Convolutions have no bias (``use_bias=False``).

TF ``SAME`` on an even input with stride 2 pads one less at the top/left
than at the bottom/right; those convolutions get that exact asymmetric zero
padding (``ops.nn._zero_pad``) in front of an unpadded HIP conv.
"""

import torch

from .common import Conv, Dense, PackedNet
from ..ops import nn as P
from ..runtime.arena import ParamSpec


def same_pad(n, k, s):
    """TF 'SAME' padding (before, after) of a k-window, stride s, over n."""
    out = (n + s - 1) // s
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


class _BiasConv(object):
    def __init__(self, net, name, cin, cout, k, stride=1, pad=0, w_init="glorot", b_init="const0.1"):
        self.conv = Conv(net, name, cin, cout, k, stride, pad)
        self.conv.w.init = w_init
        self.b = net.spec(ParamSpec(name + "_b", (cout,), "bias", init=b_init))


class PackedSqueezeNet(PackedNet):
    _FIRES = [(16, 64, False), (16, 64, True), "pool", (32, 128, False), (32, 128, True), "pool",
              (48, 192, False), (48, 192, True), (64, 256, False), (64, 256, True)]

    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedSqueezeNet, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.conv1 = _BiasConv(self, "conv1", 3, 64, 3, 2, 0)
        self.body = []
        cin, n = 64, 2
        for f in self._FIRES:
            if f == "pool":
                self.body.append("pool")
                continue
            sq, ex, res = f
            name = "fire{}".format(n)
            self.body.append({"s1": _BiasConv(self, name + "_s1", cin, sq, 1),
                              "e1": _BiasConv(self, name + "_e1", sq, ex, 1),
                              "e3": _BiasConv(self, name + "_e3", sq, ex, 3, 1, 1),
                              "res": res})
            cin, n = 2 * ex, n + 1
        self.conv10 = _BiasConv(self, "conv10", cin, num_classes, 1, w_init="0.01")
        self.build_layout()

    def _bconv(self, x, bc, act, anchor=False):
        c = bc.conv
        return P.conv2d_bias_act(x, self.ref(c.w), self.ref(bc.b), c.stride, c.pad, act=act,
                                 anchor=self.anchor if anchor else None)

    def forward(self, x, training):
        H, W = x.shape[1], x.shape[2]
        ph, pw = same_pad(H, 3, 2), same_pad(W, 3, 2)
        x = P._zero_pad(x, (ph[0], ph[1], pw[0], pw[1]))
        x = self._bconv(x, self.conv1, 1, anchor=True)
        x = P.maxpool2d(x, 3, 2, 0)
        G = self.G
        for blk in self.body:
            if blk == "pool":
                x = P.maxpool2d(x, 3, 2, 0)
                continue
            s = self._bconv(x, blk["s1"], 1)
            e = P.cat_packed([self._bconv(s, blk["e1"], 0), self._bconv(s, blk["e3"], 0)], G)
            x = P.relu_add(e, x) if blk["res"] else torch.relu(e)
        x = self._bconv(x, self.conv10, 1)
        return P.global_avgpool(x)


class PackedDenseNetTF1(PackedNet):
    growth = 24
    blocks = (6, 12, 48, 32)

    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedDenseNetTF1, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        k = self.growth
        self.stem = Conv(self, "conv0", 3, 2 * k, 7, 2, 0)
        self.stages = []
        c = 2 * k
        for bi, n in enumerate(self.blocks):
            layers = []
            for li in range(n):
                name = "dense_{}_bottleN_{}".format(bi + 1, li)
                layers.append((Conv(self, name + "_conv1", c, 4 * k, 1),
                               Conv(self, name + "_conv2", 4 * k, k, 3, 1, 1)))
                c += k
            trans = None
            if bi < len(self.blocks) - 1:
                trans = Conv(self, "trans_{}_conv1".format(bi + 1), c, k, 1)
                c = k
            self.stages.append((layers, trans))
        self.fc = Dense(self, "logits", c, num_classes)
        self.build_layout()

    def forward(self, x, training):
        H, W = x.shape[1], x.shape[2]
        ph, pw = same_pad(H, 7, 2), same_pad(W, 7, 2)
        x = P._zero_pad(x, (ph[0], ph[1], pw[0], pw[1]))
        x = self.conv(x, self.stem, anchor=True)
        G = self.G
        for layers, trans in self.stages:
            feats = [x]
            for c1, c2 in layers:
                h = self.conv(torch.relu(x), c1)
                h = self.conv(torch.relu(h), c2)
                feats.append(h)
                x = P.cat_packed(feats, G)
            if trans is not None:
                x = self.conv(torch.relu(x), trans)
                x = P.avgpool2d(x, 2, 2)
        x = P.global_avgpool(torch.relu(x))
        return self.dense(x, self.fc)
