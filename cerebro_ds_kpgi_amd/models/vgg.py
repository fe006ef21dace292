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
            hw = self._pool_hw(hw)
        self.flat = hw * hw * cin
        self.fc1 = Dense(self, "fc1", self.flat, 4096)
        self.fc2 = Dense(self, "fc2", 4096, 4096)
        self.fc3 = Dense(self, "predictions", 4096, num_classes)
        self._init_specs()
        self.build_layout()

    def _pool_hw(self, hw):
        return hw // 2                # Keras default: padding='valid'

    def _init_specs(self):
        pass

    # the block's max pool finishes its last conv's ReLU / bias backward
    # (MaxPoolHip + BiasActLink); VGG16Flat's SAME pools pad, so not there
    _pool_links = True

    def _pool(self, x):
        return P.maxpool2d(x, 2, 2, 0)

    def forward(self, x, training):
        first = True
        for blk in self.convs:
            for li, (conv, bias) in enumerate(blk):
                # a conv's output feeds only the next conv (whose dgrad epilogue
                # then applies its ReLU' and bias gradient) or, last in the
                # block, only the max pool (whose backward does)
                x = P.conv2d_bias_act(x, self.ref(conv.w), self.ref(bias), conv.stride, conv.pad,
                                      act=1, anchor=self.anchor if first else None,
                                      link_out=li + 1 < len(blk) or self._pool_links)
                first = False
            x = self._pool(x)
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


class PackedVGG16Flat(PackedVGG16):
    """The reference's own ``vgg16tfk.VGG16`` (``cerebro_gpdb/vgg16tfk.py:
    44-297``, the non-default Spark model, ``run_spark.py:111-118``): flat
    ``(112*112*3,)`` input reshaped to NHWC (our packed store already holds
    NHWC, so the reshape is free), every conv and dense kernel AND bias drawn
    from TruncatedNormal(0, 0.01) (``resnet50tfk.KI``), max pools with
    ``padding='same'`` (112 -> 56 -> 28 -> 14 -> 7 -> 4), Flatten 4x4x512 =
    8192 -> fc1 4096 -> fc2 4096 -> predictions.  69 151 528 parameters."""
    KI = "tn0.01"

    def __init__(self, num_classes=1000, input_hw=112):
        super(PackedVGG16Flat, self).__init__(num_classes, input_hw)

    def _pool_hw(self, hw):
        return (hw + 1) // 2

    def _init_specs(self):
        for s in self._specs:
            if s.kind in ("weight", "bias"):
                s.init = self.KI

    def _pool(self, x):
        H = x.shape[1]
        if H % 2:                     # TF SAME: the extra row / column at the end
            x = P._zero_pad(x, (0, 1, 0, 1))     # inputs are post-ReLU (>= 0)
        return P.maxpool2d(x, 2, 2, 0)


class PackedVGG16Torchvision(PackedNet):
    """``torchvision.models.vgg16`` — the reference's PyTorch-DDP baseline
    model (``cerebro_gpdb/run_pytorchddp.py:295-299``): the same 13 conv3x3
    (+bias, ReLU) / 5 max-pool feature stack (112 -> 3), then
    AdaptiveAvgPool2d(7, 7) (a 3x3 -> 7x7 bin average here), Flatten in
    (c, h, w) order 25088 -> Linear 4096 ReLU Dropout(0.5) -> Linear 4096
    ReLU Dropout(0.5) -> Linear 1000.  138 357 544 parameters; torch default
    init (kaiming-normal fan_out convs, zero conv biases, N(0, 0.01) linears,
    zero linear biases)."""

    def __init__(self, num_classes=1000, input_hw=112, dropout=0.5):
        super(PackedVGG16Torchvision, self).__init__()
        self.num_classes = num_classes
        self.input_hw = input_hw
        self.dropout = dropout
        self.convs = []
        cin = 3
        hw = input_hw
        for bi, (c, n) in enumerate(_CFGS[16]):
            blk = []
            for li in range(n):
                idx = len(self._specs) // 2
                conv = Conv(self, "features.{}".format(idx), cin, c, 3, 1, 1)
                conv.w.fan_in = 9 * c           # kaiming_normal_(mode="fan_out")
                bias = self.spec(ParamSpec("features.{}/bias".format(idx), (c,), "bias"))
                blk.append((conv, bias))
                cin = c
            self.convs.append(blk)
            hw = hw // 2
        self.feat_hw = hw
        self.fc1 = Dense(self, "classifier.0", cin * 49, 4096, init="0.01")
        self.fc2 = Dense(self, "classifier.3", 4096, 4096, init="0.01")
        self.fc3 = Dense(self, "classifier.6", 4096, num_classes, init="0.01")
        self.build_layout()
        self._pool_mat = None

    def _adaptive_matrix(self, n_in, n_out, device):
        """Row i averages input bins [floor(i*n_in/n_out), ceil((i+1)*n_in/n_out))."""
        m = torch.zeros(n_out, n_in, device=device)
        for i in range(n_out):
            a = (i * n_in) // n_out
            b = -(-((i + 1) * n_in) // n_out)
            m[i, a:b] = 1.0 / (b - a)
        return m

    def forward(self, x, training):
        first = True
        for bi, blk in enumerate(self.convs):
            for conv, bias in blk:
                x = P.conv2d_bias_act(x, self.ref(conv.w), self.ref(bias), conv.stride, conv.pad,
                                      act=1, anchor=self.anchor if first else None)
                first = False
            x = P.maxpool2d(x, 2, 2, 0)
            nxt = bi + 1
            x = self.bucket_mark(x, self.convs[nxt][0][0].w if nxt < len(self.convs)
                                 else self.fc1.w)
        B, H, W, GC = x.shape
        G = self.G
        C = GC // G
        if self._pool_mat is None or self._pool_mat[0].device != x.device:
            self._pool_mat = (self._adaptive_matrix(H, 7, x.device),
                              self._adaptive_matrix(W, 7, x.device))
        mh, mw = self._pool_mat
        # [B, H, W, G, C] -> [B, G, C, 7, 7] -> flatten (c, h, w) per config
        t = x.view(B, H, W, G, C).permute(0, 3, 4, 1, 2).to(mh.dtype)
        t = torch.einsum("ih,bgchw,jw->bgcij", mh, t, mw)
        x = t.reshape(B, G * C * 49).to(x.dtype)
        x = self.dense(x, self.fc1, relu=True)
        if training and self.dropout:
            x = torch.nn.functional.dropout(x, self.dropout, True)
        x = self.bucket_mark(x, self.fc2.w)
        x = self.dense(x, self.fc2, relu=True)
        if training and self.dropout:
            x = torch.nn.functional.dropout(x, self.dropout, True)
        x = self.bucket_mark(x, self.fc3.w)
        return self.dense(x, self.fc3)
