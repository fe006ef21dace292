"""Minimal packed-model building blocks.

A ``PackedNet`` declares its per-configuration parameters (``ParamSpec``) at
construction, is ``bind``-ed to an ``Arena`` holding G configurations, and
runs forward on packed NHWC activations ``[B, H, W, G*C]`` through
``ops.nn``.  Autograd drives backward; the ops write weight gradients
straight into the arena.
"""

import os

import torch

from ..ops import nn as P
from ..runtime.arena import KerasBias, ModelLayout, ParamRef, ParamSpec


class Conv(object):
    def __init__(self, net, name, cin, cout, k, stride=1, pad=0):
        self.cin, self.cout, self.k, self.stride, self.pad = cin, cout, k, stride, pad
        self.w = net.spec(ParamSpec(name + "/kernel", (cout, k, k, cin), "weight",
                                    fan_in=k * k * cin))

    def out_hw(self, h):
        return (h + 2 * self.pad - self.k) // self.stride + 1


class BN(object):
    def __init__(self, net, name, c):
        self.g = net.spec(ParamSpec(name + "/gamma", (c,), "gamma"))
        self.b = net.spec(ParamSpec(name + "/beta", (c,), "beta"))
        self.rm = net.spec(ParamSpec(name + "/moving_mean", (c,), "running_mean"))
        self.rv = net.spec(ParamSpec(name + "/moving_variance", (c,), "running_var"))


class Dense(object):
    def __init__(self, net, name, cin, cout, init="glorot"):
        self.w = net.spec(ParamSpec(name + "/kernel", (cout, cin), "weight", init=init, fan_in=cin))
        self.b = net.spec(ParamSpec(name + "/bias", (cout,), "bias"))


class PackedNet(object):
    input_kind = "image"      # image | sparse
    num_classes = 1000
    input_hw = 112
    input_c = 3
    # False: the engine runs this architecture's step eagerly instead of
    # replaying a captured HIP graph (runtime.group)
    graph_safe = True

    def __init__(self):
        self._specs = []
        self._keras_extra = {}      # kernel spec name -> KerasBias (runtime.arena)
        self.keras_order = None     # Keras get_weights() order when it differs from ours
        self.arena = None
        # runtime.baselines.GradBuckets while DDP trains this net (bucket marks)
        self.grad_buckets = None
        self.bn_momentum = 0.1
        self.bn_eps = 1e-5
        # BN backward partials in consumer dgrad epilogues (ops.nn.BNLink)
        self.bn_links = os.environ.get("CER_BN_LINKS", "1") != "0"

    def spec(self, s):
        self._specs.append(s)
        return s

    def drop_bias(self, conv, bn):
        """``conv`` has a bias in the Keras model that we do not store (it
        feeds ``bn``); serialised blobs still carry it (as zeros)."""
        name = conv.w.name.rsplit("/", 1)[0] + "/bias"
        self._keras_extra[conv.w.name] = KerasBias(name, conv.cout, bn.rm.name)

    def build_layout(self):
        self.layout = ModelLayout(self._specs, self._keras_extra, self.keras_order)
        return self.layout

    def bind(self, arena):
        self.arena = arena
        self.anchor = torch.zeros((), device=arena.device, requires_grad=True)

    @property
    def G(self):
        return self.arena.G

    def ref(self, spec):
        return ParamRef(self.arena, spec)

    # helpers used by architectures
    def conv(self, x, c, anchor=False):
        return P.conv2d(x, self.ref(c.w), c.stride, c.pad, self.anchor if anchor else None)

    def bn(self, x, b, training, relu=True, residual=None, link_out=False):
        """``link_out``: the output's only consumer is the next ``conv_bn``,
        whose dgrad epilogue then computes this BN's backward partials."""
        return P.bn_act(x, self.ref(b.g), self.ref(b.b), self.ref(b.rm), self.ref(b.rv),
                        training, relu, residual, self.bn_momentum, self.bn_eps,
                        link_out and self.bn_links)

    def conv_bn(self, x, c, b, training, relu=True, residual=None, anchor=False, join=None,
                res_join=None, link_out=False, hl_out=False):
        """act(BN(conv(x)) + residual); in training the conv epilogue feeds BN
        its batch statistics (ops.nn.PackedConvBNAct).  ``join`` / ``res_join``:
        a ``P.GradJoin`` shared with the other consumer of ``x`` / ``residual``
        (the two input gradients are summed in a dgrad epilogue).  ``hl_out``:
        the output's only consumer is the next ``conv_bn`` (HL operand format,
        ops.nn.conv_bn_act)."""
        if not training:
            return self.bn(self.conv(x, c, anchor), b, training, relu, residual)
        return P.conv_bn_act(x, self.ref(c.w), self.ref(b.g), self.ref(b.b), self.ref(b.rm),
                             self.ref(b.rv), c.stride, c.pad, relu, residual, self.bn_momentum,
                             self.bn_eps, self.anchor if anchor else None, join, res_join,
                             link_out and self.bn_links, hl_out)

    def bucket_mark(self, x, first_spec_above):
        """Gradient-bucket boundary: in backward, once the gradient reaches
        here, the gradients of every parameter from ``first_spec_above`` on
        (arena order = forward order) are final and may be all-reduced while
        the layers below run their backward."""
        gb = self.grad_buckets
        if gb is None or not torch.is_grad_enabled():
            return x
        off = first_spec_above.offset
        return P.grad_mark(x, lambda: gb.ready_from(off))

    def dense(self, x, d, relu=False, anchor=False):
        return P.linear(x, self.ref(d.w), self.ref(d.b), relu, self.anchor if anchor else None)

    def forward(self, x, training):
        raise NotImplementedError
