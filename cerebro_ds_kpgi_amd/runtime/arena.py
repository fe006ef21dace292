"""Flat per-configuration parameter arenas.

One *model state row* holds everything a configuration owns, contiguously:

    [ master fp32 params (trainable) | buffers fp32 (BN running stats) |
      adam m | adam v | step + pad ]

so a model hop is ONE contiguous buffer -> one RCCL send/recv, and a
checkpoint is one copy.  A GPU that trains G packed configurations owns a
``[G, R]`` fp32 state tensor plus:

* ``work``  ``[G, n_train]`` compute-dtype shadow of the master params
  (bf16 by default), refreshed by the fused optimizer kernel,
* ``grad``  ``[G, n_train]`` fp32 gradients, written *directly* by the
  weight-gradient kernels (no autograd AccumulateGrad pass),
* ``whl``   ``[G, n_train]`` (fp32 mode, training working sets on the HIP
  path: ``enable_whl``) the params in HL format -- every 8 as [8 x bf16 hi |
  8 x bf16 lo], the operand split of the 3-pass fp32 conv kernels -- written
  by the optimizer kernel next to the params and read by the conv / linear
  GEMMs instead of splitting the weights in their K loops,
* ``lr``/``wd`` ``[G]`` per-config hyper-parameters on device.

The weight blob order follows the model's layer order and is the same as the
reference's ``serialize_nd_weights`` flat float32 concatenation
(``cerebro_gpdb/madlib_keras_wrapper.py:119-131``) for the params of our
architecture.
"""

import math

import numpy as np
import torch

ALIGN = 64  # elements: every tensor starts 256-B aligned in fp32, 128-B in bf16


class ParamSpec(object):
    """One tensor of one configuration.  ``fmt`` names how our storage order
    maps to the Keras ``get_weights()`` array of the same tensor:

    * ``conv``  ours (cout, kh, kw, cin)  -> Keras HWIO (kh, kw, cin, cout),
    * ``dense`` ours (cout, cin)          -> Keras (cin, cout),
    * ``dw``    ours (c, kh, kw)          -> Keras depthwise (kh, kw, c, 1),
    * ``keras`` already in Keras order (biases, BN vectors, ...).

    ``auto`` picks conv for 4-D weights, dw for 3-D weights, dense for 2-D
    weights and keras otherwise."""
    __slots__ = ("name", "shape", "kind", "init", "fan_in", "offset", "numel", "fmt")

    def __init__(self, name, shape, kind="weight", init="he", fan_in=None, fmt="auto"):
        self.name = name
        self.shape = tuple(int(s) for s in shape)
        self.kind = kind          # weight | bias | gamma | beta | running_mean | running_var
        self.init = init
        self.fan_in = fan_in
        self.numel = int(np.prod(self.shape))
        self.offset = None
        if fmt == "auto":
            nd = len(self.shape)
            fmt = ({4: "conv", 3: "dw", 2: "dense"}.get(nd, "keras") if kind == "weight"
                   else "keras")
        self.fmt = fmt

    @property
    def trainable(self):
        return self.kind not in ("running_mean", "running_var")

    # ---- Keras get_weights() order (reference serialize_nd_weights blobs) ----
    @property
    def keras_shape(self):
        s = self.shape
        if self.fmt == "conv":
            return (s[1], s[2], s[3], s[0])
        if self.fmt == "dense":
            return (s[1], s[0])
        if self.fmt == "dw":
            return (s[1], s[2], s[0], 1)
        return s

    def to_keras(self, flat):
        """Our flat storage (numpy) -> the Keras-shaped array."""
        a = np.asarray(flat).reshape(self.shape)
        if self.fmt == "conv":
            return np.ascontiguousarray(a.transpose(1, 2, 3, 0))
        if self.fmt == "dense":
            return np.ascontiguousarray(a.transpose(1, 0))
        if self.fmt == "dw":
            return np.ascontiguousarray(a.transpose(1, 2, 0))[..., None]
        return a

    def from_keras(self, arr):
        """Keras-shaped array -> our flat storage order (numpy, 1-D)."""
        a = np.asarray(arr, np.float32)
        if tuple(a.shape) != self.keras_shape:
            raise ValueError("{}: Keras shape {} != {}".format(self.name, a.shape,
                                                              self.keras_shape))
        if self.fmt == "conv":
            a = a.transpose(3, 0, 1, 2)
        elif self.fmt == "dense":
            a = a.transpose(1, 0)
        elif self.fmt == "dw":
            a = a[..., 0].transpose(2, 0, 1)
        return np.ascontiguousarray(a).reshape(-1)


class KerasBias(object):
    """A conv bias Keras has and we drop (the conv feeds a training-mode
    BatchNorm, whose batch-mean subtraction cancels it exactly).  Serialised
    as zeros; a non-zero bias read from a Keras blob is folded into the BN's
    moving mean (``fold_into``), which is where Keras accumulated it."""
    __slots__ = ("name", "shape", "fold_into")

    def __init__(self, name, cout, fold_into):
        self.name = name
        self.shape = (int(cout),)
        self.fold_into = fold_into

    @property
    def keras_shape(self):
        return self.shape


def _align(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


class ModelLayout(object):
    """Ordered parameter specs of ONE configuration + their arena offsets."""

    def __init__(self, specs, keras_extra=None, keras_order=None):
        self.train_specs = [s for s in specs if s.trainable]
        self.buffer_specs = [s for s in specs if not s.trainable]
        off = 0
        for s in self.train_specs:
            s.offset = off
            off += _align(s.numel)
        self.n_train = off
        for s in self.buffer_specs:
            s.offset = off
            off += _align(s.numel)
        self.n_master = off
        self.by_name = {s.name: s for s in specs}
        self.specs = list(specs)
        # Keras get_weights() entries: our specs (in ``keras_order`` when the
        # architecture's Keras layer order differs from ours) plus the
        # dropped conv biases, each right after its kernel
        order = list(keras_order) if keras_order else [s.name for s in specs]
        assert sorted(order) == sorted(self.by_name), "keras_order must list every spec once"
        extra = dict(keras_extra or {})
        self.keras_entries = []
        for n in order:
            self.keras_entries.append(self.by_name[n])
            if n in extra:
                self.keras_entries.append(extra[n])

    @property
    def num_params(self):
        """Trainable parameter count (unpadded)."""
        return sum(s.numel for s in self.train_specs)

    def row_len(self, with_optimizer=True):
        if not with_optimizer:
            return self.n_master
        return self.n_master + 2 * self.n_train + ALIGN

    # offsets of the sections inside a state row
    @property
    def off_m(self):
        return self.n_master

    @property
    def off_v(self):
        return self.n_master + self.n_train

    @property
    def off_step(self):
        return self.n_master + 2 * self.n_train


def init_row(layout, master_row, seed):
    """Deterministic per-config initialisation of one master row (fp32 tensor).

    Drawn on the row's device so every rank produces the same initial weights
    for the same seed without a host round trip.
    """
    dev = master_row.device
    g = torch.Generator(device=dev if dev.type == "cuda" else "cpu")
    g.manual_seed(int(seed))
    master_row.zero_()
    for s in layout.specs:
        view = master_row[s.offset:s.offset + s.numel]
        if isinstance(s.init, str) and s.init.startswith("tn"):
            # Keras TruncatedNormal(0, std): normal redrawn outside +-2 std
            # (reference resnet50tfk.py KI, kernels AND biases)
            std = float(s.init[2:])
            t = torch.empty(s.numel, device=dev).normal_(0.0, 1.0, generator=g)
            while True:
                bad = t.abs() > 2.0
                nb = int(bad.sum())
                if not nb:
                    break
                t[bad] = torch.empty(nb, device=dev).normal_(0.0, 1.0, generator=g)
            view.copy_(t * std)
            continue
        if isinstance(s.init, str) and s.init.startswith("const"):
            view.fill_(float(s.init[5:]))      # e.g. TF constant_initializer(0.1) biases
            continue
        if s.kind in ("weight",):
            fan_in = s.fan_in if s.fan_in else int(np.prod(s.shape[1:]))
            if s.init == "he":
                std = math.sqrt(2.0 / fan_in)
            elif s.init == "glorot":
                fan_out = s.shape[0]
                std = math.sqrt(2.0 / (fan_in + fan_out))
            else:
                std = float(s.init)
            view.normal_(0.0, std, generator=g)
        elif s.kind in ("gamma", "running_var"):
            view.fill_(1.0)
        else:  # bias, beta, running_mean
            view.fill_(0.0)


class Arena(object):
    """State of G packed configurations of one architecture on one device."""

    def __init__(self, layout, G, device, compute_dtype=torch.bfloat16, trainable=True):
        self.layout = layout
        self.G = G
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        R = layout.row_len(True)
        self.state = torch.zeros(G, R, dtype=torch.float32, device=self.device)
        L = layout
        self.master = self.state[:, :L.n_master]
        self.params = self.state[:, :L.n_train]
        self.m = self.state[:, L.off_m:L.off_m + L.n_train]
        self.v = self.state[:, L.off_v:L.off_v + L.n_train]
        self.step = self.state[:, L.off_step:L.off_step + 1]
        # a "home" arena only parks states between rounds: no work/grad copies
        if compute_dtype == torch.float32 or not trainable:
            self.work = self.params
        else:
            self.work = torch.zeros(G, L.n_train, dtype=compute_dtype, device=self.device)
        self.grad = (torch.zeros(G, L.n_train, dtype=torch.float32, device=self.device)
                     if trainable else None)
        # True: the optimizer clears ``grad`` after consuming it, so every
        # backward starts from zeros (split-K weight-gradient kernels then
        # accumulate without a per-layer memset)
        self.grad_clean = False
        self.whl = None
        self.lr = torch.zeros(G, dtype=torch.float32, device=self.device)
        self.wd = torch.zeros(G, dtype=torch.float32, device=self.device)
        self.model_ids = [None] * G

    # ---- views -----------------------------------------------------------
    def _view(self, base, spec):
        return base[:, spec.offset:spec.offset + spec.numel].view(self.G, *spec.shape)

    def work_view(self, spec):
        return self._view(self.work, spec)

    def master_view(self, spec):
        return self._view(self.master, spec)

    def grad_view(self, spec):
        return self._view(self.grad, spec)

    # ---- state management -------------------------------------------------
    def init_model(self, row, seed):
        init_row(self.layout, self.master[row], seed)
        self.m[row].zero_()
        self.v[row].zero_()
        self.step[row].zero_()
        self.sync_work(row)

    def enable_whl(self):
        """Keep an HL image of the params (fp32 working sets on the HIP
        path): refreshed by ``sync_work`` and written by every optimizer
        step; the uniform-K conv kernels read it (conv.hip cer_conv_set_whl)."""
        if self.whl is None and self.compute_dtype == torch.float32 and self.grad is not None:
            self.whl = torch.zeros(self.G, self.layout.n_train, dtype=torch.float32,
                                   device=self.device)
            self.sync_work()
        return self.whl is not None

    def sync_work(self, row=None):
        if self.whl is not None:
            from ..ops import _hip
            _hip.hl_image(self.params if row is None else self.params[row:row + 1],
                          self.whl if row is None else self.whl[row:row + 1])
        if self.work is self.params:
            return
        if row is None:
            self.work.copy_(self.params)
        else:
            self.work[row].copy_(self.params[row])

    def reset_optimizer(self, row=None):
        sl = slice(None) if row is None else slice(row, row + 1)
        self.m[sl].zero_()
        self.v[sl].zero_()
        self.step[sl].zero_()

    def set_hparams(self, row, lr, wd):
        self.lr[row] = float(lr)
        self.wd[row] = float(wd)

    def row_weights_f32(self, row):
        """Flat float32 weight blob in the Keras ``serialize_nd_weights``
        layout (``runtime.serialize.master_to_keras``)."""
        from .serialize import master_to_keras
        master = self.master[row].detach().cpu().numpy()
        return np.concatenate([a.reshape(-1) for a in master_to_keras(self.layout, master)])

    def load_row_weights_f32(self, row, blob):
        from .serialize import blob_to_master
        self.master[row].copy_(torch.from_numpy(blob_to_master(self.layout,
                                                               np.asarray(blob, np.float32)))
                               .to(self.device))
        self.sync_work(row)


class ParamRef(object):
    """Handle to one parameter of all G packed configs (passed to ops)."""
    __slots__ = ("arena", "spec")

    def __init__(self, arena, spec):
        self.arena = arena
        self.spec = spec

    @property
    def G(self):
        return self.arena.G

    def work(self):
        return self.arena.work_view(self.spec)

    def grad(self):
        return self.arena.grad_view(self.spec)

    def master(self):
        return self.arena.master_view(self.spec)

    # raw addressing for HIP kernels: base pointer + per-config stride (elements)
    def work_ptr(self):
        w = self.arena.work
        return w.data_ptr() + self.spec.offset * w.element_size(), w.stride(0)

    def whl_ptr(self):
        """(pointer, per-config stride) of this param's HL image, or (0, 0)."""
        h = self.arena.whl
        if h is None:
            return 0, 0
        return h.data_ptr() + self.spec.offset * h.element_size(), h.stride(0)

    def grad_ptr(self):
        g = self.arena.grad
        return g.data_ptr() + self.spec.offset * g.element_size(), g.stride(0)

    def master_ptr(self):
        m = self.arena.master
        return m.data_ptr() + self.spec.offset * m.element_size(), m.stride(0)
