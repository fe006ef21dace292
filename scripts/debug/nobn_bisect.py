"""Bisect the ResNet50-noBN graph-replay NaN: model variants, replay by replay."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from cerebro_ds_kpgi_amd.models import zoo
from cerebro_ds_kpgi_amd.ops import nn as P
from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime import group as G
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

variant = sys.argv[1]
zoo.PackedResNet50NoBN.graph_safe = True
orig_fwd = zoo.PackedResNet50NoBN.forward


def fwd(self, x, training):
    x = self._cba(x, self.conv1, 1, anchor=True)
    if variant != "nopool":
        x = P.maxpool2d(x, 3, 2, 1)
    for i, blk in enumerate(self.blocks):
        if variant in ("noblocks", "pad3", "pad2", "pad1") and i > 0:
            break
        if variant.startswith("nb") and i >= int(variant[2:]):
            break
        sc = self._cba(x, blk["cs"], 0) if "cs" in blk else x
        h = self._cba(x, blk["c1"], 1)
        h = self._cba(h, blk["c2"], 1)
        h = self._cba(h, blk["c3"], 0)
        if variant == "plainadd":
            x = torch.relu(h + sc)
        elif variant == "nores":
            x = torch.relu(h)
        else:
            x = P.relu_add(h, sc)
    if variant == "noblocks":
        x = self._cba(x, self.blocks[-1]["c3"], 0) if False else x
    x = P.global_avgpool(x)
    if variant in ("noblocks", "pad3", "pad2", "pad1") or variant.startswith("nb"):
        x = torch.nn.functional.pad(x, (0, self.G * 2048 - x.shape[1])) if x.shape[1] != self.G * 2048 else x
    return self.dense(x, self.fc)


if variant.startswith("pad"):
    _orig_init = zoo.PackedResNet50NoBN.__init__

    def _init(self, *a, **k):
        _orig_init(self, *a, **k)
        self.conv1.pad = int(variant[3:])
    zoo.PackedResNet50NoBN.__init__ = _init
    zoo.PackedResNet50NoBN.forward = fwd
    variant_fwd = "noblocks"
if variant == "heinit":
    zoo.PackedResNet50NoBN.KI = "he"
elif variant == "anchorless":
    pass
elif variant != "orig":
    zoo.PackedResNet50NoBN.forward = fwd
if variant.startswith("nb"):
    zoo.PackedResNet50NoBN.forward = fwd
if os.environ.get("DBG_PIN"):
    from cerebro_ds_kpgi_amd.ops import _hip
    for kv in os.environ["DBG_PIN"].split(","):
        op, v = kv.split(":")
        _hip.conv_set_variant(int(op), int(v))
orig_t = G._Working.train_steps
state = {"first_bad": None, "step": 0}


def t(self, n):
    done = 0
    for _ in range(n):
        done += orig_t(self, 1)
        torch.cuda.synchronize()
        state["step"] += 1
        if state["first_bad"] is None and not torch.isfinite(self.arena.master).all():
            state["first_bad"] = state["step"]
    return done


G._Working.train_steps = t
msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": 8,
         "model": os.environ.get("DBG_MODEL", "resnet50_nobn")}
        for lr in (1e-4, 1e-5)]
eng = MOPEngine(msts, init_distributed(), EngineOptions(
    n_train=48, n_valid=16, slots_per_gpu=2, verbose=False, ckpt_every="none"))
for grp in eng.groups.values():
    grp.warmup_eager = int(os.environ.get("DBG_WARM", grp.warmup_eager))
eng.run(1)
print("variant", variant, "first non-finite step", state["first_bad"], "of", state["step"])
