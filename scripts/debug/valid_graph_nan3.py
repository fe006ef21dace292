"""Debug: capture-only vs replay of the validation graph (resnet50_nobn)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime import group as G
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

mode = sys.argv[1]
orig = G._Working.validate


def v(self, n):
    if mode == "capture_only" and self.vgraph is not None:
        g, self.vgraph = self.vgraph, None
        self.veager = True     # forces eager replays, keep the captured graph alive
        self._keep = g
    orig(self, n)


G._Working.validate = v
bs = 8
msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnet50_nobn"}
        for lr in (1e-4, 1e-5)]
eng = MOPEngine(msts, init_distributed(), EngineOptions(
    n_train=6 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none"))
eng.run(1)
print(mode, {m: (st["train_loss"], st["valid_loss"]) for m, st in eng.mst_state.items()})
