"""Debug: replay-by-replay finiteness of the nobn training graph across rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime import group as G
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

orig_t = G._Working.train_steps
rnd = [0]


def t(self, n):
    rnd[0] += 1
    done = 0
    for i in range(n):
        done += orig_t(self, 1)
        torch.cuda.synchronize()
        bad = []
        for s in self.arena.layout.specs[:400]:
            for nm, base in (("master", self.arena.master), ("grad", self.arena.grad)):
                if nm == "grad" and s.offset + s.numel > base.shape[1]:
                    continue
                v = base[:, s.offset:s.offset + s.numel]
                if not torch.isfinite(v).all():
                    bad.append(nm + ":" + s.name)
        print("round", rnd[0], "step", i, "graph", self.graph is not None, "eager_steps",
              self.eager_steps, "bad", bad[:6], "acc", [round(float(a), 2) for a in self.acc[:, 0]],
              flush=True)
    return done


G._Working.train_steps = t
bs = 8
msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnet50_nobn"}
        for lr in (1e-4, 1e-5)]
eng = MOPEngine(msts, init_distributed(), EngineOptions(
    n_train=6 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none"))
eng.run(2)
