"""Debug: where does the state go non-finite with graph-captured validation?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime import group as G
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

orig_v, orig_t = G._Working.validate, G._Working.train_steps


def fin(w):
    torch.cuda.synchronize()
    return bool(torch.isfinite(w.arena.state).all()), bool(torch.isfinite(w.arena.work).all())


def v(self, n):
    a = fin(self)
    orig_v(self, n)
    print("validate n=%d before %s after %s vacc %s vgraph %s" % (n, a, fin(self),
          self.vacc.tolist(), self.vgraph is not None), flush=True)


def t(self, n):
    a = fin(self)
    r = orig_t(self, n)
    print("train n=%d before %s after %s acc %s graph %s" % (n, a, fin(self), self.acc.tolist(),
          self.graph is not None), flush=True)
    return r


G._Working.validate, G._Working.train_steps = v, t
bs = 8
msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": "resnet50_nobn"}
        for lr in (1e-4, 1e-5)]
graphs = os.environ.get("DBG_GRAPHS", "1") == "1"
eng = MOPEngine(msts, init_distributed(), EngineOptions(
    n_train=6 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none",
    use_graphs=graphs))
eng.run(2)
eng.close()
