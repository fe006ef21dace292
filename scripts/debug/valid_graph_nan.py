"""Debug: ResNet50-noBN engine run with the validation step graph-captured:
per-round losses and state finiteness (why does train loss go NaN?)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50_nobn"
bs = 8
msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": model}
        for lr in (1e-4, 1e-5)]
eng = MOPEngine(msts, init_distributed(), EngineOptions(
    n_train=6 * bs, n_valid=2 * bs, slots_per_gpu=2, verbose=False, ckpt_every="none"))
for grp in eng.groups.values():
    orig_v = None
for ep in range(2):
    eng.run(1) if ep == 0 else eng.run(1)
    for m, st in eng.mst_state.items():
        print("epoch", ep, "model", m, "train", st["train_loss"], "valid", st["valid_loss"])
    for key, grp in eng.groups.items():
        print("home state finite:", bool(torch.isfinite(grp.home.state).all()))
        for G, w in grp._work.items():
            print(" work G", G, "state finite", bool(torch.isfinite(w.arena.state).all()),
                  "vgraph", w.vgraph is not None, "graph", w.graph is not None)
eng.close()
