"""Determinism check: eager x2 and graph x2 engine runs of one model (losses)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

model, bs = sys.argv[1], int(sys.argv[2])
msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": bs, "model": model}
        for lr in (1e-4, 1e-5)]
ctx = init_distributed()
for graphs in (False, False, True, True):
    eng = MOPEngine(msts, ctx, EngineOptions(n_train=8 * bs, n_valid=2 * bs, slots_per_gpu=2,
                                             verbose=False, ckpt_every="none", use_graphs=graphs))
    eng.run(2)
    print("graphs" if graphs else "eager ", [[round(v, 4) for v in st["train_loss"] + st["valid_loss"]]
                                             for st in eng.mst_state.values()], flush=True)
    eng.close()
