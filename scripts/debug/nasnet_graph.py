"""Bisect the NASNet HIP-graph NaN by forcing op families to the torch path."""
import torch
from cerebro_ds_kpgi_amd.ops import backend
from cerebro_ds_kpgi_amd.parallel import init_distributed
from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine

backend.set_backend("hip")
ctx = init_distributed()
for force in ([], ["dwconv"], ["bn"], ["conv"], ["pool"], ["conv", "bn", "dwconv", "pool", "linear"]):
    backend.force_torch_ops(force)
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": 4, "model": "nasnetmobile"}
            for lr in (1e-4, 1e-5)]
    eng = MOPEngine(msts, ctx, EngineOptions(n_train=24, n_valid=4, slots_per_gpu=2, verbose=False,
                                             ckpt_every="none", use_graphs=True))
    eng.run(1)
    print("force", force, {m: st["train_loss"] for m, st in eng.mst_state.items()}, flush=True)
    eng.close()
