"""Entry points, schedule() facade, baselines and async TPE over MOP (CPU)."""

import json
import os

import pytest

os.environ.setdefault("CEREBRO_BACKEND", "torch")


def _ctx():
    from cerebro_ds_kpgi_amd.parallel import init_distributed
    return init_distributed(device_type="cpu")


def _tiny(n=2, lrs=(1e-3, 1e-2, 3e-3, 2e-3)):
    return [{"learning_rate": lrs[i], "lambda_value": 1e-4, "batch_size": 8, "model": "tinycnn"}
            for i in range(n)]


def test_run_mop_cli_writes_global_log(tmp_path):
    from cerebro_ds_kpgi_amd.runners import run_mop
    logs = tmp_path / "run_logs" / "cerebro"
    run_mop.main(["--run", "--tiny", "--num_epochs", "1", "--train_per_partition", "32",
                  "--valid_per_partition", "16", "--compute_dtype", "fp32", "--backend", "torch",
                  "--logs_root", str(logs), "--models_root", str(tmp_path / "models")])
    g = (tmp_path / "run_logs" / "global.log").read_text().splitlines()
    assert g[0].startswith("udaf, Start time:") and g[1].startswith("udaf, End time:")
    assert g[2].startswith("udaf, TOTAL EXECUTION TIME OVER ALL MST ")
    summ = json.loads((logs / "summary.json").read_text())
    assert summ["configs"] == 2 and summ["train_images"] == 2 * 2 * 32


def test_schedule_facade_grid_search(tmp_path):
    from cerebro_ds_kpgi_amd.api import schedule
    from cerebro_ds_kpgi_amd.selection.hyperopt_helper import mst_eval_fn
    state = schedule(data_set_name="tiny", initial_msts=_tiny(3), mst_eval_fn=mst_eval_fn(2),
                     ckpt_root=str(tmp_path / "ck"), log_files_root=str(tmp_path / "lg"),
                     ctx=_ctx(), n_train=32, n_valid=16, compute_dtype="fp32", verbose=False,
                     slots_per_gpu=2)
    assert all(len(s["train_loss"]) == 2 and s["state"] == "COMPLETED" for s in state.values())


def test_schedule_custom_model_fn_and_train_fn(tmp_path):
    """A custom model_fn(mst) -> PackedNet is registered and trained; a
    Keras-style closure or a custom train_fn fails loudly."""
    from cerebro_ds_kpgi_amd.api import schedule
    from cerebro_ds_kpgi_amd.models.small import PackedTinyCNN
    from cerebro_ds_kpgi_amd.selection.hyperopt_helper import mst_eval_fn

    class Wide(PackedTinyCNN):
        pass

    built = []

    def model_fn(mst):
        built.append(mst["learning_rate"])
        return Wide()
    kw = dict(data_set_name="tiny", initial_msts=_tiny(2), mst_eval_fn=mst_eval_fn(1),
              ctx=_ctx(), n_train=32, n_valid=16, compute_dtype="fp32", verbose=False,
              slots_per_gpu=2)
    state = schedule(model_fn=model_fn, **kw)
    assert len(built) >= 2 and all(len(s["train_loss"]) == 1 for s in state.values())
    with pytest.raises(NotImplementedError):
        schedule(train_fn=lambda *a: None, **kw)
    with pytest.raises(TypeError):
        schedule(model_fn=lambda generator: (lambda data, mst, purpose: None), **dict(
            kw, initial_msts=[dict(m, model=None) for m in _tiny(1)]))


def test_async_tpe_over_mop():
    """Cerebro-hyperopt contract: configs finishing their epochs report to TPE
    and new configs join the running MOP until max_num_config."""
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    from cerebro_ds_kpgi_amd.selection import hyperopt_helper as hh
    grid = {"learning_rate": [1e-4, 1e-1], "lambda_value": [1e-4], "batch_size": [8, 8],
            "model": ["tinycnn"]}

    class A:
        size = 2
    hp, msts, trials, domain, rand, _ = hh.init_hyperopt(grid, A())
    eng = MOPEngine(msts, _ctx(), EngineOptions(n_train=32, n_valid=16, compute_dtype="fp32",
                                                verbose=False, ckpt_every="none",
                                                slots_per_gpu=2))
    fn = hh.mst_eval_fn_hyperopt(1, hp, trials, domain, 6, rand, 2, param_grid=grid)
    eng.run(10, mst_eval_fn=fn)
    assert len(eng.msts) == 6
    assert all(s["state"] == "COMPLETED" for s in eng.mst_state.values())
    assert len(trials.completed()) == 6


def test_ctq_hyperopt_batches(tmp_path):
    """CTQ-Hyperopt: batches of `concurrency` configs, one MOP session each,
    every trial reported before the next batch is proposed."""
    import argparse
    import pickle
    from cerebro_ds_kpgi_amd.runners.common import run_batched_hyperopt
    grid = {"learning_rate": [1e-4, 1e-1], "lambda_value": [1e-4], "batch_size": [8, 8],
            "model": ["tinycnn"]}
    args = argparse.Namespace(concurrency=2, size=2, max_num_config=5, num_epochs=1,
                              logs_root=str(tmp_path), criteo=False)
    ctx = _ctx()
    import cerebro_ds_kpgi_amd.runners.common as C
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions
    orig = C._opts
    C._opts = lambda a, sched, loader: EngineOptions(
        scheduler=sched, n_train=32, n_valid=16, compute_dtype="fp32", verbose=False,
        ckpt_every="none", slots_per_gpu=2)
    try:
        run = run_batched_hyperopt(args, ctx, None, param_grid=grid)
    finally:
        C._opts = orig
    assert len(run.msts) == 5 and len(run.mst_state) == 5
    assert all(len(s["valid_loss"]) == 1 for s in run.mst_state.values())
    with open(os.path.join(str(tmp_path), "models_info_grand.pkl"), "rb") as f:
        assert sorted(pickle.load(f)) == [0, 1, 2]          # batches of 2, 2, 1


@pytest.mark.parametrize("engine", ["ma", "ddp", "task"])
def test_baseline_engines_train(engine, tmp_path):
    from cerebro_ds_kpgi_amd.runtime.baselines import DDPEngine, MAEngine
    from cerebro_ds_kpgi_amd.runtime.engine import EngineOptions, MOPEngine
    # logs_root: the run manifest is written too (task parallel once failed there)
    o = EngineOptions(n_train=64, n_valid=16, compute_dtype="fp32", verbose=False,
                      ckpt_every="none", scheduler="task" if engine == "task" else "rotation",
                      partitions=2, logs_root=str(tmp_path))
    cls = {"ma": MAEngine, "ddp": DDPEngine, "task": MOPEngine}[engine]
    eng = cls(_tiny(2), _ctx(), o)
    eng.run(3)
    for st in eng.mst_state.values():
        assert len(st["train_loss"]) == 3
        assert st["train_loss"][-1] < st["train_loss"][0]


def test_log_analyzer_breakdown(tmp_path):
    """--trace run -> analyzer reproduces makespan + breakdown categories."""
    from cerebro_ds_kpgi_amd.runners import run_da_cerebro_standalone as r
    from cerebro_ds_kpgi_amd.tools import log_analyzer as la
    logs = tmp_path / "run_logs" / "da"
    r.main(["--run", "--tiny", "--num_epochs", "2", "--train_per_partition", "32",
            "--valid_per_partition", "16", "--compute_dtype", "fp32", "--backend", "torch",
            "--trace", "--logs_root", str(logs), "--models_root", str(tmp_path / "models")])
    res = la.main(["--logs_root", str(logs), "--json", str(tmp_path / "a.json")])
    assert res["exp"] and res["makespan_s"] > 0
    bd = res["breakdown"]
    assert set(bd["gpu_seconds"]) == set(la.CATEGORIES)
    assert bd["gpu_seconds"]["train_valid"] > 0 and sorted(bd["per_epoch"]) == [1, 2]
    assert abs(sum(bd["fraction"].values()) - 1.0) < 1e-6 or bd["gpu_seconds"]["idle"] == 0
    # lock-step runs trace a hop phase, asynchronous runs the exposed arrival wait
    names = set(res["trace_seconds"])
    assert {"train", "valid"} <= names and names & {"hop", "wait_arrival"}
    assert res["best"]["epochs"] == [1, 2]
    assert list(res["system"].values())[0]["seconds"] >= 0


def _store_digest(t):
    import hashlib
    return hashlib.sha1(t.contiguous().cpu().numpy().tobytes()).hexdigest()


def test_schedule_filesystem_input_fn_trains_on_those_partitions(tmp_path, monkeypatch):
    """the reference's filesystem entry point passes
    ``input_fn`` / ``input_fn_criteo`` with a ``DATA_CATALOG``
    (``run_filesystem_cerebro_standalone.py:24-51,85-98``); schedule() must
    load exactly those partitions (store bytes == the files' bytes), and an
    unknown input_fn must raise instead of training on synthetic data."""
    import numpy as np
    from cerebro_ds_kpgi_amd.api import schedule
    from cerebro_ds_kpgi_amd.data import fs
    from cerebro_ds_kpgi_amd.runtime import engine as engine_mod
    from cerebro_ds_kpgi_amd.selection.hyperopt_helper import mst_eval_fn
    root = str(tmp_path / "criteo")
    cat = fs.write_fs_dataset(root, "criteo", 2, 48, 16)
    seen = {}
    orig_close = engine_mod.MOPEngine.close

    def spy_close(self):
        seen["train_x"] = _store_digest(self.store.train_x)
        seen["train_y"] = _store_digest(self.store.train_y)
        seen["P"] = self.P
        orig_close(self)
    monkeypatch.setattr(engine_mod.MOPEngine, "close", spy_close)
    msts = [{"learning_rate": lr, "lambda_value": 1e-4, "batch_size": 16, "model": "confA"}
            for lr in (1e-3, 1e-4)]
    state = schedule(data_set_name="criteo", input_fn=fs.input_fn_criteo,
                     initial_msts=msts, mst_eval_fn=mst_eval_fn(1),
                     data_catalog={"criteo": cat}, ctx=_ctx(), compute_dtype="fp32",
                     verbose=False, ckpt_every="none")
    assert all(len(s["train_loss"]) == 1 for s in state.values())
    # what the files hold, through the reference's own input_fn contract
    want_x, want_y = [], []
    for i in range(2):
        ref = fs.input_fn_criteo(os.path.join(root, cat["train"][i]))
        want_x.append(fs._criteo_ids(ref["images"]))
        want_y.append(ref["labels"].argmax(1).astype(np.int32))
    import torch
    assert seen["P"] == 2
    assert seen["train_x"] == _store_digest(torch.from_numpy(np.stack(want_x)))
    assert seen["train_y"] == _store_digest(torch.from_numpy(np.stack(want_y)))
    # a catalog data_root alone selects the same source
    schedule(initial_msts=msts[:1], mst_eval_fn=mst_eval_fn(1), data_catalog=cat,
             ctx=_ctx(), compute_dtype="fp32", verbose=False, ckpt_every="none")
    assert seen["train_x"] == _store_digest(torch.from_numpy(np.stack(want_x)))

    def my_input_fn(path):
        return None
    with pytest.raises(ValueError, match="unsupported input_fn"):
        schedule(input_fn=my_input_fn, initial_msts=msts, data_catalog=cat, ctx=_ctx())
    with pytest.raises(ValueError, match="data_root"):
        schedule(input_fn=fs.input_fn, initial_msts=msts, ctx=_ctx())
    with pytest.raises(ValueError, match="neither"):
        schedule(initial_msts=msts, data_catalog={"data_root": str(tmp_path)}, ctx=_ctx())
