"""Cerebro-compatible front door: ``schedule(...)``.

Same keyword signature as the external Cerebro standalone scheduler the
reference drives (``cerebro_gpdb/run_da_cerebro_standalone.py:84-120``,
``run_filesystem_cerebro_standalone.py:85-98``):

    schedule(data_set_name, input_fn, model_fn, train_fn, initial_msts,
             mst_eval_fn, ckpt_root, preload_data_to_mem, log_files_root,
             backend, data_catalog, workers=None, save_every=False)

On MI355X the data plane, the model and the train step are the framework's
own (HBM partition store, packed HIP models, fused step), so:

* ``input_fn`` selects the data source: ``data.da.input_fn`` (or a catalog
  whose ``data_root`` holds a DA manifest) -> Direct-Access pages; anything
  else / ``None`` -> synthetic partitions of the dataset's shape;
* ``model_fn`` / ``train_fn`` are accepted for source compatibility; the
  model is built from each MST's ``model`` name (``models.registry``) and
  trained by the native step.  A custom callable logs a notice;
* ``workers`` / ``backend`` are accepted; the GPUs of the torchrun world are
  the workers; ``preload_data_to_mem`` is always true (HBM-resident);
* ``mst_eval_fn(mst_state) -> (stop_list, update_list, new_msts)`` is called
  after every epoch exactly like Cerebro's, so grid search
  (``selection.hyperopt_helper.mst_eval_fn``) and async TPE
  (``mst_eval_fn_hyperopt``) work unchanged.

Returns ``mst_state`` (per-config train/valid loss and error lists).
"""

import os

from .data.catalog import make_data_catalog
from .parallel import init_distributed
from .runtime.engine import EngineOptions, MOPEngine
from .utils.logging import logs


def _catalog_root(data_catalog):
    """``data_root`` of a Cerebro catalog ({name: {...}} or the inner dict)."""
    if not data_catalog:
        return ""
    inner = data_catalog
    if "data_root" not in inner and len(inner) == 1:
        inner = next(iter(inner.values()))
    return inner.get("data_root", "")


def _is_da(input_fn, data_catalog):
    from .data.da import MANIFEST
    if input_fn is not None and getattr(input_fn, "__module__", "").endswith("data.da"):
        return True
    root = _catalog_root(data_catalog)
    return bool(root) and os.path.exists(os.path.join(root, MANIFEST))


def schedule(data_set_name=None, input_fn=None, model_fn=None, train_fn=None,
             initial_msts=None, mst_eval_fn=None, ckpt_root="", preload_data_to_mem=True,
             log_files_root="", backend="hip", data_catalog=None, workers=None,
             save_every=False, num_epochs=None, ctx=None, **engine_kw):
    msts = list(initial_msts or [])
    if not msts:
        raise ValueError("schedule() needs initial_msts")
    for name, fn in (("model_fn", model_fn), ("train_fn", train_fn)):
        if fn is not None and not getattr(fn, "_cerebro_native", False):
            logs("schedule(): custom {} ignored; the native packed HIP step is used".format(name))
    ctx = ctx or init_distributed()
    loader = None
    if _is_da(input_fn, data_catalog):
        from .data.da import da_partition_loader
        root = engine_kw.pop("da_root", None) or _catalog_root(data_catalog)
        loader = da_partition_loader(root, ctx.device)
    opts = EngineOptions(models_root=ckpt_root, logs_root=log_files_root, store_loader=loader,
                         ckpt_every="subepoch" if save_every else engine_kw.pop("ckpt_every", "epoch"),
                         **engine_kw)
    eng = MOPEngine(msts, ctx, opts)
    if data_catalog is None and ctx.rank == 0:
        data_catalog = make_data_catalog(data_set_name or eng.dataset, eng.P, ctx.world)
    epochs = num_epochs or 10 ** 6   # Cerebro runs until mst_eval_fn stops every config
    if mst_eval_fn is None:
        from .selection.hyperopt_helper import mst_eval_fn as grid_stop
        mst_eval_fn = grid_stop(num_epochs or 10)
        epochs = num_epochs or 10
    eng.run(epochs, mst_eval_fn=mst_eval_fn)
    eng.close()
    return eng.mst_state
