"""Cerebro-compatible front door: ``schedule(...)``.

Same keyword signature as the external Cerebro standalone scheduler the
reference drives (``cerebro_gpdb/run_da_cerebro_standalone.py:84-120``,
``run_filesystem_cerebro_standalone.py:85-98``):

    schedule(data_set_name, input_fn, model_fn, train_fn, initial_msts,
             mst_eval_fn, ckpt_root, preload_data_to_mem, log_files_root,
             backend, data_catalog, workers=None, save_every=False)

On MI355X the data plane, the model and the train step are the framework's
own (HBM partition store, packed HIP models, fused step), so:

* ``input_fn`` + ``data_catalog`` select the data source
  (``_data_source``): ``data.da.input_fn`` (or a catalog whose ``data_root``
  holds a DA manifest) -> Direct-Access pages; ``data.fs.input_fn`` /
  ``input_fn_criteo`` (or a catalog ``data_root`` with ``train/`` partitions)
  -> the filesystem partitions; no ``input_fn`` and no ``data_root`` ->
  synthetic partitions of the dataset's shape (logged); any other
  ``input_fn`` raises ``ValueError``;
* ``model_fn``: ``None`` / ``native_model_fn`` build each MST's ``model``
  from ``models.registry``.  A custom ``model_fn(mst)`` must return either an
  architecture name or a ``models.common.PackedNet`` (our packed-model API:
  ``ParamSpec`` declarations + a forward over ``ops.nn``); the returned
  architecture is registered and trained by the native step.  The
  reference's Keras closure ``model_fn(generator)(data, mst, purpose)`` cannot
  run here and raises ``TypeError`` instead of being silently ignored;
* ``train_fn``: ``None`` / ``native_train_fn`` = the fused HIP step
  (forward, softmax-CE, backward, Adam).  Any other callable raises
  ``NotImplementedError`` (the step is a captured HIP graph, not a Python
  function of a Keras model);
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


def _fn_module(fn):
    return getattr(fn, "__module__", "") or ""


def _data_source(input_fn, data_catalog, data_set_name):
    """Resolve the reference's data arguments to (kind, root, dataset).

    kind: ``"da"`` (Greenplum-format pages through the C++ reader),
    ``"fs"`` (``.npy`` partitions in the reference's filesystem layout) or
    ``"synthetic"`` (no ``input_fn`` and no catalog ``data_root``: synthetic
    partitions of the dataset's shape, said so in the log).  The reference
    passes ``input_fn`` / ``input_fn_criteo`` with a ``DATA_CATALOG``
    (``run_filesystem_cerebro_standalone.py:24-51,85-98``) or the DA
    ``input_fn`` (``run_da_cerebro_standalone.py:84-120``); any other
    ``input_fn`` is refused rather than silently replaced by synthetic data.
    """
    from .data import da, fs
    root = _catalog_root(data_catalog)
    mod = _fn_module(input_fn)
    name = getattr(input_fn, "__name__", "")
    dataset = data_set_name
    if input_fn is not None:
        if mod.endswith("data.da"):
            kind = "da"
        elif mod.endswith("data.fs") and name in ("input_fn", "input_fn_criteo"):
            kind = "fs"
            if name == "input_fn_criteo":
                dataset = dataset or "criteo"
        else:
            raise ValueError(
                "schedule(): unsupported input_fn {}.{}; pass data.fs.input_fn / "
                "data.fs.input_fn_criteo (filesystem partitions) or data.da.input_fn "
                "(Direct-Access pages) with a data_catalog whose data_root holds them, or "
                "input_fn=None for synthetic data".format(mod, name))
        if not root:
            raise ValueError("schedule(): input_fn {} needs a data_catalog with a data_root"
                             .format(name))
    elif root:
        if os.path.exists(os.path.join(root, da.MANIFEST)):
            kind = "da"
        elif fs.is_fs_root(root):
            kind = "fs"
        else:
            raise ValueError("schedule(): data_catalog data_root {} holds neither a DA "
                             "manifest nor filesystem partitions".format(root))
    else:
        return "synthetic", "", dataset
    if kind == "da" and not os.path.exists(os.path.join(root, da.MANIFEST)):
        raise ValueError("schedule(): data_root {} holds no DA manifest ({})"
                         .format(root, da.MANIFEST))
    if kind == "fs":
        if not fs.is_fs_root(root):
            raise ValueError("schedule(): data_root {} holds no train/ partitions".format(root))
        if dataset is None:
            dataset = fs.fs_dataset_of(root)
    return kind, root, dataset


def _da_input_fn():
    from .data.da import input_fn
    return input_fn


def native_model_fn(mst):
    """The framework's model factory (the default ``model_fn``)."""
    return mst["model"]


def native_train_fn(*a, **k):
    """Marker for the native fused train step (the default ``train_fn``)."""
    raise RuntimeError("native_train_fn is a marker; the engine runs the fused HIP step")


native_model_fn._cerebro_native = True
native_train_fn._cerebro_native = True


def _adopt_model_fn(model_fn, msts):
    """Apply a custom ``model_fn(mst)`` to every MST (see module docstring)."""
    from .models.common import PackedNet
    from .models.registry import MODEL_FACTORIES, dataset_of, register_model
    out = []
    for mst in msts:
        try:
            got = model_fn(mst)
        except TypeError as e:
            raise TypeError("schedule(): model_fn must be model_fn(mst) -> architecture name "
                            "or PackedNet (a Keras model_fn(generator)(data, mst, purpose) "
                            "closure cannot run on this framework): {}".format(e))
        m = dict(mst)
        if isinstance(got, str):
            if got not in MODEL_FACTORIES:
                raise ValueError("schedule(): model_fn returned unknown architecture {!r}"
                                 .format(got))
            m["model"] = got
        elif isinstance(got, PackedNet):
            import hashlib
            cls = type(got)
            sig = hashlib.sha1(repr([(s.name, s.shape) for s in got.layout.specs])
                               .encode()).hexdigest()[:8]
            name = "custom:{}.{}:{}".format(cls.__module__, cls.__qualname__, sig)
            ds = getattr(got, "dataset", None) or dataset_of(mst.get("model", ""))
            register_model(name, lambda mst=dict(mst): model_fn(mst), ds)
            m["model"] = name
        else:
            raise TypeError("schedule(): model_fn returned {!r}; expected an architecture name "
                            "or a PackedNet".format(type(got).__name__))
        out.append(m)
    return out


def schedule(data_set_name=None, input_fn=None, model_fn=None, train_fn=None,
             initial_msts=None, mst_eval_fn=None, ckpt_root="", preload_data_to_mem=True,
             log_files_root="", backend="hip", data_catalog=None, workers=None,
             save_every=False, num_epochs=None, ctx=None, **engine_kw):
    msts = list(initial_msts or [])
    if not msts:
        raise ValueError("schedule() needs initial_msts")
    if train_fn is not None and not getattr(train_fn, "_cerebro_native", False):
        raise NotImplementedError(
            "schedule(): custom train_fn is not supported; the native fused step (forward, "
            "softmax-CE, backward, Adam on HIP kernels) trains every config. Pass "
            "train_fn=None or api.native_train_fn")
    if model_fn is not None and not getattr(model_fn, "_cerebro_native", False):
        msts = _adopt_model_fn(model_fn, msts)
        logs("schedule(): model_fn -> architectures {}".format(sorted({m["model"] for m in msts})))
    ctx = ctx or init_distributed()
    if engine_kw.get("da_root"):
        data_catalog = {"data_root": engine_kw.pop("da_root")}
        input_fn = input_fn if input_fn is not None else _da_input_fn()
    kind, root, dataset = _data_source(input_fn, data_catalog, data_set_name)
    loader = None
    if kind == "da":
        from .data.da import da_partition_loader
        loader = da_partition_loader(root, ctx.device)
    elif kind == "fs":
        from .data import fs
        loader = fs.fs_partition_loader(root, dataset, ctx.device)
        nparts = fs.count_partitions(root)
        engine_kw.setdefault("dataset", dataset)
        if engine_kw.get("slots_per_gpu") is None:
            engine_kw["slots_per_gpu"] = max(1, nparts // ctx.world)
        if engine_kw["slots_per_gpu"] * ctx.world > nparts:
            raise ValueError("schedule(): {} GPUs x {} slots need {} partitions; {} holds {}"
                             .format(ctx.world, engine_kw["slots_per_gpu"],
                                     engine_kw["slots_per_gpu"] * ctx.world, root, nparts))
    else:
        logs("schedule(): no input_fn / data_root -> synthetic {} partitions"
             .format(dataset or "dataset-shaped"))
    logs("schedule(): data source {}{}".format(kind, " " + root if root else ""))
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
