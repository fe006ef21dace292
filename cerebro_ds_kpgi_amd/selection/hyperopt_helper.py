"""Model-selection drivers over MOP: grid stopper and async TPE.

Implements the contracts of the reference's (missing) ``hyperopt_helper``
module and of the ``mst_eval_fn`` callbacks:

* ``init_hyperopt(param_grid, args, search_space_only=False)`` ->
  ``(hyperopt_params, msts, trials, domain, rand, model_options)`` or
  ``(search_space, rand)``; call sites ``run_da_cerebro_standalone.py:81-82``,
  ``run_hyperopt.py:104-105``.
* ``hyperopt_add_one_batch_configs(param_grid, hyperopt_params, msts, domain,
  trials, concurrency)`` -> ``(hyperopt_params, msts, start, end)``
  (``run_ctq_hyperopt.py:98-108``).
* ``mst_eval_fn(epoch)`` / ``mst_eval_fn_hyperopt(...)``: callbacks of
  ``schedule()`` returning ``(stop_list, update_mst_id_list, new_msts)``
  (``run_cerebro_standalone_helper.py:292-376``).

The reference's CTQ-hyperopt batch update indexes the trial list from 0
instead of the batch start (``run_ctq_hyperopt.py:110-120``); here every
trial is reported by its own tid.
"""

import numpy as np

from ..config.catalog import SEED, param_grid_hyperopt
from . import tpe


def batch_choices(param_grid=param_grid_hyperopt):
    """Batch sizes TPE chooses from: every integer in the reference range
    [lo, hi] (run_ctq_hyperopt.py:76-91), or -- ``batch_size_buckets`` in the
    grid -- only those values (all inside the range).  Bucketing is what lets
    a TPE batch pack: configs of one (architecture, batch size) train as ONE
    launch stream on a GPU, while 8 distinct batch sizes are 8 single-config
    pack groups (profiles/r3_hyperopt.md)."""
    lo, hi = param_grid["batch_size"][0], param_grid["batch_size"][1]
    b = param_grid.get("batch_size_buckets")
    if not b:
        return list(range(lo, hi + 1))
    bad = [x for x in b if not lo <= x <= hi]
    if bad:
        raise ValueError("batch_size_buckets {} outside the search range [{}, {}]"
                         .format(bad, lo, hi))
    return sorted(set(int(x) for x in b))


def build_search_space(param_grid=param_grid_hyperopt):
    """Reference space (run_ctq_hyperopt.py:76-91): model/lambda choices,
    log-uniform lr, batch size a choice over ``batch_choices``."""
    return {
        "model": tpe.choice("model", param_grid["model"]),
        "lambda_value": tpe.choice("lambda_value", param_grid["lambda_value"]),
        "learning_rate": tpe.loguniform("learning_rate", param_grid["learning_rate"][0],
                                        param_grid["learning_rate"][1]),
        "batch_size": tpe.choice("batch_size", batch_choices(param_grid)),
    }


class Domain(object):
    def __init__(self, space):
        self.space = space

    def to_mst(self, vals):
        p = tpe.vals_to_params(self.space, vals)
        return {"learning_rate": float(p["learning_rate"]), "lambda_value": p["lambda_value"],
                "batch_size": int(p["batch_size"]), "model": p["model"]}


def init_hyperopt(param_grid=param_grid_hyperopt, args=None, search_space_only=False,
                  cerebro=False, seed=SEED):
    space = build_search_space(param_grid)
    rand = np.random.RandomState(seed)
    if search_space_only:
        return space, rand
    trials = tpe.Trials()
    domain = Domain(space)
    concurrency = getattr(args, "size", 8) if args is not None else 8
    hyperopt_params, msts = [], []
    hyperopt_params, msts, _, _ = hyperopt_add_one_batch_configs(
        param_grid, hyperopt_params, msts, domain, trials, concurrency, rand=rand)
    model_options = list(param_grid["model"])
    return hyperopt_params, msts, trials, domain, rand, model_options


def hyperopt_add_one_batch_configs(param_grid, hyperopt_params, msts, domain, trials,
                                   concurrency, rand=None):
    rand = rand if rand is not None else np.random.RandomState(SEED)
    start = len(msts)
    for _ in range(concurrency):
        vals = tpe.tpe_suggest(domain.space, trials, rand)
        doc = trials.insert(vals)
        hyperopt_params.append(doc)
        msts.append(domain.to_mst(vals))
    return hyperopt_params, msts, start, len(msts)


def report_batch(trials, hyperopt_params, start, end, losses):
    """Report the losses of configs [start, end) — by their own tid."""
    for i, loss in zip(range(start, end), losses):
        trials.report(hyperopt_params[i]["tid"], loss)


def mst_eval_fn(epoch):
    """Grid search stopper: stop every config once it has ``epoch`` epochs."""
    def helper(mst_state):
        stop = [k for k, st in mst_state.items() if len(st["train_loss"]) == epoch]
        return stop, [], []
    return helper


def mst_eval_fn_hyperopt(epoch, hyperopt_params, trials, domain, max_num_config, rand,
                         concurrency, model_options=None, param_grid=param_grid_hyperopt):
    """Async TPE: when a RUNNING config reaches ``epoch`` epochs report its last
    validation loss; if any finished and fewer than ``max_num_config``
    configs exist, propose ``concurrency`` new ones."""
    def helper(mst_state):
        stop = []
        generate = False
        for mst_id, st in mst_state.items():
            if len(st["train_loss"]) == epoch and st.get("state") == "RUNNING":
                stop.append(mst_id)
                trials.report(hyperopt_params[mst_id]["tid"], st["valid_loss"][-1])
                generate = True
        new_msts = []
        if generate and len(mst_state) < max_num_config:
            n = min(concurrency, max_num_config - len(mst_state))
            for _ in range(n):
                vals = tpe.tpe_suggest(domain.space, trials, rand)
                doc = trials.insert(vals)
                hyperopt_params.append(doc)
                new_msts.append(domain.to_mst(vals))
        return stop, [], new_msts
    return helper
