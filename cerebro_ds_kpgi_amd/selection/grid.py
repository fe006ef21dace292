"""Grid generation and experiment selection.

Behavioural parity with reference ``cerebro_gpdb/in_rdbms_helper.py:156-229``:

* ``get_msts`` enumerates the cartesian product in key order, then sorts by
  batch size and (stably) by model name; the ``hetro`` grid replicates a fast
  and a slow MST ``fast``/``slow`` times.
* ``get_exp_specific_msts`` picks the grid from experiment flags and applies
  ``--sanity`` (first 8), ``--pytorchddp_sanity`` (batch // size) and
  ``--run_single`` (one MST).
"""

import itertools

from ..config import catalog as cat


def get_msts(param_grid=cat.param_grid, hetro_dedub=False):
    names = list(param_grid.keys())
    if "hetro" in names:
        pair = []
        for i in range(2):
            pair.append({
                "learning_rate": param_grid["learning_rate"][i],
                "lambda_value": param_grid["lambda_value"][i],
                "batch_size": param_grid["batch_size"][i],
                "model": param_grid["model"][i],
            })
        if hetro_dedub:
            return pair
        slow, fast = pair
        msts = [dict(fast) for _ in range(param_grid["fast"])] + \
            [dict(slow) for _ in range(param_grid["slow"])]
        assert len(msts) == param_grid["total"], "Length must agree"
        return msts
    combos = [dict(zip(names, values))
              for values in itertools.product(*[param_grid[n] for n in names])]
    combos = sorted(combos, key=lambda m: m["batch_size"])
    combos = sorted(combos, key=lambda m: m["model"])
    return combos


def get_exp_specific_msts(args):
    if getattr(args, "criteo", False):
        grid = cat.param_grid_criteo_breakdown if args.criteo_breakdown else cat.param_grid_criteo
        msts = get_msts(grid)
    elif getattr(args, "tiny", False):
        msts = get_msts(cat.param_grid_tiny)
    elif getattr(args, "drill_down_hetero_rv", False):
        msts = get_msts(cat.param_grid_hetero_rv)
    elif args.drill_down_hetro:
        msts = get_msts(cat.param_grid_hetro, hetro_dedub=args.drill_down_hetro_db_load)
    elif args.drill_down_model_size:
        msts = get_msts(cat.param_grid_model_size[args.drill_down_model_size_identifier])
    elif args.best_model_run:
        msts = get_msts(cat.param_grid_best_model)
    elif args.drill_down_scalability:
        msts = get_msts(cat.param_grid_scalability)
    elif args.hyperopt:
        # initial (model x lambda) corners; TPE proposes the rest
        grid = {k: (v if k in ("lambda_value", "model") else v[:1])
                for k, v in cat.param_grid_hyperopt.items()}
        msts = get_msts(grid)
    else:
        msts = get_msts()
    if args.sanity:
        msts = msts[:8]
    if args.pytorchddp_sanity:
        for m in msts:
            m["batch_size"] = m["batch_size"] // args.size
    if args.run_single:
        msts = [msts[args.single_mst_index]]
    return msts
