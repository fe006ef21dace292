"""Discrete-event simulator of the MOP schedulers.

Reproduces the reference's hetero-scheduler study
(``cerebro_gpdb/hetero_simluator.ipynb`` cells 2-6): sub-epoch runtimes per
model, W workers, one epoch; lock-step rotation (UDAF) vs greedy (CTQ), plus
the analytic models

* ``UDAF ≈ p^W·M + (1 − p^W)·scale·M``   (all W concurrent models fast with prob p^W)
* ``CTQ  ≈ M · l_mean``                  (work-conserving)

The simulator drives the *same* scheduler classes the GPU runtime uses, so
its results double as scheduler tests.
"""

import random

import numpy as np

from .policies import GreedyScheduler, RotationScheduler


def simulate_rotation(runtimes, num_workers):
    """Makespan of one lock-step epoch: sum over sub-epochs of the slowest job."""
    models = list(range(len(runtimes)))
    sched = RotationScheduler(models, list(range(num_workers)))
    sched.start_epoch(1)
    total = 0.0
    while True:
        rnd = sched.next_round()
        if rnd is None:
            break
        total += max([runtimes[m] for m in rnd.values()]) if rnd else 0.0
        sched.finish_round(rnd)
    sched.monitor.check_epoch_complete()
    return total


def simulate_greedy(runtimes, num_workers, rng=None, return_jobs=False):
    """Event-driven greedy epoch.  ``rng`` shuffles the pair list (a
    ``random.Random`` or the ``random`` module itself)."""
    models = list(range(len(runtimes)))
    workers = list(range(num_workers))
    sched = GreedyScheduler(models, workers, shuffle=False)
    sched.start_epoch(1)
    (rng or random).shuffle(sched.pending)
    now = 0.0
    finish_at = {}
    running = {}
    jobs = []
    while not sched.epoch_done():
        for w in workers:
            if w in sched.idle_workers:
                m = sched.assign(w)
                if m is not None:
                    running[w] = m
                    finish_at[w] = now + runtimes[m]
                    jobs.append({"model_key": m, "dist_key": w, "start_time": now,
                                 "end_time": finish_at[w]})
        first, t_next = None, None
        for w in workers:
            if w in running and (t_next is None or finish_at[w] < t_next):
                first, t_next = w, finish_at[w]
        if first is None:
            raise RuntimeError("greedy simulation stalled")
        sched.complete(running.pop(first), first)
        del finish_at[first]
        now = t_next
    sched.monitor.check_epoch_complete()
    return (now, jobs) if return_jobs else now


def predict_rotation_runtime(W, M, scale, p):
    return p ** W * 1 * M + (1 - p ** W) * scale * M


def predict_greedy_runtime(M, l_mean):
    return M * l_mean


def bernoulli_runtimes(p=0.9, scale=100, size=256, exact_counts=False, np_rng=None):
    """Fast (1) / slow (scale) runtimes; ``exact_counts`` = notebook's new_way."""
    r = np_rng if np_rng is not None else np.random
    if exact_counts:
        fast = int(round(size * p))
        out = np.array([scale] * (size - fast) + [1] * fast, dtype=float)
        r.shuffle(out)
    else:
        out = r.binomial(1, p, size).astype(float)
        out[out == 0] = scale
        out[out == 1] = 1
    return out


def sweep(runtimes, max_workers=32, p=0.8, rng=None):
    """Rows of (W, rot, rot_pred, greedy, greedy_pred, speedup, pred_speedup)."""
    runtimes = list(runtimes)
    lmax, lmin, lmean = max(runtimes), min(runtimes), float(np.mean(runtimes))
    scale = lmax / lmin
    rows = []
    for W in range(1, max_workers + 1):
        rot = simulate_rotation(runtimes, W)
        rot_p = predict_rotation_runtime(W, len(runtimes), scale, p)
        gr = simulate_greedy(runtimes, W, rng=rng)
        gr_p = predict_greedy_runtime(len(runtimes), lmean)
        rows.append((W, rot, rot_p, gr, gr_p, rot / gr, rot_p / gr_p))
    return rows
