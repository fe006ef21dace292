"""Scheduler invariants + simulator parity with the reference notebook.

Golden numbers: ``cerebro_gpdb/hetero_simluator.ipynb`` cell 6 recorded
output (48 configs, 38 fast + 10 slow, scale 7.9427, seed 2020, W = 1..8).
"""

import itertools
import random

import numpy as np
import pytest

from cerebro_ds_kpgi_amd.scheduler import (GreedyScheduler, RotationScheduler,
                                           SchedulerInvariantError, TaskParallelScheduler,
                                           predict_greedy_runtime, predict_rotation_runtime,
                                           rotate, simulate_greedy, simulate_rotation)

S = 7.942693044033185
NB_RUNTIMES = [1, 1, 1, 1, 1, 1, S, 1, 1, 1, 1, 1, 1, 1, S, 1, 1, 1, S, 1, 1, 1, 1, 1, 1, 1, 1,
               S, 1, S, 1, 1, 1, S, 1, 1, S, 1, 1, 1, 1, S, 1, 1, 1, S, S, 1.0]
NB_UDAF = [117.42693044033184, 166.02578174856416, 207.68194001276322, 249.33809827696234,
           270.1661774090619, 290.99425654116146, 304.8796426292278, 318.7650287172942]
NB_CTQ = [117.42693044033187, 117.42693044033189, 117.42693044033187, 117.42693044033189,
          120.36962348436506, 124.36962348436506, 117.42693044033187, 120.36962348436506]


def test_rotate_matches_reference_definition():
    assert rotate([0, 1, 2, 3], 1) == [3, 0, 1, 2]
    assert rotate([0, 1, 2, 3], 0) == [0, 1, 2, 3]
    assert rotate([0, 1, 2, 3], 5) == [3, 0, 1, 2]


def test_simulator_parity_with_notebook():
    arr = np.array(NB_RUNTIMES)
    random.seed(2020)
    random.shuffle(arr)
    for W in range(1, 9):
        assert simulate_rotation(list(arr), W) == pytest.approx(NB_UDAF[W - 1], rel=1e-12)
        assert simulate_greedy(list(arr), W) == pytest.approx(NB_CTQ[W - 1], rel=1e-12)


def test_analytic_predictions():
    assert predict_rotation_runtime(1, 48, S, 0.8) == pytest.approx(114.64985322271856)
    assert predict_greedy_runtime(48, float(np.mean(NB_RUNTIMES))) == pytest.approx(117.42693044033186)


@pytest.mark.parametrize("S_models,W", [(8, 8), (8, 2), (3, 5), (10, 4), (1, 1)])
def test_rotation_covers_every_pair_once(S_models, W):
    sch = RotationScheduler(list(range(S_models)), list(range(W)))
    sch.start_epoch(1)
    seen = []
    while True:
        rnd = sch.next_round()
        if rnd is None:
            break
        # one model per worker, one worker per model
        assert len(set(rnd.values())) == len(rnd)
        seen += [(m, w) for w, m in rnd.items()]
        sch.finish_round(rnd)
    assert sorted(seen) == sorted(itertools.product(range(S_models), range(W)))
    sch.monitor.check_epoch_complete()
    assert len(sch.rounds) == max(S_models, W)


def test_rotation_is_ring_shift():
    sch = RotationScheduler(list(range(8)), list(range(8)))
    sch.start_epoch(1)
    r0 = sch.next_round()
    sch.finish_round(r0)
    r1 = sch.next_round()
    inv0 = {m: w for w, m in r0.items()}
    inv1 = {m: w for w, m in r1.items()}
    assert all(inv1[m] == (inv0[m] + 1) % 8 for m in range(8))


@pytest.mark.parametrize("seed", [0, 1, 2018])
def test_greedy_event_driven_invariants(seed):
    rng = random.Random(seed)
    runtimes = [rng.choice([1, 3, 8]) for _ in range(12)]
    t, jobs = simulate_greedy(runtimes, 5, rng=random.Random(seed), return_jobs=True)
    assert len(jobs) == 12 * 5
    # no overlap on a worker or for a model
    for key in ("dist_key", "model_key"):
        by = {}
        for j in jobs:
            by.setdefault(j[key], []).append((j["start_time"], j["end_time"]))
        for iv in by.values():
            iv.sort()
            for a, b in zip(iv, iv[1:]):
                assert a[1] <= b[0] + 1e-12
    assert t >= sum(runtimes) * 5 / 5 - 1e-9


def test_invariant_monitor_rejects_violations():
    sch = GreedyScheduler([0, 1], [0, 1], shuffle=False)
    sch.start_epoch(1)
    sch.monitor.start(0, 0)
    with pytest.raises(SchedulerInvariantError):
        sch.monitor.start(0, 1)
    with pytest.raises(SchedulerInvariantError):
        sch.monitor.start(1, 0)
    with pytest.raises(SchedulerInvariantError):
        sch.monitor.check_epoch_complete()


def test_task_parallel_each_model_once():
    sch = TaskParallelScheduler(list(range(5)), list(range(2)))
    sch.start_epoch(1)
    done = []
    while not sch.epoch_done():
        for w in (0, 1):
            m = sch.assign(w)
            if m is not None:
                done.append(m)
                sch.complete(m, w)
    assert sorted(done) == list(range(5))


def test_packed_hetero_projection():
    """tools.hetero_project packed mode: the simulator trains every (model,
    partition) pair once per epoch under both policies, a pack of g configs
    costs the interpolated pack step, and one model per GPU with unit pack
    cost reproduces the unpacked greedy / rotation ordering (rotation, with a
    barrier per round, is never faster than greedy there)."""
    from cerebro_ds_kpgi_amd.tools import hetero_project as hp
    f = hp._pack_time(1.0, 4.0, 4)
    assert f(0) == 0.0 and f(1) == 1.0 and f(4) == 4.0 and abs(f(2) - 2.0) < 1e-12
    rows = hp.project_packed({"fast": (0.004, 0.02, 8), "slow": (0.017, 0.03, 10)},
                             workers=(2, 8), V=1, seeds=2)
    for r in rows:
        assert r["rotation_h"] >= r["greedy_h"] * 0.999, r
    # packing: at one GPU holding every partition the slow configs share packs
    one = hp.project_packed({"fast": (0.004, 0.02, 8), "slow": (0.017, 0.03, 10)},
                            workers=(1,), V=8, seeds=1)[0]
    unpacked = hp.project_packed({"fast": (0.004, 0.032, 8), "slow": (0.017, 0.17, 10)},
                                 workers=(1,), V=8, seeds=1)[0]
    assert one["greedy_h"] < unpacked["greedy_h"] and one["rotation_h"] < unpacked["rotation_h"]


def _slow_first(slow):
    # the engine's key shape: (-steps per visit, pack key)
    return lambda m: (-128, ("nasnetmobile", "4")) if m in slow else (-4, ("mobilenetv2", "128"))


def test_rotation_pack_order_coschedules_a_pack():
    """Pack-aware rotation (MOPScheduler.pack_key_fn): the slow configs are
    adjacent in the rotation order, so a sub-epoch holds all of them at once
    (one G-config pack) and they finish in the fewest sub-epochs; every
    (model, worker) pair is still trained exactly once."""
    slow = {1, 4, 7}
    models, workers = list(range(9)), list(range(3))
    plain = RotationScheduler(models, workers)
    packed = RotationScheduler(models, workers)
    packed.pack_key_fn = _slow_first(slow)
    rounds = {}
    for name, sch in (("plain", plain), ("packed", packed)):
        sch.start_epoch(0)
        pairs = [(m, w) for rnd in sch.rounds for w, m in rnd.items()]
        assert sorted(pairs) == sorted((m, w) for m in models for w in workers)
        rounds[name] = [sum(m in slow for m in rnd.values()) for rnd in sch.rounds]
    # the pack: some sub-epoch trains all three slow configs together, and
    # the slow work spans fewer sub-epochs than in id order
    assert max(rounds["packed"]) == 3 and max(rounds["plain"]) < 3
    assert (sum(1 for c in rounds["packed"] if c) < sum(1 for c in rounds["plain"] if c))


def test_greedy_pack_order_hands_out_slow_pack_first():
    """Pack-aware greedy: longest-processing-time first -- in the first wave
    every worker that can take a slow config does, so they run as one pack;
    the invariants still hold over the epoch."""
    slow = {2, 5}
    models, workers = list(range(6)), list(range(4))
    sch = GreedyScheduler(models, workers, seed=3)
    sch.pack_key_fn = _slow_first(slow)
    sch.start_epoch(0)
    first = {w: sch.assign(w) for w in workers}
    assert sum(m in slow for m in first.values()) == len(slow)
    running = dict(first)
    while running:
        w = next(iter(running))
        sch.complete(running.pop(w), w)
        m = sch.assign(w)
        if m is not None:
            running[w] = m
        for w2 in workers:
            if w2 not in running:
                m2 = sch.assign(w2)
                if m2 is not None:
                    running[w2] = m2
    assert sch.epoch_done()
    sch.monitor.check_epoch_complete()


def test_greedy_wave_matching_places_the_whole_slow_pack():
    """assign_many with the pack-aware order: a maximum matching per key
    class.  First-fit gives worker 0 model A and leaves B, whose only
    remaining partition is 0, idle; the matching moves A to worker 1."""
    sch = GreedyScheduler([0, 1, 2], [0, 1], seed=0, shuffle=False)
    sch.pack_key_fn = lambda m: (-128,) if m in (0, 1) else (-4,)
    sch.start_epoch(0)
    # A = 0 may go to either worker, B = 1 has only worker 0 left
    sch.pending = [(0, 0), (0, 1), (1, 0), (2, 0), (2, 1)]
    sch.monitor.done.add((1, 1))
    got = sch.assign_many([0, 1])
    assert got == {0: 1, 1: 0}
    # without the pack-aware order: the policy's own first-fit
    plain = GreedyScheduler([0, 1, 2], [0, 1], seed=0, shuffle=False)
    plain.start_epoch(0)
    plain.pending = [(0, 0), (0, 1), (1, 0), (2, 0), (2, 1)]
    assert plain.assign_many([0, 1]) == {0: 0, 1: 2}


def test_class_projection_bounds():
    """tools.hetero_project --classes (BASELINE config 4): both policies train
    every (model, partition) pair; with one slot per GPU they tie at N = 8
    (each sub-epoch waits for the slowest model), more GPUs never take longer,
    and a class-homogeneous workload gives rotation = greedy at N = 1."""
    from cerebro_ds_kpgi_amd.tools import hetero_project as hp

    def cls(name, n, b, t1, tg, g):
        return {"name": name, "n": n, "batch": b, "t": hp._pack_time(t1, tg, g)}
    classes = [cls("r50_b32", 2, 32, 0.0038, 0.0052, 2), cls("r50_b64", 2, 64, 0.0051, 0.0080, 2),
               cls("vgg_b32", 2, 32, 0.0080, 0.0113, 2), cls("vgg_b64", 2, 64, 0.0120, 0.0182, 2)]
    rows = hp.project_classes(classes, workers=(1, 2, 4, 8), seeds=2, train=2048, valid=81)
    by = {r["workers"]: r for r in rows}
    assert abs(by[8]["speedup"] - 1.0) < 1e-9
    for a, b in ((1, 2), (2, 4), (4, 8)):
        assert by[b]["greedy_s"] <= by[a]["greedy_s"] * 1.001
        assert by[b]["rotation_s"] <= by[a]["rotation_s"] * 1.001
    same = hp.project_classes([cls("r50_b32", 8, 32, 0.0038, 0.0052, 2)], workers=(1,), seeds=1,
                              train=2048, valid=81)[0]
    assert abs(same["speedup"] - 1.0) < 0.05, same
