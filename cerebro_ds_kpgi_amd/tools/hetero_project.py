"""Greedy (CTQ) vs rotation (UDAF) makespan of the reference's 48-config
heterogeneous workload from MEASURED per-config training rates.

    python -m cerebro_ds_kpgi_amd.tools.hetero_project --fast_img_s 5200 --slow_img_s 310

The workload (``cerebro_gpdb/imagenetcat.py:50-60``):
38 x MobileNetV2 batch 128 (fast) + 10 x NASNetMobile batch 4 (slow), one
epoch of ImageNet over W workers, one data partition per worker.  A
sub-epoch of model m on one partition takes
``(train / W) / rate_m + (valid / W) / (valid_speedup * rate_m)``
seconds, where each rate is one config training alone on one MI355X
(``bench.py --model ... --batch ... --configs 1``).  Both schedulers run in
``scheduler/simulator.py``, which drives the runtime's own scheduler
classes, at W = 2, 4, 6 and 8.  The reference's measured hours and its
simulator fit (slow/fast = 7.94) are printed alongside.
"""

import argparse
import json
import random

from ..scheduler.simulator import simulate_greedy, simulate_rotation

TRAIN, VALID = 1281280, 50000
REF_HOURS = {8: (8.99, 3.29), 6: (9.91, 4.07), 4: (11.59, 5.25), 2: (14.25, 9.30)}


def project(fast_img_s, slow_img_s, n_fast=38, n_slow=10, workers=(2, 4, 6, 8),
            valid_speedup=3.0, seeds=5):
    out = []
    for W in workers:
        def sub(rate):
            return (TRAIN / W) / rate + (VALID / W) / (valid_speedup * rate)
        runtimes = [sub(fast_img_s)] * n_fast + [sub(slow_img_s)] * n_slow
        rot = simulate_rotation(runtimes, W)
        greedy = min(simulate_greedy(runtimes, W, rng=random.Random(s)) for s in range(seeds))
        ref = REF_HOURS.get(W)
        out.append({"workers": W, "rotation_h": rot / 3600.0, "greedy_h": greedy / 3600.0,
                    "speedup": rot / greedy,
                    "ref_udaf_h": ref[0] if ref else None, "ref_ctq_h": ref[1] if ref else None,
                    "ref_speedup": ref[0] / ref[1] if ref else None,
                    "slow_fast_ratio": fast_img_s / slow_img_s})
    return out


def _pack_time(t1, tg, g_meas):
    """Step time of a pack of g configs, linear between the measured
    one-config (t1) and g_meas-config (tg) step times (a pack step costs a
    fixed launch part plus a per-config part)."""
    slope = (tg - t1) / max(g_meas - 1, 1)
    return lambda g: 0.0 if g <= 0 else t1 + (g - 1) * slope


def simulate_packed(policy, n_fast, n_slow, W, V, t_fast, t_slow, b_fast=128, b_slow=4,
                    valid_speedup=3.0, seed=2018, pack_order=True):
    """Makespan (s) of one epoch of the hetero workload on W GPUs with V
    partitions each (P = W V), as THIS runtime executes it: a GPU trains the
    models on its V partitions as packs (one launch stream per architecture:
    pack step time t_fast(g) / t_slow(g) for g configs).  ``rotation``: the
    UDAF round plan, every round ends at a barrier over all GPUs;
    ``greedy``: CTQ, an idle GPU takes per idle partition the first runnable
    (model, partition) pair of the shuffled list (scheduler classes of
    ``scheduler.policies``).  ``pack_order``: the engine's default
    pack-aware order (``MOPEngine.pack_order_key``: most steps per visit
    first, packs adjacent); False = the policies' own orders."""
    import heapq
    from ..scheduler.policies import GreedyScheduler, RotationScheduler
    P = W * V
    models = list(range(n_fast + n_slow))
    slow = set(range(n_fast, n_fast + n_slow))
    parts = list(range(P))
    gpu_of = {p: p // V for p in parts}

    def pack_seconds(ms):
        ns = sum(1 for m in ms if m in slow)
        nf = len(ms) - ns
        tr = (TRAIN / P)
        va = (VALID / P)
        t = 0.0
        if nf:
            t += (tr / b_fast) * t_fast(nf) + (va / b_fast) * t_fast(nf) / valid_speedup
        if ns:
            t += (tr / b_slow) * t_slow(ns) + (va / b_slow) * t_slow(ns) / valid_speedup
        return t

    def key(m):            # MOPEngine.pack_order_key: (-steps per visit, pack key)
        b = b_slow if m in slow else b_fast
        return (-(TRAIN / P / b), "slow" if m in slow else "fast")

    if policy == "rotation":
        sch = RotationScheduler(models, parts, seed=seed)
        sch.pack_key_fn = key if pack_order else None
        sch.start_epoch(1)
        total = 0.0
        for rnd in sch.rounds:
            per_gpu = {}
            for p, m in rnd.items():
                per_gpu.setdefault(gpu_of[p], []).append(m)
            total += max((pack_seconds(ms) for ms in per_gpu.values()), default=0.0)
        return total
    sch = GreedyScheduler(models, parts, seed=seed, shuffle=True)
    sch.pack_key_fn = key if pack_order else None
    sch.start_epoch(1)
    now, events, busy = 0.0, [], set()

    def dispatch(g):
        got = sch.assign_many([p for p in range(g * V, (g + 1) * V) if p in sch.idle_workers])
        jobs = [(m, p) for p, m in got.items()]
        if jobs:
            busy.add(g)
            heapq.heappush(events, (now + pack_seconds([m for m, _ in jobs]), g, jobs))
    for g in range(W):
        dispatch(g)
    while events:
        now, g, jobs = heapq.heappop(events)
        busy.discard(g)
        for m, p in jobs:
            sch.complete(m, p)
        for h in range(W):
            if h not in busy:
                dispatch(h)
    if not sch.epoch_done():
        raise RuntimeError("packed greedy simulation stalled")
    return now


def simulate_classes(policy, classes, W, V, train=TRAIN, valid=VALID, valid_speedup=3.0,
                     seed=2018, pack_order=True):
    """General form of ``simulate_packed``: ``classes`` = [{"name", "n",
    "batch", "t": g -> seconds per packed step of g configs}]; every class
    is its own pack key (architecture, batch size).  Returns the makespan (s)
    of one epoch on W GPUs with V partitions each."""
    import heapq
    from ..scheduler.policies import GreedyScheduler, RotationScheduler
    P = W * V
    cls_of = []
    for ci, c in enumerate(classes):
        cls_of += [ci] * int(c["n"])
    models = list(range(len(cls_of)))
    parts = list(range(P))
    gpu_of = {p: p // V for p in parts}

    def pack_seconds(ms):
        per = {}
        for m in ms:
            per[cls_of[m]] = per.get(cls_of[m], 0) + 1
        t = 0.0
        for ci, g in per.items():
            c = classes[ci]
            t += (train / P / c["batch"]) * c["t"](g) + \
                (valid / P / c["batch"]) * c["t"](g) / valid_speedup
        return t

    def key(m):
        c = classes[cls_of[m]]
        return (-(train / P / c["batch"]), c["name"])

    if policy == "rotation":
        sch = RotationScheduler(models, parts, seed=seed)
        sch.pack_key_fn = key if pack_order else None
        sch.start_epoch(1)
        total = 0.0
        for rnd in sch.rounds:
            per_gpu = {}
            for p, m in rnd.items():
                per_gpu.setdefault(gpu_of[p], []).append(m)
            total += max((pack_seconds(ms) for ms in per_gpu.values()), default=0.0)
        return total
    sch = GreedyScheduler(models, parts, seed=seed, shuffle=True)
    sch.pack_key_fn = key if pack_order else None
    sch.start_epoch(1)
    now, events, busy = 0.0, [], set()

    def dispatch(g):
        got = sch.assign_many([p for p in range(g * V, (g + 1) * V) if p in sch.idle_workers])
        jobs = [(m, p) for p, m in got.items()]
        if jobs:
            busy.add(g)
            heapq.heappush(events, (now + pack_seconds([m for m, _ in jobs]), g, jobs))
    for g in range(W):
        dispatch(g)
    while events:
        now, g, jobs = heapq.heappop(events)
        busy.discard(g)
        for m, p in jobs:
            sch.complete(m, p)
        for h in range(W):
            if h not in busy:
                dispatch(h)
    if not sch.epoch_done():
        raise RuntimeError("packed greedy simulation stalled")
    return now


def project_classes(classes, workers=(1, 2, 4, 8), n_partitions=8, seeds=3, valid_speedup=3.0,
                    train=TRAIN, valid=VALID):
    """Rotation vs greedy makespans of a class workload (BASELINE config 4,
    ``--classes``) with the reference's 8 partitions spread over W GPUs."""
    out = []
    for W in workers:
        V = max(1, n_partitions // W)
        rot = simulate_classes("rotation", classes, W, V, train, valid, valid_speedup)
        gr = min(simulate_classes("greedy", classes, W, V, train, valid, valid_speedup, seed=s)
                 for s in range(seeds))
        out.append({"workers": W, "slots_per_gpu": V, "rotation_s": rot, "greedy_s": gr,
                    "speedup": rot / gr})
    return out


def project_packed(step_s, workers=(1, 2, 4, 6, 8), V=None, n_fast=38, n_slow=10, seeds=3,
                   valid_speedup=3.0, pack_order=True):
    """Rotation vs greedy hours from MEASURED pack step times
    ``step_s = {"fast": (t1, tg, g), "slow": (t1, tg, g)}`` (seconds per
    packed step at 1 and g configs: bench.py --configs 1 / g)."""
    tf = _pack_time(*step_s["fast"])
    ts = _pack_time(*step_s["slow"])
    out = []
    for W in workers:
        v = V or max(1, (n_fast + n_slow) // (W * 4))
        rot = simulate_packed("rotation", n_fast, n_slow, W, v, tf, ts,
                              valid_speedup=valid_speedup, pack_order=pack_order)
        gr = min(simulate_packed("greedy", n_fast, n_slow, W, v, tf, ts, seed=s,
                                 valid_speedup=valid_speedup, pack_order=pack_order)
                 for s in range(seeds))
        ref = REF_HOURS.get(W)
        out.append({"workers": W, "slots_per_gpu": v, "rotation_h": rot / 3600.0,
                    "greedy_h": gr / 3600.0, "speedup": rot / gr,
                    "ref_udaf_h": ref[0] if ref else None, "ref_ctq_h": ref[1] if ref else None,
                    "ref_speedup": ref[0] / ref[1] if ref else None})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--fast_img_s", type=float, default=0.0,
                    help="MobileNetV2 bs128, one config alone, images/s")
    ap.add_argument("--slow_img_s", type=float, default=0.0,
                    help="NASNetMobile bs4, one config alone, images/s")
    ap.add_argument("--valid_speedup", type=float, default=3.0)
    ap.add_argument("--packed", default="",
                    help="pack step times (s) as 'fast_t1,fast_tg,g_fast,slow_t1,slow_tg,g_slow' "
                         "(bench.py ms_per_step / 1000 at --configs 1 and g): project the "
                         "runtime's packed execution instead of one model per worker")
    ap.add_argument("--slots_per_gpu", type=int, default=0)
    ap.add_argument("--pack_order", default="true", choices=["true", "false"],
                    help="the engine's pack-aware scheduling order (default) or the policies' own")
    ap.add_argument("--classes", default="",
                    help="generic class workload, ';'-separated 'name,n,batch,t1,tg,g' (pack "
                         "step seconds at 1 and g configs), e.g. BASELINE config 4: "
                         "resnet50_b32,2,32,...;vgg16_b64,2,64,... (fast / slow ignored)")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--train_images", type=int, default=TRAIN)
    a = ap.parse_args(argv)
    if a.classes:
        classes = []
        for item in a.classes.split(";"):
            f = item.split(",")
            classes.append({"name": f[0], "n": int(f[1]), "batch": int(f[2]),
                            "t": _pack_time(float(f[3]), float(f[4]), int(f[5]))})
        rows = project_classes(classes, n_partitions=a.partitions, valid_speedup=a.valid_speedup,
                               train=a.train_images,
                               valid=int(a.train_images * VALID / TRAIN))
        print("| workers | slots / GPU | rotation (UDAF) s | greedy (CTQ) s | rotation / greedy |")
        print("|---:|---:|---:|---:|---:|")
        for r in rows:
            print("| {} | {} | {:.1f} | {:.1f} | {:.2f}x |".format(
                r["workers"], r["slots_per_gpu"], r["rotation_s"], r["greedy_s"], r["speedup"]))
        print(json.dumps(rows))
        return rows
    if a.packed:
        f = [float(x) for x in a.packed.split(",")]
        rows = project_packed({"fast": (f[0], f[1], int(f[2])), "slow": (f[3], f[4], int(f[5]))},
                              V=a.slots_per_gpu or None, valid_speedup=a.valid_speedup,
                              pack_order=a.pack_order == "true")
        print("| workers | slots / GPU | rotation (UDAF) h | greedy (CTQ) h | speedup | "
              "reference UDAF / CTQ h | reference speedup |")
        print("|---:|---:|---:|---:|---:|---|---:|")
        for r in rows:
            print("| {} | {} | {:.3f} | {:.3f} | {:.2f}x | {} / {} | {} |".format(
                r["workers"], r["slots_per_gpu"], r["rotation_h"], r["greedy_h"], r["speedup"],
                r["ref_udaf_h"], r["ref_ctq_h"],
                "{:.2f}x".format(r["ref_speedup"]) if r["ref_speedup"] else "-"))
        print(json.dumps(rows))
        return rows
    rows = project(a.fast_img_s, a.slow_img_s, valid_speedup=a.valid_speedup)
    print("| workers | rotation (UDAF) h | greedy (CTQ) h | speedup | reference UDAF / CTQ h "
          "| reference speedup |")
    print("|---:|---:|---:|---:|---|---:|")
    for r in rows:
        print("| {} | {:.3f} | {:.3f} | {:.2f}x | {} / {} | {:.2f}x |".format(
            r["workers"], r["rotation_h"], r["greedy_h"], r["speedup"], r["ref_udaf_h"],
            r["ref_ctq_h"], r["ref_speedup"]))
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
