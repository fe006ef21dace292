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


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--fast_img_s", type=float, required=True,
                    help="MobileNetV2 bs128, one config alone, images/s")
    ap.add_argument("--slow_img_s", type=float, required=True,
                    help="NASNetMobile bs4, one config alone, images/s")
    ap.add_argument("--valid_speedup", type=float, default=3.0)
    a = ap.parse_args(argv)
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
