"""Scheduling policies.

* ``RotationScheduler`` — UDAF / MADlib ``fit_multiple_model`` semantics
  (reference ``hetero_simluator.ipynb`` cell 2 ``rotate`` /
  ``UDAFSimulator.generate_schedule``): at sub-epoch ``s`` worker ``i`` trains
  ``rotate(models, i)[s]``; every sub-epoch ends at a global barrier.  On a
  ring of partitions this is a *ring shift*: each model moves to the next
  partition, so across GPUs it is one xGMI neighbour send per GPU.
* ``GreedyScheduler`` — CTQ / Cerebro semantics (reference
  ``cerebro_gpdb/ctq.py:247-261,448-508``): per epoch, all (model, worker)
  pairs in a seeded shuffled order; an idle worker takes the first pair whose
  worker matches and whose model is idle.  Work-conserving, event driven (no
  busy-wait: the runtime calls ``assign`` on completion events).
* Both take the engine's pack-aware order (``MOPScheduler.pack_key_fn``):
  configs that pack into one launch stream are co-scheduled, the ones with
  the most steps per visit first (the 48-config hetero drill-down:
  ``profiles/r4_hetero.md``).
* ``TaskParallelScheduler`` — Hyperopt-Spark semantics: one
  model per worker for the whole epoch over the *replicated* dataset.
"""

import random

from .base import MOPScheduler


def rotate(seq, n):
    """Rotate right by n (reference notebook ``rotate``: ``l[-n:] + l[:-n]``)."""
    n = n % len(seq) if seq else 0
    return seq[-n:] + seq[:-n] if n else list(seq)


class RotationScheduler(MOPScheduler):
    lockstep = True

    def start_epoch(self, epoch):
        super(RotationScheduler, self).start_epoch(epoch)
        L = max(len(self.models), len(self.workers))
        slots = self.pack_sorted(self.models) + [None] * (L - len(self.models))
        self.rounds = []
        for s in range(L):
            rnd = {}
            for i, w in enumerate(self.workers):
                m = rotate(slots, i)[s]
                if m is not None:
                    rnd[w] = m
            self.rounds.append(rnd)
        self.subepoch = 0

    def assign(self, worker):
        if self.subepoch >= len(self.rounds):
            return None
        m = self.rounds[self.subepoch].get(worker)
        if m is None or m not in self.idle_models or (m, worker) not in self.pending:
            return None
        self._start(m, worker)
        return m

    def next_round(self):
        """Lock-step API: the full {worker: model} map of the next sub-epoch."""
        if self.subepoch >= len(self.rounds):
            return None
        rnd = self.rounds[self.subepoch]
        for w, m in sorted(rnd.items()):
            self._start(m, w)
        return dict(rnd)

    def finish_round(self, rnd):
        for w, m in rnd.items():
            self.complete(m, w)
        self.subepoch += 1

    # asynchronous runtime: the next round's map is known before the current
    # round's workers are free (its hops start while they still validate)
    def peek_round(self):
        if self.subepoch >= len(self.rounds):
            return None
        return dict(self.rounds[self.subepoch])

    def start_round(self):
        """Start the peeked round (its workers must be free)."""
        return self.next_round()

    def end_round(self):
        self.subepoch += 1


class GreedyScheduler(MOPScheduler):
    def __init__(self, models, workers, seed=2018, shuffle=True):
        super(GreedyScheduler, self).__init__(models, workers, seed)
        self.shuffle = shuffle
        self.rng = random.Random(seed)

    def start_epoch(self, epoch):
        super(GreedyScheduler, self).start_epoch(epoch)
        if self.shuffle:
            self.rng.shuffle(self.pending)
        self.pending = self.pack_sorted(self.pending, model_of=lambda mw: mw[0])

    def assign(self, worker):
        if worker not in self.idle_workers:
            return None
        for m, w in self.pending:
            if w == worker and m in self.idle_models:
                self._start(m, w)
                return m
        return None

    def assign_many(self, workers):
        """Assign idle models to the idle ``workers`` together ({worker:
        model}): one wave of workers freed at once (a GPU's partition slots
        at the end of its batch).  Without the pack-aware order this is
        ``assign`` per worker (first runnable pair of the queue).  With it,
        each key class (most steps per visit first) gets a MAXIMUM matching
        of its idle models to the wave's still-free workers (augmenting
        paths, visited in queue order): the first-fit loop left the slow
        pack's tail at 2-3 configs per wave where each config still had a
        free partition to go to (profiles/r4_hetero.md)."""
        workers = [w for w in workers if w in self.idle_workers]
        if self.pack_key_fn is None:
            out = {}
            for w in workers:
                m = self.assign(w)
                if m is not None:
                    out[w] = m
            return out
        free = set(workers)
        pend = [(m, w) for m, w in self.pending if w in free and m in self.idle_models]
        keyed = {}
        for m, _ in pend:
            if m not in keyed:
                keyed[m] = self.pack_key_fn(m)
        match_w, match_m = {}, {}
        for k in sorted(set(keyed.values())):
            adj = {}
            for m, w in pend:
                if keyed[m] == k:
                    adj.setdefault(m, []).append(w)

            def augment(m, seen):
                for w in adj[m]:
                    if w in seen:
                        continue
                    seen.add(w)
                    cur = match_w.get(w)
                    if cur is None or (keyed[cur] == k and augment(cur, seen)):
                        match_w[w] = m
                        match_m[m] = w
                        return True
                return False
            for m in adj:
                if m not in match_m:
                    augment(m, set())
        for w in workers:                        # queue / worker order of the starts
            if w in match_w:
                self._start(match_w[w], w)
        return {w: match_w[w] for w in workers if w in match_w}


class TaskParallelScheduler(MOPScheduler):
    """Each job = one model trained on *all* partitions (replicated data).

    Bookkeeping is per (model, "ALL") so the invariants still apply.
    """

    ALL = "ALL"

    def start_epoch(self, epoch):
        super(TaskParallelScheduler, self).start_epoch(epoch)
        self.pending_models = list(self.models)
        self.running = {}
        self.pending = []

    def epoch_done(self):
        return not self.pending_models and not self.running

    def assign(self, worker):
        if worker in self.running or not self.pending_models:
            return None
        m = self.pending_models.pop(0)
        self.running[worker] = m
        self.idle_workers.discard(worker)
        self.idle_models.discard(m)
        return m

    def complete(self, model, worker):
        assert self.running.get(worker) == model
        del self.running[worker]
        self.idle_workers.add(worker)
        self.idle_models.add(model)


def make_scheduler(name, models, workers, seed=2018, shuffle=True):
    if name == "rotation":
        return RotationScheduler(models, workers, seed)
    if name == "greedy":
        return GreedyScheduler(models, workers, seed, shuffle=shuffle)
    if name == "task":
        return TaskParallelScheduler(models, workers, seed)
    raise ValueError("unknown scheduler {}".format(name))
