"""MOP scheduling core: (model, worker) visit bookkeeping + invariants.

Model Hopper Parallelism: data partitions ("workers" here are
*virtual workers* = one data partition each) never move; S configurations
hop between them.  A *sub-epoch* is one (model, worker) visit; an *epoch* is
complete when every model has visited every worker once.  Invariants that
every policy must hold (reference ``cerebro_gpdb/ctq.py:448-508``):

1. each (model, worker) pair is trained exactly once per epoch,
2. a model is on at most one worker at a time,
3. a worker trains at most one model at a time.

``InvariantMonitor`` enforces them at runtime (scheduler
invariant assertions) for every scheduler and in the simulator.
"""


class SchedulerInvariantError(RuntimeError):
    pass


class InvariantMonitor(object):
    def __init__(self, models, workers):
        self.models = list(models)
        self.workers = list(workers)
        self.reset()

    def reset(self):
        self.done = set()
        self.model_on = {}    # model -> worker
        self.worker_has = {}  # worker -> model

    def start(self, model, worker):
        if model in self.model_on:
            raise SchedulerInvariantError(
                "model {} already running on worker {}".format(model, self.model_on[model]))
        if worker in self.worker_has:
            raise SchedulerInvariantError(
                "worker {} already running model {}".format(worker, self.worker_has[worker]))
        if (model, worker) in self.done:
            raise SchedulerInvariantError("pair {} trained twice in one epoch".format((model, worker)))
        self.model_on[model] = worker
        self.worker_has[worker] = model

    def finish(self, model, worker):
        if self.model_on.get(model) != worker:
            raise SchedulerInvariantError("finish of a job that is not running: {}".format((model, worker)))
        del self.model_on[model]
        del self.worker_has[worker]
        self.done.add((model, worker))

    def check_epoch_complete(self, models=None):
        models = self.models if models is None else models
        missing = [(m, w) for m in models for w in self.workers if (m, w) not in self.done]
        if missing:
            raise SchedulerInvariantError("epoch incomplete, missing {}".format(missing[:8]))
        if self.model_on:
            raise SchedulerInvariantError("jobs still running at epoch end: {}".format(self.model_on))


class MOPScheduler(object):
    """Base class.  Subclasses implement ``assign(worker)``.

    ``models`` is a list of model ids, ``workers`` a list of virtual-worker
    (partition) ids.  Models may be added between epochs (hyperopt) and
    removed (early stop) via ``add_models`` / ``remove_models``.
    """

    lockstep = False

    def __init__(self, models, workers, seed=2018):
        self.models = list(models)
        self.workers = list(workers)
        self.seed = seed
        self.epoch = 0
        self.monitor = InvariantMonitor(self.models, self.workers)
        self.idle_models = set()
        self.idle_workers = set()

    # -- epoch lifecycle --------------------------------------------------
    # Pack-aware order (set by the engine; None = the policy's own order):
    # a key per model, sorted ascending.  The engine keys configs by
    # (-steps per visit, pack key), so the configs with the most steps per
    # partition visit come first and configs that pack into one launch
    # stream (same architecture, batch size, optimizer) are adjacent.  The
    # rotation then trains them in the same sub-epochs and the greedy policy
    # hands them out first (longest-processing-time first): one G-config
    # pack instead of G one-config ones spread over G rounds.  Ties keep the
    # policy's order (the greedy shuffle stays random within a group).
    pack_key_fn = None

    def pack_sorted(self, items, model_of=lambda m: m):
        if self.pack_key_fn is None:
            return list(items)
        return sorted(items, key=lambda it: self.pack_key_fn(model_of(it)))

    def start_epoch(self, epoch):
        self.epoch = epoch
        self.monitor = InvariantMonitor(self.models, self.workers)
        self.idle_models = set(self.models)
        self.idle_workers = set(self.workers)
        self.pending = [(m, w) for m in self.models for w in self.workers]

    def epoch_done(self):
        return not self.pending and not self.monitor.model_on

    def add_models(self, models):
        for m in models:
            if m not in self.models:
                self.models.append(m)

    def remove_models(self, models):
        self.models = [m for m in self.models if m not in set(models)]

    # -- resume support ---------------------------------------------------
    def rng_state(self):
        """JSON-able RNG state (None for deterministic policies)."""
        rng = getattr(self, "rng", None)
        if rng is None:
            return None
        v, internal, gauss = rng.getstate()
        return [v, list(internal), gauss]

    def set_rng_state(self, state):
        if state is not None and getattr(self, "rng", None) is not None:
            self.rng.setstate((state[0], tuple(state[1]), state[2]))

    # -- job lifecycle ----------------------------------------------------
    def assign(self, worker):
        raise NotImplementedError

    def _start(self, model, worker):
        self.monitor.start(model, worker)
        self.pending.remove((model, worker))
        self.idle_models.discard(model)
        self.idle_workers.discard(worker)

    def complete(self, model, worker):
        self.monitor.finish(model, worker)
        self.idle_models.add(model)
        self.idle_workers.add(worker)

    # -- split completion (asynchronous runtime) --------------------------
    # A sub-epoch job = train + validate.  Its model's state is final when
    # training ends, so the model may start its next sub-epoch elsewhere
    # while this worker still validates it; the worker frees after validation.
    def release_model(self, model, worker):
        """Training of (model, worker) done: the pair is done, the model idle."""
        self.monitor.finish(model, worker)
        self.idle_models.add(model)

    def release_worker(self, worker):
        self.idle_workers.add(worker)

    def abort(self, model, worker):
        """A failed job: the pair goes back to the front of the queue."""
        if self.monitor.model_on.get(model) == worker:
            del self.monitor.model_on[model]
            del self.monitor.worker_has[worker]
        if (model, worker) not in self.pending:
            self.pending.insert(0, (model, worker))
        self.idle_models.add(model)
        self.idle_workers.add(worker)

    def assign_all_idle(self):
        """Offer every idle worker a job (worker order = id order, like CTQ's loop)."""
        out = []
        for w in sorted(self.idle_workers):
            m = self.assign(w)
            if m is not None:
                out.append((m, w))
        return out
