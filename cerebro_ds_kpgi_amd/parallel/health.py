"""Worker heartbeats and a watchdog over the c10d store.

The reference has no failure detection beyond re-raising a CTQ job's
exception as ``FATAL ERROR`` (``cerebro_gpdb/ctq.py:411-423,488-489``) and
shell-level restarts (``runner_helper.sh:36-58``).  Here every rank runs a
daemon thread that stamps ``hb/{rank}`` in the rendezvous store every
``interval`` seconds; rank 0's watchdog declares a rank *lost* when its
stamp is older than ``timeout`` and then

1. logs ``WORKER {r} LOST`` and writes ``{logs_root}/failed_workers.json``,
2. calls ``on_failure(lost_ranks)`` — by default it terminates the job with
   exit code ``EXIT_WORKER_LOST`` so ``torchrun --max-restarts`` relaunches
   it and the engine resumes from the last sub-epoch checkpoint
   (``runtime/engine.py`` ``--resume``).

The stamp carries a *progress* record besides the time: the engine marks
the start and end of every sub-epoch job (``progress(step, busy)``).  The
beating thread is independent of the training thread, so a live stamp alone
proves only that the process runs; a rank that has been inside one job for
longer than ``stall_timeout`` (e.g. wedged in an RCCL call or a hung kernel)
is flagged ``STALLED`` and handled like a lost one.  Idle ranks (waiting for
an assignment) are never flagged as stalled.
"""

import json
import os
import threading
import time

EXIT_WORKER_LOST = 17


def default_store():
    import torch.distributed as dist
    if not dist.is_initialized():
        return None
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # pragma: no cover - private API moved
        return None


class Heartbeat(object):
    def __init__(self, store, rank, world, interval=1.0, timeout=30.0, logs_root="",
                 on_failure=None, prefix="cerebro_hb", stall_timeout=None):
        self.store = store
        self.rank, self.world = rank, world
        self.interval, self.timeout = interval, timeout
        self.stall_timeout = stall_timeout
        self._prog = [0, False, time.time()]      # step, busy, time of last change
        self.stalled = []
        self.logs_root = logs_root
        self.on_failure = on_failure or self._die
        self.prefix = prefix
        self.lost = []
        self._stop = threading.Event()
        self._threads = []

    def _key(self, r):
        return "{}/{}".format(self.prefix, r)

    def progress(self, step, busy):
        """Training thread: a job started (busy=True) or ended (False)."""
        self._prog = [int(step), bool(busy), time.time()]

    def beat(self):
        self.store.set(self._key(self.rank), json.dumps([time.time()] + self._prog))

    def records(self):
        """{rank: (stamp age, busy, seconds since the last progress mark)}."""
        now = time.time()
        out = {}
        for r in range(self.world):
            try:
                # check() first: get() on a missing key would block until timeout
                if not self.store.check([self._key(r)]):
                    out[r] = None
                    continue
                t, _, busy, tp = json.loads(self.store.get(self._key(r)).decode())
                out[r] = (now - t, busy, now - tp)
            except Exception:
                out[r] = (float("inf"), False, 0.0)
        return out

    def ages(self):
        return {r: (None if v is None else v[0]) for r, v in self.records().items()}

    def check(self):
        """Ranks whose heartbeat is stale, or that have been inside one job
        for longer than ``stall_timeout`` (never-started ranks are ignored)."""
        bad, stalled = [], []
        for r, v in self.records().items():
            if v is None:
                continue
            if v[0] > self.timeout:
                bad.append(r)
            elif self.stall_timeout and v[1] and v[2] > self.stall_timeout:
                bad.append(r)
                stalled.append(r)
        self.stalled = stalled
        return sorted(bad)

    def _beat_loop(self):
        while not self._stop.is_set():
            try:
                self.beat()
            except Exception:
                pass   # store gone: the watchdog (or the job) ends us
            self._stop.wait(self.interval)

    def _watch_loop(self):
        while not self._stop.wait(self.interval):
            lost = self.check()
            if lost:
                self.lost = lost
                self._report(lost)
                self.on_failure(lost)
                return

    def _report(self, lost):
        from ..utils.logging import logs
        for r in lost:
            if r in self.stalled:
                logs("WORKER {} STALLED (inside one job for > {:.0f}s)".format(
                    r, self.stall_timeout))
            else:
                logs("WORKER {} LOST (no heartbeat for > {:.0f}s)".format(r, self.timeout))
        if self.logs_root:
            os.makedirs(self.logs_root, exist_ok=True)
            with open(os.path.join(self.logs_root, "failed_workers.json"), "w") as f:
                json.dump({"lost": lost, "stalled": list(self.stalled), "time": time.time(),
                           "timeout": self.timeout, "stall_timeout": self.stall_timeout}, f)

    def _die(self, lost):  # pragma: no cover - exercised in multi-process runs
        os._exit(EXIT_WORKER_LOST)

    def start(self, watchdog=None):
        self.beat()
        t = threading.Thread(target=self._beat_loop, daemon=True)
        t.start()
        self._threads.append(t)
        if watchdog if watchdog is not None else self.rank == 0:
            w = threading.Thread(target=self._watch_loop, daemon=True)
            w.start()
            self._threads.append(w)
        return self

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)


# ---------------------------------------------------------------------------
# hop watchdog
# ---------------------------------------------------------------------------
EXIT_HOP_STALL = 18
EXIT_HOP_ERROR = 19      # a hop that failed (mis-order, corruption, service error), not a stall


class HopWatch(object):
    """Bounded waits for the hop data plane.

    A wedged RCCL group never raises before the process group's timeout
    (30 min), so a hang in a multi-GPU run would burn the whole job with no
    word on which hop stalled.  Every rank registers its in-flight hop
    operations here (``begin`` / ``end``): the hop service's header and
    payload groups, the lock-step runtime's boundary, and the main thread's
    wait for an arrival whose record is already published.  A daemon thread
    checks their ages every ``interval`` seconds; past ``bound()`` =
    ``timeout_s`` + 2 x the longest job this rank has heard of (a published
    hop's source can still be draining that job's kernels), or when another
    rank has raised the job-wide abort flag in the rendezvous store, it

    1. prints ``HOP WATCHDOG rank r: ...`` with every pending operation
       (kind, age, hop ids, models, peers, bytes), the groups posted and the
       last hops completed, to stderr,
    2. writes the same record to ``{logs_root}/hop_stall_rank{r}.json``,
    3. raises the abort flag (a local trigger) so every other rank reports
       and exits too, and
    4. ends the process with ``EXIT_HOP_STALL`` (``os._exit``: no re-exec,
       no waiting on the wedged communicator).

    ``abort(reason)`` is the same path for a hop error that would leave the
    peers blocked in a group (e.g. ``HopOrderError`` on one endpoint); it
    ends every rank with ``EXIT_HOP_ERROR`` and a record whose ``kind`` is
    ``"error"`` (a stall's is ``"stall"``), so the two are told apart.  Once
    ``stop()`` has been called (the run is ending) an abort is ignored: the
    caller's own exception and cleanup then run as usual."""

    def __init__(self, rank, world, timeout_s, store=None, key="cerebro_hopwatch",
                 logs_root="", interval=0.5, on_fire=None):
        self.rank, self.world = rank, world
        self.timeout_s = float(timeout_s)
        self.store = store
        self.key = key + "/abort"
        self.logs_root = logs_root
        self.interval = interval
        self.on_fire = on_fire or self._exit
        self.pending = {}
        self.lock = threading.Lock()
        self.jmax = 0.0
        self.groups = 0
        self.done = []
        self.fired = None
        self._n = 0
        self._stop = threading.Event()
        self._thread = None

    # -- registry ------------------------------------------------------------
    def begin(self, kind, t0=None, **info):
        with self.lock:
            self._n += 1
            self.pending[self._n] = dict(kind=kind, t0=time.time() if t0 is None else t0,
                                         **info)
            if kind == "group":
                self.groups += 1
            return self._n

    def end(self, tok):
        with self.lock:
            rec = self.pending.pop(tok, None)
            if rec is not None and rec.get("hops"):
                self.done = (self.done + list(rec["hops"]))[-16:]

    def note_job(self, seconds):
        if seconds and seconds > self.jmax:
            self.jmax = float(seconds)

    def bound(self):
        return self.timeout_s + 2.0 * self.jmax

    # -- watch thread ----------------------------------------------------------
    def start(self):
        self._thread = threading.Thread(target=self._loop, name="cerebro-hopwatch",
                                        daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _remote_abort(self):
        if self.store is None:
            return None
        try:
            if self.store.check([self.key]):
                return self.store.get(self.key).decode()
        except Exception:
            return None
        return None

    def check(self, now=None):
        """The first stalled operation (or None)."""
        now = time.time() if now is None else now
        b = self.bound()
        with self.lock:
            for tok, rec in self.pending.items():
                if now - rec["t0"] > b:
                    return rec
        return None

    def _loop(self):
        while not self._stop.wait(self.interval):
            rec = self.check()
            if rec is not None:
                self._fire("{} stalled for {:.1f}s (bound {:.1f}s)".format(
                    rec["kind"], time.time() - rec["t0"], self.bound()), local=True)
                return
            why = self._remote_abort()
            if why is not None:
                code, _, text = why.partition("|")
                code = int(code) if code.isdigit() else EXIT_HOP_STALL
                self._fire("abort raised by another rank: " + text, local=False, code=code)
                return

    def abort(self, reason, code=EXIT_HOP_ERROR):
        """A hop error on this rank: stop every rank now (see class doc)."""
        if self._stop.is_set():
            return
        self._fire(reason, local=True, code=code)

    def diagnostic(self, reason, code=EXIT_HOP_STALL):
        now = time.time()
        with self.lock:
            pend = [dict(rec, age_s=round(now - rec["t0"], 3)) for rec in self.pending.values()]
            for p in pend:
                p.pop("t0", None)
            return {"rank": self.rank, "world": self.world, "time": now, "reason": reason,
                    "kind": "stall" if code == EXIT_HOP_STALL else "error", "exit_code": code,
                    "bound_s": self.bound(), "pending": pend, "groups_posted": self.groups,
                    "last_done": list(self.done)}

    def _fire(self, reason, local, code=EXIT_HOP_STALL):
        import sys
        if self.fired is not None:
            return
        d = self.diagnostic(reason, code)
        self.fired = d
        msg = "HOP WATCHDOG rank {}: {}; pending {}; groups posted {}; last hops done {}".format(
            self.rank, reason, json.dumps(d["pending"]), d["groups_posted"], d["last_done"])
        try:
            sys.stderr.write(msg + "\n")
            sys.stderr.flush()
        except Exception:
            pass
        if self.logs_root:
            try:
                os.makedirs(self.logs_root, exist_ok=True)
                with open(os.path.join(self.logs_root,
                                       "hop_stall_rank{}.json".format(self.rank)), "w") as f:
                    json.dump(d, f)
            except Exception:
                pass
        if local and self.store is not None:
            try:
                self.store.set(self.key, "{}|rank {}: {}".format(code, self.rank, reason))
            except Exception:
                pass
        self.on_fire(d)

    def _exit(self, diag):  # pragma: no cover - exercised in multi-process runs
        os._exit(diag.get("exit_code", EXIT_HOP_STALL))
