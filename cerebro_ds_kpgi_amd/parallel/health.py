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
