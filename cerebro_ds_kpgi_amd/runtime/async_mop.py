"""Event-driven (asynchronous) MOP runtime: work-conserving greedy scheduling
and model hops overlapped with compute.

The lock-step runtime (``engine.MOPEngine.run_round``) ends every sub-epoch
with a barrier over all ranks, so a "greedy" schedule degenerates to
rotation and a hop can only start once every GPU is done.  This runtime
replaces the barrier with events (reference semantics:
``cerebro_gpdb/ctq.py:448-508`` -- an idle worker immediately takes the next
runnable (model, partition) pair; the client there busy-polls job
processes, here workers post completion events):

* **Coordinator** (a thread on rank 0) owns the scheduler.  Workers post
  ``train_done`` (the model's state is final -- it is free to start its next
  sub-epoch elsewhere while this worker still validates it) and ``job_done``
  (train + validation finished, metrics attached -- the worker is free).
  On every event the coordinator hands the next runnable pairs to idle
  workers (greedy) or, for rotation (UDAF), starts the next lock-step round
  once every worker is free -- but publishes that round's hops as soon as
  every model's training is done, so the transfers overlap validation.
* **Hop service** (one thread, one HIP stream and ONE communicator per
  rank): hops are published as one global sequence ``hop/0, hop/1, ...``
  (the coordinator publishes the hops of near-simultaneous events as one
  burst); every rank walks it in order and posts ALL the published
  transfers it is an endpoint of as one ``batch_isend_irecv`` group
  (``ncclGroupStart/End``), so a ring shift's send r->r+1 and receive
  r-1->r progress together, while the transfers overlap whatever the rank is
  computing.  Deadlock freedom and the stream budget are argued in
  ``HopService`` and ``profiles/r4_hop_design.md``.
  The receiver's compute stream waits on the arrival event only when the
  model is actually needed; ``hop_time`` counts that exposed wait, and
  ``hop_busy_time`` the transfers themselves.
* **Worker** (each rank's main thread): waits for its next assignment,
  trains its jobs packed per pack group (kept resident in the working
  arena: a job that stays on this GPU is a ``part_of_row`` change, no state
  copy), posts the events, validates.

Control messages ride a TCP key-value store (rank 0 hosts a
``torch.distributed.TCPStore``; an in-process store at world size 1), data
rides RCCL (gloo on CPU).  Fault handling: a ``SoftFault`` in a job sends
its pairs back to the queue (the model's previous holder still has its
pre-job state); anything else stops every rank with the error.
Checkpoints are epoch-granular here (sub-epoch ``resume`` uses the
lock-step runtime).
"""

import collections
import contextlib
import datetime
import json
import os
import statistics
import threading
import time

import torch
import torch.distributed as dist

from ..scheduler.policies import RotationScheduler
from ..utils.keys import model_key


# ---------------------------------------------------------------------------
# key-value control channel
# ---------------------------------------------------------------------------
class LocalStore(object):
    """In-process stand-in for TCPStore (world size 1): set / get / add / wait."""

    def __init__(self):
        self._d = {}
        self._cv = threading.Condition()

    def set(self, key, value):
        with self._cv:
            self._d[key] = value if isinstance(value, bytes) else str(value).encode()
            self._cv.notify_all()

    def add(self, key, n):
        with self._cv:
            v = int(self._d.get(key, b"0")) + int(n)
            self._d[key] = str(v).encode()
            self._cv.notify_all()
            return v

    def get(self, key, timeout=None):
        with self._cv:
            if not self._cv.wait_for(lambda: key in self._d, timeout):
                raise TimeoutError("LocalStore: no key {}".format(key))
            return self._d[key]

    def delete_key(self, key):
        with self._cv:
            self._d.pop(key, None)

    def check(self, keys):
        with self._cv:
            return all(k in self._d for k in keys)


class Channel(object):
    """Typed JSON messages over the store.  Streams: per-rank assignments
    ``a/<rank>/<k>``, the event log ``e/<i>`` (counter ``ne``), the global
    hop sequence ``h/<i>``, and the final state ``final``.

    A blocking TCPStore call holds the client's socket, so every thread
    talks through its own client (``fork``)."""

    def __init__(self, store, prefix, timeout, addr=None):
        self.store = store
        self.pfx = prefix
        self.timeout = timeout
        self.addr = addr

    def fork(self):
        if self.addr is None:
            return Channel(self.store, self.pfx, self.timeout)
        return Channel(tcp_client(self.addr, self.timeout), self.pfx, self.timeout, self.addr)

    def _k(self, *parts):
        return "/".join([self.pfx] + [str(p) for p in parts])

    def _get(self, key):
        if isinstance(self.store, LocalStore):
            return self.store.get(key, timeout=self.timeout)
        self.store.wait([key], datetime.timedelta(seconds=self.timeout))
        return self.store.get(key)

    def put(self, key_parts, obj):
        self.store.set(self._k(*key_parts), json.dumps(obj).encode())

    def take(self, key_parts):
        return json.loads(self._get(self._k(*key_parts)).decode())

    # events
    def post_event(self, ev):
        i = self.store.add(self._k("ne"), 1) - 1
        self.put(("e", i), ev)

    def event(self, i):
        return self.take(("e", i))

    # assignments / hops
    def assign(self, rank, k, rec):
        self.put(("a", rank, k), rec)

    def assignment(self, rank, k):
        return self.take(("a", rank, k))

    def hop(self, h, rec):
        self.put(("h", h), rec)

    def next_hop(self, h):
        return self.take(("h", h))

    def has_hop(self, h):
        """Non-blocking: is hop record ``h`` published yet?"""
        return self.store.check([self._k("h", h)])

    def has_event(self, i):
        """Non-blocking: is event ``i`` posted yet?"""
        return self.store.check([self._k("e", i)])

    def put_final(self, obj):
        self.put(("final",), obj)

    def get_final(self):
        return self.take(("final",))


def tcp_client(addr, timeout):
    """A client of the job's rendezvous store (MASTER_ADDR:MASTER_PORT, the
    store ``torch.distributed`` was initialised from -- no new listener)."""
    return dist.TCPStore(addr[0], addr[1], None, False,
                         timeout=datetime.timedelta(seconds=timeout), wait_for_workers=False)


def rendezvous_addr():
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = os.environ.get("MASTER_PORT")
    return (host, int(port)) if port else None


# ---------------------------------------------------------------------------
# coordinator (rank 0)
# ---------------------------------------------------------------------------
class Coordinator(object):
    """Scheduler owner, driven by completion events.

    * greedy: an idle rank takes, per idle partition it owns, the first
      runnable pair of the shuffled pair list (CTQ ``_get_runnable_model``);
    * rotation: the UDAF round plan, executed as a data flow -- rank r runs
      its share of round s+1 as soon as its round s is done and the models it
      needs for s+1 are trained (no global barrier: a slow rank delays only
      the ranks that wait for its models).  The visit order is exactly the
      round plan's, so results equal the lock-step runtime's.  A model's hop
      to its next partition is published the moment its training ends.

    ``round_budget`` limits a rotation session to that many rounds with
    ``steps_of(round)`` steps per job (``run_steps`` / the bench)."""

    def __init__(self, eng, chan, sched, policy, first_epoch, num_epochs, mst_eval_fn=None,
                 steps_of=None, round_budget=None):
        self.eng = eng
        self.chan = chan.fork()                        # this thread's own store client
        self.sched = sched
        self.policy = policy
        self.first_epoch = first_epoch
        self.num_epochs = num_epochs
        self.mst_eval_fn = mst_eval_fn
        self.steps_of = steps_of
        self.round_budget = round_budget
        self.world = eng.ctx.world
        self.parts_of = collections.defaultdict(list)
        for p in range(eng.P):
            self.parts_of[eng.owner(p)].append(p)
        self.k = collections.defaultdict(int)          # next assignment slot per rank
        self.ntk = 0                                   # hop tickets (decided hops)
        self.nseq = 0                                  # global hop sequence (published)
        self.nev = 0
        self.batch = {}                                # rank -> running batch record
        self.holder = dict(eng.holder)                 # committed state location
        self.hop_sent = {}                             # model -> rank a hop already targets
        self.retries = collections.Counter()
        self.error = None
        self.round_base = 0                            # rotation rounds of earlier epochs
        self.rounds_done = 0
        self.nbatch = 0                                # batches finished (greedy subepoch id)
        self._hop_buf = []                             # [ticket, record, t decided], unpublished
        self._train_s, self._train_n = 0.0, 0            # job training times
        self._train_recent = collections.deque(maxlen=32)  # recent job times (hold: median)
        self._train_max = 0.0                            # longest (hop watchdog bound)
        self.hops = None                                 # this rank's HopService (measured T)
        self.hold_log = []                               # (ticket, model, src, dst, held s, margin s)
        self.thread = None

    # -- plumbing ----------------------------------------------------------
    def start(self):
        self.thread = threading.Thread(target=self._main, name="cerebro-coordinator",
                                       daemon=True)
        self.thread.start()
        return self

    def join(self):
        if self.thread is not None:
            self.thread.join()

    def _send(self, rank, rec):
        self.chan.assign(rank, self.k[rank], rec)
        self.k[rank] += 1

    def _broadcast(self, rec):
        for r in range(self.world):
            self._send(r, rec)

    def _next_event(self):
        ev = self.chan.event(self.nev)
        self.nev += 1
        return ev

    def _main(self):
        try:
            self._run()
        except BaseException as e:          # never leave the workers waiting
            self.error = "{}: {}".format(type(e).__name__, e)
            try:
                self._flush_hops()
                self._broadcast({"t": "stop", "error": self.error})
                self.chan.hop(self.nseq, {"t": "stop"})
            except Exception:
                pass
            return
        self._flush_hops()
        self._broadcast({"t": "stop", "error": None})
        self.chan.hop(self.nseq, {"t": "stop"})

    # -- hop publication ---------------------------------------------------
    # A hop gets a *ticket* when it is decided (the job records name their
    # incoming hops by ticket) and a place in the global hop sequence only
    # when it is published, so hops can be published in any order.  Hops
    # published together form one burst: every rank's hop service finds them
    # at once and posts its share as ONE group on the one hop communicator.
    # A rotation's ring shift (each rank sends r -> r+1 and receives r-1 ->
    # r) wants one burst: published one by one, a rank's receive from its
    # predecessor would sit in front of its own send (one communicator = one
    # RCCL stream) and, when the ranks finish within a transfer time of each
    # other, the shift would chain through the ring (up to N transfer times
    # instead of one).
    #
    # Rotation therefore holds a decided hop back while a rank that is about
    # to finish is still training -- "about to" meaning its job has run for
    # the median job time give or take the hold margin (2 x the measured
    # transfer time, at least HOLD_MIN_S): only those ranks' hops can still
    # join the burst before a chain would cost more than the wait.  A rank
    # past that window (a straggler) or far from it (it started late) holds
    # nothing back, a hop to a rank that is still far from done is published
    # at once (its transfer overlaps the receiver's compute), and no hop is
    # held longer than the margin (or HOLD_MAX_S): the wait is bounded by what
    # a receiver would lose to a chain, not by the slowest rank or the job
    # length.
    HOLD_MIN_S = 0.002
    HOLD_MAX_S = 0.5
    HOP_GBPS = 50.0          # assumed per-hop rate until one is measured (xGMI, one link)

    def _flush_hops(self, entries=None):
        """Publish ``entries`` (default: every buffered hop) as one burst."""
        if entries is None:
            entries = self._hop_buf
        if not entries:
            return
        pub = {id(e) for e in entries}
        now = time.time()
        margin = self._margin_s()
        n = len(entries)
        for i, e in enumerate(entries):
            tk, rec, t_dec = e
            held = now - t_dec
            rec["more"] = i + 1 < n          # the burst continues: read on
            rec["hold"] = round(held, 6)
            self.chan.hop(self.nseq, rec)
            self.nseq += 1
            self.hold_log.append((tk, rec["m"], rec["src"], rec["dst"], held, margin))
        self._hop_buf = [e for e in self._hop_buf if id(e) not in pub]

    def _hop_est_s(self):
        """One hop's transfer time: measured on this rank's hop service once
        it has moved something, else the state row's bytes at HOP_GBPS."""
        svc = self.hops
        if svc is not None and svc.groups:
            return svc.busy / svc.groups
        return self.eng.hop_estimate_s(self.HOP_GBPS)

    def _margin_s(self):
        return min(self.HOLD_MAX_S, max(self.HOLD_MIN_S, 2.0 * self._hop_est_s()))

    def _about_to_finish(self, b, now, margin):
        if not self._train_recent:
            return True                           # nothing measured yet: every rank is
        med = statistics.median(self._train_recent)
        return abs((now - b["t0"]) - med) <= margin

    def _releasable(self, now):
        """The buffered hops to publish now (rotation hold, see above)."""
        if self.policy != "rotation":
            return list(self._hop_buf)
        margin = self._margin_s()
        buffered = {e[0] for e in self._hop_buf}
        # ranks really computing: training, with every incoming hop published
        computing = {r: b for r, b in self.batch.items() if b["train_left"] and
                     all(tk is None or tk not in buffered for tk in b["hops"])}
        near = {r for r, b in computing.items() if self._about_to_finish(b, now, margin)}
        out = []
        for e in self._hop_buf:
            if not near or now - e[2] >= margin:
                out.append(e)
            elif e[1]["dst"] in computing and e[1]["dst"] not in near:
                out.append(e)                     # overlaps the receiver's compute
        return out

    def _wait_event(self):
        """Next event; buffered hops are published before blocking on it."""
        while self._hop_buf:
            if self.chan.has_event(self.nev):
                break                                  # collect its hops too
            rel = self._releasable(time.time())
            if rel:
                self._flush_hops(rel)
            if not self._hop_buf:
                break
            time.sleep(0.0005)
        return self._next_event()

    def _budget_left(self):
        return self.round_budget is None or self.rounds_done < self.round_budget

    # -- epochs ------------------------------------------------------------
    def _run(self):
        eng = self.eng
        epoch = self.first_epoch
        self.last_epoch = epoch - 1
        while self._budget_left() and (self.round_budget is not None or
                                       epoch <= self.num_epochs):
            active = [m for m in range(len(eng.coord_msts))
                      if eng.mst_state[m]["state"] == "RUNNING"]
            if not active:
                break
            sched = self.sched
            sched.models = list(active)
            sched.start_epoch(epoch)
            self._broadcast({"t": "epoch", "epoch": epoch})
            eng.coord_log("EPOCH:{}".format(epoch))
            complete = self._run_epoch(epoch)
            if not complete:
                break                                  # bench budget hit mid-epoch
            sched.monitor.check_epoch_complete(sched.models)
            self._end_epoch(epoch)
            self.last_epoch = epoch
            epoch += 1

    def _run_epoch(self, epoch):
        """Returns False when a round budget stopped the epoch early."""
        sched = self.sched
        self.epoch_nbatch = 0
        self._next_where = None
        if self.policy == "rotation":
            self.L = len(sched.rounds)
            self.rnext = {r: 0 for r in range(self.world)}
            self.where = [{m: p for p, m in rnd.items()} for rnd in sched.rounds]
            for m in sched.models:
                s0 = self._mnext(m)
                if s0 is not None and self._round_allowed(s0):
                    self._pre_hop(m, self.eng.owner(self.where[s0][m]))
        self._pump(epoch)
        while self.batch:
            self._handle(self._wait_event(), epoch)
            self._pump(epoch)
        self._flush_hops()
        if self.policy == "rotation":
            done = min(self.rnext.values()) if self.rnext else 0
            self.round_base += self.L
            self.rounds_done = self.round_base if done >= self.L else self.round_base - self.L + done
            return sched.epoch_done()
        if not sched.epoch_done():
            raise RuntimeError("greedy scheduler stalled with pending pairs {}".format(
                sched.pending[:6]))
        return True

    def _round_allowed(self, s):
        return self.round_budget is None or self.round_base + s < self.round_budget

    # -- dispatch ----------------------------------------------------------
    def _pump(self, epoch):
        if self.policy == "rotation":
            self._pump_rotation(epoch)
        else:
            self._pump_greedy(epoch)

    def _pump_greedy(self, epoch):
        sched = self.sched
        for r in range(self.world):
            if r in self.batch:
                continue
            got = sched.assign_many([p for p in self.parts_of[r] if p in sched.idle_workers])
            jobs = [(m, p) for p, m in got.items()]
            if jobs:
                self._dispatch(r, jobs, epoch, self.round_base + self.epoch_nbatch)

    def _pump_rotation(self, epoch):
        sched = self.sched
        for r in range(self.world):
            if r in self.batch:
                continue
            s = self.rnext[r]
            while s < self.L and self._round_allowed(s):
                jobs = [(m, p) for p, m in sorted(sched.rounds[s].items())
                        if self.eng.owner(p) == r and (m, p) in sched.pending]
                if jobs:
                    break
                s += 1                                 # nothing of round s on this rank
            self.rnext[r] = s
            if s >= self.L or not self._round_allowed(s):
                continue
            if not all(m in sched.idle_models and self._mnext(m) == s for m, _ in jobs):
                continue                               # a model it needs is not there yet
            for m, p in jobs:
                sched._start(m, p)
            self._dispatch(r, jobs, epoch, self.round_base + s, rnd=s)

    def _mnext(self, m):
        """Rotation: the first round in which m still has a pending visit."""
        pend = self.sched.pending
        for s, where in enumerate(self.where):
            p = where.get(m)
            if p is not None and (m, p) in pend:
                return s
        return None

    def _pre_hop(self, m, dst):
        """Decide m's hop to ``dst`` (its state is final; published by
        ``_wait_event``); returns the hop's ticket (None: no transfer needed)."""
        src = self.holder.get(m)
        if src is None or src == dst:
            return None
        sent = self.hop_sent.get(m)
        if sent is not None and sent[0] == dst:
            return sent[1]
        tk = self.ntk
        self._hop_buf.append([tk, {"t": "hop", "tk": tk, "m": m, "src": src, "dst": dst,
                                   "jt": self._train_max}, time.time()])
        self.ntk += 1
        self.hop_sent[m] = (dst, tk)
        return tk

    def _prefetch_next_epoch(self, m):
        """Rotation, m's last visit of the epoch just ended: its first visit
        of the next epoch is known when no ``mst_eval_fn`` can change the
        active set -- start that hop now, behind this epoch's validation."""
        if self.mst_eval_fn is not None or (self.round_budget is None and
                                            self.sched.epoch >= self.num_epochs):
            return
        if getattr(self, "_next_where", None) is None:
            nxt = RotationScheduler(list(self.sched.models), list(self.sched.workers))
            nxt.pack_key_fn = self.sched.pack_key_fn      # the same order as the real one
            nxt.start_epoch(self.sched.epoch + 1)
            self._next_where = [{mm: p for p, mm in rnd.items()} for rnd in nxt.rounds]
        for s, where in enumerate(self._next_where):
            if m in where:
                if self.round_budget is None or self.round_base + self.L + s < self.round_budget:
                    self._pre_hop(m, self.eng.owner(where[m]))
                return

    def _dispatch(self, r, jobs, epoch, subepoch, rnd=None):
        recs = []
        for m, p in jobs:
            src = self.holder.get(m)
            recs.append([m, p, src, self._pre_hop(m, r)])
        self.batch[r] = {"jobs": recs, "train_left": {m for m, _ in jobs},
                         "subepoch": subepoch, "round": rnd, "t0": time.time(),
                         "hops": [rec[3] for rec in recs]}
        steps = (self.steps_of(self.round_base + rnd)
                 if (self.steps_of is not None and rnd is not None) else None)
        self._send(r, {"t": "jobs", "epoch": epoch, "jobs": recs, "max_steps": steps,
                       "subepoch": subepoch})

    # -- events ------------------------------------------------------------
    def _handle(self, ev, epoch):
        eng = self.eng
        t = ev["t"]
        r = ev["rank"]
        b = self.batch.get(r)
        if t == "train_done":
            jt = time.time() - b["t0"]
            self._train_s += jt
            self._train_n += 1
            self._train_recent.append(jt)
            self._train_max = max(self._train_max, jt)
            for m in ev["models"]:
                p = next(p for mm, p, _, _ in b["jobs"] if mm == m)
                self.sched.release_model(m, p)
                self.holder[m] = r
                self.hop_sent.pop(m, None)
                b["train_left"].discard(m)
                if b["round"] is not None:
                    s2 = self._mnext(m)
                    if s2 is None:
                        self._prefetch_next_epoch(m)
                    elif self._round_allowed(s2):
                        self._pre_hop(m, eng.owner(self.where[s2][m]))
            return
        if t != "job_done":
            raise RuntimeError("unknown event {}".format(ev))
        del self.batch[r]
        if ev.get("fatal"):
            raise RuntimeError("rank {} failed: {}".format(r, ev["error"]))
        if ev.get("error"):                           # SoftFault: requeue the pairs
            for m, p, src, _ in b["jobs"]:
                if m not in b["train_left"]:
                    continue                           # trained; only its metrics are lost
                self.retries[(m, p)] += 1
                if self.retries[(m, p)] > eng.o.max_retries:
                    raise RuntimeError("pair {} failed {} times; giving up".format(
                        (m, p), self.retries[(m, p)]))
                self.sched.abort(m, p)
                # the failed rank received every incoming state before it
                # failed and its home rows hold the pre-job states
                self.holder[m] = r
                self.hop_sent.pop(m, None)
                fj = {"status": "FAILED", "epoch": epoch, "subepoch": b["subepoch"],
                      "attempt": self.retries[(m, p)] - 1, "rank": r, "partition": p,
                      "error": ev["error"], "model_key": model_key(m, eng.coord_msts[m])}
                eng.failures.append(fj)
                eng.coord_log("JOB FAILED {} on partition {} (rank {}): {} -> requeued"
                              .format(fj["model_key"], p, r, ev["error"]))
            for m, p, _, _ in b["jobs"]:
                self.sched.release_worker(p)
            return
        for m, p, _, _ in b["jobs"]:
            self.sched.release_worker(p)
        g = {"rank": r, "t_start": ev["t_start"], "t_hop": ev["t_hop"], "t_end": ev["t_end"]}
        for res in ev["results"]:
            eng._record_job(epoch, g, res, subepoch=b["subepoch"])
        eng.round_idx += 1
        self.epoch_nbatch += 1
        if b["round"] is not None:
            self.rnext[r] = b["round"] + 1

    def _end_epoch(self, epoch):
        eng = self.eng
        eng._epoch_summary(epoch)
        if eng.o.logs_root:
            from .checkpoint import dump_infos
            dump_infos(eng.o.logs_root, eng.models_info, eng.jobs_info)
        if self.mst_eval_fn is not None:
            stop, _, new_msts = self.mst_eval_fn(eng.mst_state)
            for m in stop:
                eng.mst_state[m]["state"] = "COMPLETED"
            if new_msts:
                ids = eng.coord_add_msts(new_msts)
                self.sched.add_models(ids)
                self._broadcast({"t": "add", "msts": new_msts})
                for m in ids:
                    self.holder[m] = None
        if eng.o.ckpt_every != "none" and eng.o.models_root:
            by_rank = collections.defaultdict(list)
            for m in range(len(eng.coord_msts)):
                h = self.holder.get(m)
                by_rank[0 if h is None else h].append(m)
            for r in range(self.world):
                self._send(r, {"t": "ckpt", "epoch": epoch, "models": by_rank.get(r, []),
                               "version": eng.ckpt_version(epoch)})
            acks = 0
            while acks < self.world:
                ev = self._next_event()
                if ev["t"] != "ckpt_done":
                    raise RuntimeError("unexpected event at checkpoint: {}".format(ev))
                acks += 1
            eng.write_resume(epoch, -1, True, None, version=eng.ckpt_version(epoch))


# ---------------------------------------------------------------------------
# hop service (every rank, world > 1)
# ---------------------------------------------------------------------------
class HopService(object):
    """Walks the global hop sequence and posts every transfer this rank is
    an endpoint of, on ONE process group (one RCCL communicator, created once
    by ``MOPEngine``), from ONE thread, on ONE HIP stream.

    Each pass takes every hop record already published after the last one
    it posted (at least one: it blocks for the next) and posts this rank's
    transfers among them, in global order, as ONE ``batch_isend_irecv`` group
    (``ncclGroupStart; Send/Recv...; ncclGroupEnd``); the pass ends when the
    group has completed.  A rotation's ring shift (every rank sends r -> r+1
    and receives r-1 -> r) is published as one burst by the coordinator, so
    each rank's send and receive progress together in one group.

    Why this cannot deadlock (RCCL semantics):

    * per rank pair, both endpoints post their common transfers in global
      hop order (NCCL matches point-to-point operations per peer in posting
      order; a debug digest travels right after its transfer, on both sides);
    * calls inside a group progress independently of each other, so a group
      is blocked only by an operation whose peer has not yet posted it;
    * groups are contiguous ranges of a rank's transfers in global order.
      If rank a's running group waits for transfer x, the peer b is still
      running a group whose transfers all precede x; that group waits for a
      transfer y < x, and so on: the chain of hop ids strictly decreases, so
      the smallest blocked transfer has both endpoints posted and completes.
      Different ranks may split the sequence into different groups; the
      argument does not need them to agree.
    * One communicator means one RCCL stream: its kernels are issued in that
      same global order on the process's hardware queues, so no kernel of
      another communicator can sit in front of it in a shared queue (the
      hazard of the round-3 design: 7 two-rank communicators per rank, driven
      concurrently from 7 threads).

    A send first makes the hop stream wait (device side) for the model's
    parking copy only; an arrival is a HIP event the compute stream waits on
    when the model is needed.  Stream budget: ``profiles/r4_hop_design.md``."""

    MAX_GROUP = 64                            # hop records per pass, at most

    def __init__(self, eng, chan, group):
        self.eng = eng
        self.chan = chan.fork()
        self.rank = eng.ctx.rank
        self.group = group
        self.cuda = eng.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=eng.device) if self.cuda else None
        self.final = {}                       # model -> cuda event of its last parking
        self.arrived = {}                     # hop ticket -> [threading.Event, cuda event]
        self.lock = threading.Lock()
        self._cv = threading.Condition()      # in-flight group / pause (quiet)
        self._inflight = 0
        self._paused = False
        self.bytes = 0
        self.busy = 0.0
        self.groups = 0                       # batch_isend_irecv groups posted
        self.spans = []                       # (t0, t1, "send"|"recv", model, peer, bytes, seq, hold)
        self.hold = 0.0                       # coordinator hold of the hops received here
        self.error = None
        self.stopping = False                     # the stop record has been read
        self.watch = eng.hop_watch                # parallel.health.HopWatch (or None)
        self.seen = {}                            # hop ticket -> time its record was read
        self.thread = None

    def start(self):
        self.thread = threading.Thread(target=self._main, name="cerebro-hops", daemon=True)
        self.thread.start()
        return self

    def join(self):
        if self.thread is not None:
            self.thread.join()

    # -- main-thread API ---------------------------------------------------
    def mark_final(self, m):
        """Main thread: m's state is parked in its home row (enqueued)."""
        ev = None
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
        with self.lock:
            self.final[m] = ev

    def wait_arrival(self, h):
        """Main thread: block until the hop with ticket ``h`` has landed
        (host side), then order the compute stream after it (device side)."""
        with self.lock:
            slot = self.arrived.setdefault(h, [threading.Event(), None])
        tok = None
        try:
            while not slot[0].wait(0.5):
                if self.error:
                    raise RuntimeError("hop service failed: " + self.error)
                if tok is None and self.watch is not None:
                    # bounded from the moment the record was published
                    # (before that, the source is still training the model)
                    with self.lock:
                        ts = self.seen.get(h)
                    if ts is not None:
                        tok = self.watch.begin("arrival", t0=ts, hops=[h])
        finally:
            if tok is not None:
                self.watch.end(tok)
        if slot[1] is not None:
            torch.cuda.current_stream().wait_event(slot[1])
        with self.lock:
            del self.arrived[h]
            self.seen.pop(h, None)

    class _Quiet(object):
        def __init__(self, svc):
            self.svc = svc

        def __enter__(self):
            with self.svc._cv:
                self.svc._paused = True
                while self.svc._inflight:
                    self.svc._cv.wait(1.0)
            return self

        def __exit__(self, *exc):
            with self.svc._cv:
                self.svc._paused = False
                self.svc._cv.notify_all()
            return False

    def quiet(self):
        """Context: no transfer runs inside (the home arena may be rebuilt)."""
        return HopService._Quiet(self)

    # -- service thread ----------------------------------------------------
    def _main(self):
        try:
            if self.cuda:
                with torch.cuda.device(self.eng.device), torch.cuda.stream(self.stream):
                    self._loop()
            else:
                self._loop()
        except BaseException as e:
            self.error = "{}: {}".format(type(e).__name__, e)
            if self.watch is not None and not self.stopping:
                # peers may sit in a group with this rank: stop every rank
                # with a diagnostic rather than leave them blocked (exit code
                # EXIT_HOP_ERROR, not a stall; skipped once the stop record
                # is in: the run is being torn down and the main thread's
                # own error path reports)
                self.watch.abort("hop service failed on rank {}: {}".format(
                    self.rank, self.error))

    def _loop(self):
        h = 0
        while True:
            recs = [(h, self.chan.next_hop(h))]          # blocks for the next record
            h += 1
            # the rest of a burst (being written), then any later burst
            # already published
            while (recs[-1][1]["t"] != "stop" and len(recs) < self.MAX_GROUP
                   and (recs[-1][1].get("more") or self.chan.has_hop(h))):
                recs.append((h, self.chan.next_hop(h)))
                h += 1
            stop = recs[-1][1]["t"] == "stop"
            self.stopping = self.stopping or stop
            mine = [(hid, r["m"], r["src"], r["dst"], r["tk"], r.get("hold", 0.0))
                    for hid, r in recs if r["t"] == "hop" and self.rank in (r["src"], r["dst"])]
            now = time.time()
            with self.lock:
                for hid, r in recs:
                    if r["t"] == "hop" and r["dst"] == self.rank:
                        self.seen[r["tk"]] = now
            if self.watch is not None:
                self.watch.note_job(max(r.get("jt", 0.0) for _, r in recs))
            if mine:
                with self._cv:
                    while self._paused:
                        self._cv.wait(1.0)
                    self._inflight += 1
                try:
                    self._post_group(mine)
                finally:
                    with self._cv:
                        self._inflight -= 1
                        self._cv.notify_all()
            if stop:
                return

    def _post_group(self, items):
        """Post ``items`` (this rank's transfers, global order) as one group
        and wait for it (``parallel.hop.post_transfers``: headers checked
        first, then the payloads); then publish the arrivals."""
        from ..parallel.hop import checksum, post_transfers, verify_digests
        eng = self.eng
        tx, nsend = [], 0
        t0 = time.time()
        tk_of = {it[0]: it[4] for it in items}
        for hid, m, src, dst, _, _ in items:
            grp = eng.group_of[m]
            row = grp.home.state[grp.home_row[m]]
            buf = row if eng.o.hop_optimizer_state else row[:grp.layout.n_master]
            if self.rank == src:
                with self.lock:
                    ev = self.final.get(m)
                if ev is not None:
                    self.stream.wait_event(ev)           # the parking copy only
                nsend += 1
                with self.lock:
                    self.bytes += buf.numel() * buf.element_size()
            tx.append((hid, m, src, dst, buf))
        digest_of = (lambda m, b: checksum(b)) if eng.o.hop_check else None
        with eng.tracer.span("hop", n=len(items), sends=nsend, recvs=len(tx) - nsend):
            if nsend and eng.o.sim_hop_seconds:           # test hook: slow links
                time.sleep(eng.o.sim_hop_seconds)
            if eng.o.sim_hop_stall == self.rank and self.watch is not None:
                # test hook: this rank's first group wedges (a hung RCCL call)
                self.watch.begin("group", hops=[it[0] for it in tx], stalled_by_test=True)
                time.sleep(3600)
            recvs = post_transfers(tx, self.rank, self.group, digest_of=digest_of,
                                   watch=self.watch)
            done = None
            if self.cuda:
                done = torch.cuda.Event()
                done.record(self.stream)
                self.stream.synchronize()
        self.groups += 1
        verify_digests(recvs, self.rank)
        t1 = time.time()
        with self.lock:
            self.busy += t1 - t0
            for (hid, m, src, dst, _, hold), (_, _, _, _, buf) in zip(items, tx):
                send = self.rank == src
                self.spans.append((t0, t1, "send" if send else "recv", m, dst if send else src,
                                   buf.numel() * buf.element_size(), hid, hold))
                if not send:
                    self.hold += hold
            for hid, m, _, _ in recvs:
                slot = self.arrived.setdefault(tk_of[hid], [threading.Event(), None])
                slot[1] = done
                slot[0].set()


# ---------------------------------------------------------------------------
# worker (every rank's main thread)
# ---------------------------------------------------------------------------
def run_worker(eng, chan, hops):
    """Execute this rank's assignment stream until ``stop``; returns the
    coordinator's error (None on success)."""
    rank = eng.ctx.rank
    k = 0
    while True:
        rec = chan.assignment(rank, k)
        k += 1
        t = rec["t"]
        if t == "stop":
            return rec.get("error")
        if t == "epoch":
            eng.epoch = rec["epoch"]
            eng.store.new_epoch(rec["epoch"])
            continue
        if t == "add":
            if hops is not None:
                with hops.quiet():                  # no transfer reads the old home arena
                    eng.worker_add_msts(rec["msts"])
            else:
                eng.worker_add_msts(rec["msts"])
            continue
        if t == "ckpt":
            for grp in eng.groups.values():
                grp.park_all()
            eng.checkpoint_all(rec["epoch"], models=rec["models"], holder_ok=True,
                               version=rec.get("version"))
            eng.writer.flush()
            chan.post_event({"t": "ckpt_done", "rank": rank})
            continue
        assert t == "jobs", rec
        _run_batch(eng, chan, hops, rec)


class _Lanes(object):
    """Concurrent pack groups within one batch.  A group past its warm-up
    (``_Working.replay_ready``: its steps are graph replays, no host-side op
    runs) sends its work to the stream of its lane (``PackGroup.lane``;
    ``engine.lane_stream``) after that stream has waited for the caller's
    (hop arrivals, parking); ``join`` makes the caller's stream wait for every
    lane.  Groups sharing a lane share its stream (and the lane's split-K
    workspace, baked into their graphs), so they stay serialised.  A group
    still warming up (its eager steps autotune kernels and must not be timed
    beside other work) runs on the caller's stream BEFORE any lane work is
    issued (``order``): in a Hyperopt run new trials keep bringing new pack
    groups, and a batch with one warming group used to run all of its groups
    serially.  On the CPU, or with fewer than two ready groups, everything
    runs on the caller's stream."""

    def __init__(self, eng, working, valid):
        cuda = eng.device.type == "cuda"
        self.ready = {k for k, w in working.items() if cuda and w.replay_ready(valid)}
        self.active = len(self.ready) > 1
        self.eng = eng
        self.main = torch.cuda.current_stream() if self.active else None
        self.used = {}
        if self.active:
            eng.lane_batches += 1

    def order(self, working):
        """Group keys, warming-up groups first (they run on the caller's stream)."""
        return sorted(working, key=lambda k: k in self.ready)

    def on(self, grp, key=None):
        if not self.active or (key is not None and key not in self.ready):
            return contextlib.nullcontext()
        st = self.used.get(grp.lane)
        if st is None:
            st = self.eng.lane_stream(grp.lane)
            st.wait_stream(self.main)
            self.used[grp.lane] = st
        return torch.cuda.stream(st)

    def join(self):
        for st in self.used.values():
            self.main.wait_stream(st)


def _run_batch(eng, chan, hops, rec):
    from .engine import SoftFault
    rank = eng.ctx.rank
    tr = eng.tracer
    t_start = time.time()
    jobs = [tuple(j) for j in rec["jobs"]]         # (model, partition, holder, hop ticket)
    models = [j[0] for j in jobs]
    error = None
    results, trained = [], 0
    t_hop = t_start
    eng.mark_progress(True)
    try:
        # arrivals: the compute stream waits for a hop only now
        with tr.span("wait_arrival", subepoch=rec["subepoch"]):
            for m, p, src, hid in jobs:
                if hid is not None:
                    hops.wait_arrival(hid)
                    eng.group_of[m].invalidate(m)
        t_hop = time.time()
        eng.hop_time += t_hop - t_start
        eng._fault_check_batch(rec["subepoch"])
        per_group = collections.defaultdict(list)
        for m, p, _, _ in jobs:
            per_group[eng.group_of[m].key].append((m, eng.local_part(p)))
        working = {}
        for key, gj in per_group.items():
            working[key] = eng.groups[key].begin_batch(gj)
        steps_of = {}
        # several pack groups whose steps are all graph replays run at once,
        # one stream per lane (the groups' first steps -- eager warm-up with
        # kernel autotuning, capture -- stay serial on the caller's stream)
        lanes = _Lanes(eng, working, valid=False)
        for key in lanes.order(working):
            w = working[key]
            grp = eng.groups[key]
            B = grp.batch_size
            steps = eng.n_train // B
            if rec.get("max_steps"):
                steps = min(steps, rec["max_steps"])
            steps_of[key] = steps
            with lanes.on(grp, key), tr.span("train", sync=eng._sync, arch=key[0], G=w.G,
                                        steps=steps):
                w.prepare(eng.o.hop_optimizer_state)
                w.train_steps(steps)
                delay = eng.o.sim_job_seconds
                if delay:                            # test hook: heterogeneous job lengths
                    time.sleep(max(delay[m % len(delay)] for m, _ in w.jobs))
            trained += steps * B * w.G
        lanes.join()
        # the states are final: park them (the home row is the committed
        # copy a hop or a retry starts from), then free the models
        for key in working:
            eng.groups[key].park_all()
        if hops is not None:
            for m in models:
                hops.mark_final(m)
        chan.post_event({"t": "train_done", "rank": rank, "models": models})
        vlanes = _Lanes(eng, working, valid=True)
        for key in vlanes.order(working):
            w = working[key]
            grp = eng.groups[key]
            B = grp.batch_size
            vsteps = eng.n_valid // B
            if rec.get("max_steps"):
                full = max(eng.n_train // B, 1)
                vsteps = max(1, -(-vsteps * steps_of[key] // full))
            with vlanes.on(grp, key), tr.span("valid", sync=eng._sync, arch=key[0], G=w.G,
                                         steps=vsteps):
                w.validate(vsteps)
                if eng.o.sim_valid_seconds:
                    time.sleep(eng.o.sim_valid_seconds)
        vlanes.join()
        for key, w in working.items():
            B = eng.groups[key].batch_size
            mets = w.read_metrics()                 # one host sync per group
            for row, (m, lp) in enumerate(w.jobs):
                results.append({"model": m, "dist_key": eng.store.pids[lp], "metrics": mets[row],
                                "steps": steps_of[key], "batch": B, "partition": lp})
    except SoftFault as e:
        # every incoming state has arrived; the home rows hold the pre-job
        # states, the working copies of this batch are void
        error = str(e)
        for grp in eng.groups.values():
            grp.drop_residency(models)
    except BaseException as e:
        chan.post_event({"t": "job_done", "rank": rank, "error": "{}: {}".format(
            type(e).__name__, e), "fatal": True, "results": [], "t_start": t_start,
            "t_hop": t_start, "t_end": time.time()})
        raise
    if eng._sync is not None:
        eng._sync()
    if eng.hop_watch is not None:
        eng.hop_watch.note_job(time.time() - t_start)
    if error is None:
        eng.train_images += trained
    eng.mark_progress(False)
    with tr.span("report", subepoch=rec["subepoch"]):
        chan.post_event({"t": "job_done", "rank": rank, "error": error, "fatal": False,
                         "results": results, "t_start": t_start, "t_hop": t_hop,
                         "t_end": time.time()})


# ---------------------------------------------------------------------------
# session driver
# ---------------------------------------------------------------------------
def run_session(eng, policy, first_epoch, num_epochs, mst_eval_fn=None, steps_of=None,
                round_budget=None):
    """One asynchronous run on every rank (collective); returns when the
    coordinator stops.  Rank 0's coordinator state (metrics, holders) is
    shared with every rank at the end."""
    ctx = eng.ctx
    chan = eng.control_channel()
    hops = None
    if ctx.world > 1:
        hops = HopService(eng, chan, eng.hop_group()).start()
    coord = None
    if ctx.rank == 0:
        eng.coord_begin()
        coord = Coordinator(eng, chan, eng.async_scheduler(policy), policy, first_epoch,
                            num_epochs, mst_eval_fn, steps_of, round_budget)
        coord.hops = hops
        coord.start()
    err = None
    try:
        err = run_worker(eng, chan, hops)
    finally:
        if coord is not None:
            coord.join()
        if hops is not None:
            hops.join()
    if coord is not None:
        err = err or coord.error
    for grp in eng.groups.values():
        grp.park_all()
    if hops is not None:
        eng.hop_bytes += hops.bytes
        eng.hop_busy_time += hops.busy
        eng.hop_groups += hops.groups
        eng.hop_hold_time += hops.hold
        eng.hop_spans.extend(hops.spans)
        if hops.error and not err:
            err = "hop service: " + hops.error
    # share rank 0's bookkeeping with every rank (JSON over the control store)
    if ctx.rank == 0:
        chan.put_final({
            "holder": {str(m): h for m, h in coord.holder.items()},
            "mst_state": {str(m): v for m, v in eng.mst_state.items()},
            "jobs_info": {str(e): [[k[0], k[1], j] for k, j in jobs.items()]
                          for e, jobs in eng.jobs_info.items()},
            "models_info": dict(eng.models_info), "msts": eng.coord_msts,
            "failures": eng.failures, "round_idx": eng.round_idx, "error": err,
            "last_epoch": coord.last_epoch, "rounds_done": coord.rounds_done})
    fin = chan.get_final()
    if hops is not None:
        # per-hop telemetry of the session into rank 0's metrics.jsonl
        # (bytes, post -> arrival, coordinator hold, peer)
        spans = ctx.all_gather_object(hops.spans)
        if ctx.rank == 0:
            eng.log_hop_records(spans, coord.hold_log)
    ctx.barrier()
    eng.coord_end(fin)
    if fin["error"]:
        raise RuntimeError("asynchronous MOP run failed: " + fin["error"])
    return fin
