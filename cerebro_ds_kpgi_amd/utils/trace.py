"""Chrome-trace spans for runtime phases.

Each rank records spans (``hop``, ``train``, ``valid``, ``checkpoint``,
``etl``...) with wall-clock begin/end and optional HIP-event device
durations; ``Tracer.dump`` writes ``trace_rank{r}.json`` in the Chrome
``traceEvents`` format (open in chrome://tracing or Perfetto).  The span names
double as the reference's event vocabulary for the log analyzer
(``plots/plots.ipynb`` cell 0 ``semantics``).
"""

import contextlib
import json
import os
import threading
import time


class Tracer(object):
    def __init__(self, rank=0, enabled=True):
        self.rank = rank
        self.enabled = enabled
        self.events = []
        self.t0 = time.time()
        self._lock = threading.Lock()
        self._tids = {}

    def _tid(self):
        """One trace row per thread (main = 0; the asynchronous runtime's hop
        and coordinator threads get their own rows)."""
        name = threading.current_thread().name
        if name not in self._tids:
            self._tids[name] = 0 if name == "MainThread" else len(self._tids) + 1
        return self._tids[name]

    def _us(self, t):
        return (t - self.t0) * 1e6

    @contextlib.contextmanager
    def span(self, name, cat="runtime", sync=None, **args):
        if not self.enabled:
            yield
            return
        if sync is not None:
            sync()
        t = time.time()
        try:
            yield
        finally:
            if sync is not None:
                sync()
            e = time.time()
            with self._lock:
                self.events.append({"name": name, "cat": cat, "ph": "X", "ts": self._us(t),
                                    "dur": (e - t) * 1e6, "pid": self.rank,
                                    "tid": self._tid(), "args": args})

    def instant(self, name, **args):
        if self.enabled:
            with self._lock:
                self.events.append({"name": name, "ph": "i", "ts": self._us(time.time()),
                                    "pid": self.rank, "tid": self._tid(), "s": "p",
                                    "args": args})

    def dump(self, directory):
        if not self.enabled or not directory:
            return None
        os.makedirs(directory, exist_ok=True)
        path = os.path.join(directory, "trace_rank{}.json".format(self.rank))
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)
        return path

    def totals(self):
        out = {}
        for e in self.events:
            if e.get("ph") == "X":
                out[e["name"]] = out.get(e["name"], 0.0) + e["dur"] / 1e6
        return out


NULL = Tracer(enabled=False)
