"""Wall-clock event logging with the reference's line formats.

The reference's analysis tooling parses these exact strings, so the formats
are kept byte-compatible (reference ``cerebro_gpdb/utils.py:40-149``):

* ``logs(msg)``        -> ``"{msg}: YYYY-mm-dd HH:MM:SS"``
* ``logsc(name)``      -> ``"Start {name}: ..."`` / ``"End {name}: ..."`` and
  optionally ``"ELAPSED TIME: {s}"``
* ``DiskLogs(files)``  -> ``logs`` teed to files
* ``global.log`` START / END / TOTAL lines of ``runner_helper.sh:61-68``.
"""

import datetime
import os
import sys
import time

DEBUG = True


class LOG_KEYS(object):
    DATA_LOADING = "DATA LOADING"
    TRAINING = "TRAINING"
    VALIDATING = "VALIDATING"
    MODEL_INIT = "MODEL INITIALIZING"
    MODEL_TRAINVALID = "MODEL TRAIN/VALID"


def tstamp():
    return datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S")


_QUIET = os.environ.get("CEREBRO_QUIET", "0") == "1"


def logs(message):
    printed = "{}: {}".format(message, tstamp())
    if not _QUIET:
        print(printed)
        sys.stdout.flush()
    return printed


def DiskLogs(filenames):
    def logs_disk(message):
        printed = logs(message)
        for filename in filenames:
            with open(filename, "a") as f:
                f.write(printed + "\n")
    return logs_disk


def timeit_factory(debug=DEBUG):
    def timeit(func):
        def timed(*args, **kwargs):
            if debug:
                logs("Start inside {}".format(func.__name__))
            result = func(*args, **kwargs)
            if debug:
                logs("End inside {}".format(func.__name__))
            return result
        timed.__name__ = func.__name__
        return timed
    return timeit


class logsc(object):
    """Context manager printing Start/End lines, optionally recording elapsed s."""

    def __init__(self, log, debug=DEBUG, logs_fn=logs, elapsed_time=False,
                 log_dict=None):
        self.log = log
        self.debug = debug
        self.logs_fn = logs_fn
        self.elapsed_time = elapsed_time
        self.log_dict = log_dict if log_dict is not None else {}

    def __enter__(self):
        self.start = datetime.datetime.now()
        if self.debug:
            self.logs_fn("Start {}".format(self.log))
        return self

    def __exit__(self, exc_type, exc, tb):
        self.end = datetime.datetime.now()
        if self.debug:
            self.logs_fn("End {}".format(self.log))
        self.elapsed = (self.end - self.start).total_seconds()
        if self.elapsed_time:
            if not _QUIET:
                print("ELAPSED TIME: {}".format(self.elapsed))
            self.log_dict[self.log] = self.elapsed
        return False


class GlobalLog(object):
    """``global.log`` bracket of one experiment (runner_helper.sh PRINT_START/END).

    Makespan is measured exactly like the reference's shell ``SECONDS``:
    wall time between the Start and End lines.
    """

    def __init__(self, log_dir, exp_name):
        self.path = os.path.join(log_dir, "global.log")
        self.exp_name = exp_name
        os.makedirs(log_dir, exist_ok=True)

    def _write(self, line):
        with open(self.path, "a") as f:
            f.write(line + "\n")

    def start(self):
        self.t0 = time.time()
        self._write("{}, Start time: {}".format(self.exp_name, tstamp()))

    def end(self):
        seconds = time.time() - self.t0
        self._write("{}, End time: {}".format(self.exp_name, tstamp()))
        self._write("{}, TOTAL EXECUTION TIME OVER ALL MST {}".format(
            self.exp_name, int(round(seconds))))
        return seconds


_ONCE = set()


def log_once(message):
    """``logs`` a message the first time it is seen in this process."""
    if message in _ONCE:
        return None
    _ONCE.add(message)
    return logs(message)
