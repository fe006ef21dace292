"""Restricted unpickling of run records (utils/safe_pickle.py)."""

import os
import pickle

import numpy as np
import pytest

from cerebro_ds_kpgi_amd.utils import safe_pickle


def test_round_trip_of_ctq_records():
    rec = {"model_1": [{"epoch": 1, "loss_train": 6.9, "metric_valid": np.float32(0.12),
                        "start": 1.0, "ok": True, "tags": ("a", "b")}],
           "jobs": [[0, 1, 2]], "n": np.int64(3)}
    got = safe_pickle.loads(pickle.dumps(rec))
    assert got["model_1"][0]["loss_train"] == 6.9
    assert float(got["model_1"][0]["metric_valid"]) == pytest.approx(0.12)
    assert int(got["n"]) == 3


class _Evil(object):
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_refuses_globals_outside_the_allowlist():
    with pytest.raises(pickle.UnpicklingError):
        safe_pickle.loads(pickle.dumps(_Evil()))
