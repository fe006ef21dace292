"""Scheduling logic of the batched weight gradients (ops/streams.py), on CPU.

The GPU tier checks the numerics of the side-stream split
(tests/test_graph_gpu.py); here the launch pattern itself is pinned with the
flush replaced by a recorder: the adaptive split (packs of >= 4 configs,
runtime/group.py) launches ONE side batch of ceil(frac * previous step's
layer count) layers and the tail on the current stream.
"""

import pytest

from cerebro_ds_kpgi_amd.ops import streams as S


@pytest.fixture
def recorder(monkeypatch):
    calls = []
    count = [0]

    def fake_hold_count(*a, **k):
        pass

    def fake_flush(discard=False, side=False):
        if not S._HELD:
            return
        calls.append(("side" if side else "main", len(S._HELD), S._SPLIT_GRID if side else 0))
        del S._HELD[:]

    monkeypatch.setattr(S, "flush_wgrad", fake_flush)
    monkeypatch.setattr(S.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(S, "_LAST", {})
    yield calls


@pytest.mark.parametrize("n,frac,want", [(53, 0.5, 27), (54, 0.5, 27), (10, 0.4, 4)])
def test_adaptive_split_one_side_batch_then_tail(recorder, n, frac, want):
    for step in range(3):
        del recorder[:]
        with S.deferred_wgrad(True, side_frac=frac, key="k"):
            for i in range(n):
                S.hold(object(), grad_ptr=4 * i)
        if step == 0:      # no layer count yet: one batch at the end
            assert recorder == [("main", n, 0)]
        else:
            assert recorder == [("side", want, S._SPLIT_GRID), ("main", n - want, 0)]
    assert S._SPLIT_AT == 0 and not S._DEFER


def test_no_split_without_fraction(recorder):
    for _ in range(2):
        with S.deferred_wgrad(True, key="small"):
            for i in range(20):
                S.hold(object())
    assert recorder == [("main", 20, 0)] * 2


def test_layer_counts_are_per_key(recorder):
    with S.deferred_wgrad(True, side_frac=0.5, key="a"):
        for i in range(40):
            S.hold(object())
    with S.deferred_wgrad(True, side_frac=0.5, key="b"):
        for i in range(8):
            S.hold(object())
    del recorder[:]
    with S.deferred_wgrad(True, side_frac=0.5, key="b"):
        for i in range(8):
            S.hold(object())
    assert recorder == [("side", 4, S._SPLIT_GRID), ("main", 4, 0)]
