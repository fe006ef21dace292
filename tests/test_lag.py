"""Lagged Adam (runtime/group.py ``_lag_issue``): chunk boundaries (CPU) and
the arena's wait bookkeeping (no GPU needed for the boundaries)."""

from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.runtime.group import lag_bounds


def test_lag_bounds_cover_the_arena_at_parameter_starts():
    layout = create_model_from_mst({"model": "resnet50"}).layout
    b = lag_bounds(layout)
    starts = {s.offset for s in layout.train_specs}
    assert b[0] == 0 and b[-1] == layout.n_train
    assert all(x < y for x, y in zip(b, b[1:]))
    assert all(x in starts for x in b[1:-1])
    assert all(x % 8 == 0 for x in b)
    # the first chunk (what the stem waits for) is a small slice of the arena
    assert b[1] <= layout.n_train // 16
    assert 4 <= len(b) - 1 <= 8


def test_lag_bounds_tiny_layout():
    layout = create_model_from_mst({"model": "resnet18"}).layout
    b = lag_bounds(layout, fracs=(0.5,))
    assert b[0] == 0 and b[-1] == layout.n_train and len(b) in (2, 3)
