"""The profiling tools that turn rocprofv3 output into the tables under
profiles/ (CPU: synthetic CSVs in the rocprofv3 column layout).

* ``tools.hbm_pmc``: per-kernel bytes per step between Adam dispatches, and
  the last step's dispatches ranked by their gap to the HBM floor.
* ``tools.pmc_table``: SQ counters of several passes merged per dispatch,
  as fractions of the wave cycles.
* ``tools.prof_summary.family``: the kernel-family grouping of the summaries.
"""

import csv
import os

import pytest

from cerebro_ds_kpgi_amd.tools import hbm_pmc, pmc_table
from cerebro_ds_kpgi_amd.tools.prof_summary import family

COLS = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size", "Start_Timestamp",
        "End_Timestamp", "Counter_Name", "Counter_Value"]


def _write(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(COLS, r)))


def _step_rows(ctr, kb):
    """Two training steps: conv (grid 1024, 10 us), bn (grid 256, 4 us),
    adam (grid 64, 20 us) each; ``kb``: KB per kernel for this counter."""
    rows, t, i = [], 1000, 0
    for _ in range(2):
        for name, grid, us in (("void igemm_nt32<64, 64>(NTParams)", 1024, 10),
                               ("void bn_apply_fwd_fold<float>(float const*)", 256, 4),
                               ("void adam_kernel<false>(float*)", 64, 20)):
            rows.append((i, name, grid * 256, 256, t, t + us * 1000, ctr, kb[name.split("<")[0]]))
            t += us * 1000 + 500
            i += 1
    return rows


@pytest.fixture
def hbm_dir(tmp_path):
    read = {"void igemm_nt32": 600.0, "void bn_apply_fwd_fold": 200.0, "void adam_kernel": 900.0}
    wrote = {"void igemm_nt32": 300.0, "void bn_apply_fwd_fold": 200.0, "void adam_kernel": 600.0}
    _write(str(tmp_path / "FETCH_SIZE" / "p_counter_collection.csv"), _step_rows("FETCH_SIZE", read))
    _write(str(tmp_path / "WRITE_SIZE" / "p_counter_collection.csv"), _step_rows("WRITE_SIZE", wrote))
    return str(tmp_path)


def test_hbm_pmc_per_step(hbm_dir):
    out = hbm_pmc.read_pass(hbm_dir, "FETCH_SIZE", 1)
    # one step: the dispatches after the first Adam up to the last one
    assert out["igemm_nt32<64, 64>"][0] == 1 and out["igemm_nt32<64, 64>"][1] == 600.0
    assert out["adam_kernel<false>"][0] == 1
    assert abs(out["bn_apply_fwd_fold<float>"][2] - 4000.0) < 1e-6


def test_hbm_pmc_dispatch_floor(hbm_dir, capsys):
    d = hbm_pmc.read_dispatches(hbm_dir, "FETCH_SIZE")
    assert [k for _, k, _, _, _ in d] == ["igemm_nt32<64, 64>", "bn_apply_fwd_fold<float>",
                                          "adam_kernel<false>"]
    hbm_pmc.dispatch_table(hbm_dir, 10, 6.0)
    text = capsys.readouterr().out
    assert "3 dispatches" in text
    # ranked by time above the floor: adam 20 us - (0.9 + 0.6) MB / 6 TB/s = 19.8 us,
    # conv 10 us - 0.9 MB / 6 TB/s = 9.8 us, bn 4 us - 0.4 MB / 6 TB/s = 3.9 us
    body = [l for l in text.splitlines() if l.startswith("| ") and "dispatch" not in l]
    assert [("adam" in l, "igemm" in l, "bn_apply" in l) for l in body] == [
        (True, False, False), (False, True, False), (False, False, True)], body
    assert body[0].endswith("| 0.2 | 19.8 |") and body[1].endswith("| 0.1 | 9.8 |"), body


def test_pmc_table_merges_passes(tmp_path):
    a = [(7, "void igemm_nn32<64, 64>(NTParams)", 256 * 100, 256, 0, 50000, c, v)
         for c, v in (("SQ_WAVE_CYCLES", 1000.0), ("SQ_WAIT_ANY", 250.0),
                      ("SQ_WAIT_INST_ANY", 400.0), ("SQ_ACTIVE_INST_ANY", 350.0),
                      ("SQ_WAVES", 10.0))]
    b = [(7, "void igemm_nn32<64, 64>(NTParams)", 256 * 100, 256, 0, 50000, c, v)
         for c, v in (("SQ_INSTS_MFMA", 480.0), ("SQ_INSTS_VALU", 1350.0))]
    b.append((8, "void bn_apply_fwd_fold<float>(float const*)", 256, 256, 0, 1000,
              "SQ_INSTS_VALU", 5.0))
    _write(str(tmp_path / "a" / "x" / "p_counter_collection.csv"), a)
    _write(str(tmp_path / "b" / "x" / "p_counter_collection.csv"), b)
    rows = pmc_table.table(pmc_table.load([str(tmp_path / "a"), str(tmp_path / "b")]))
    assert len(rows) == 1                       # conv kernels only
    r = rows[0]
    assert r["grid"] == 100 and r["us"] == 50.0 and r["waves"] == 10
    assert (r["wait"], r["issue-stall"], r["active"]) == (0.25, 0.4, 0.35)
    assert r["mfma/w"] == 48.0 and r["valu/w"] == 135.0


@pytest.mark.parametrize("name,fam", [
    ("void wgrad_batch32<128, 128, false>(WGBatch)", "conv/linear wgrad"),
    ("void igemm_nn32<64, 64, 2, false, 2, 0>(NTParams, int, FastDiv)", "conv dgrad"),
    ("void bn_apply_fwd_fold<float>(float const*, int)", "batchnorm"),
    ("void adam_kernel<false>(float*, long)", "adam"),
])
def test_prof_summary_families(name, fam):
    assert family(name).startswith(fam), (name, family(name))
