"""End to end on the GPU: the reference's north-star entry point
(run_da_cerebro_standalone: DA-Cerebro, 8-config ResNet-50 scalability grid)
over Direct-Access partitions written in the Greenplum page format, through
the C++ page/TOAST/pglz reader into the HBM partition store, MOP training on
the HIP kernels, CTQ-layout checkpoints and the reference log files."""

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_da_cerebro_standalone_end_to_end(tmp_path):
    from cerebro_ds_kpgi_amd.data import da
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.runners import run_da_cerebro_standalone
    _hip.lib()                         # the HIP path must be the one that runs
    root = str(tmp_path / "da")
    da.write_dataset(root, "imagenet", 8, n_train=64, n_valid=32, buffer_size=16)
    logs = tmp_path / "run_logs" / "cerebro-da"
    models = tmp_path / "models"
    run_da_cerebro_standalone.main([
        "--run", "--num_epochs", "1", "--drill_down_scalability", "--size", "1", "--da",
        "--da_root", root, "--train_per_partition", "64", "--valid_per_partition", "32",
        "--backend", "hip", "--logs_root", str(logs), "--models_root", str(models)])
    summ = json.loads((logs / "summary.json").read_text())
    assert summ["configs"] == 8 and summ["train_images"] == 8 * 8 * 64
    g = (tmp_path / "run_logs" / "global.log").read_text()
    assert "TOTAL EXECUTION TIME OVER ALL MST" in g
    blobs = sorted(p for p in os.listdir(models) if p.endswith("model:resnet50"))
    assert len(blobs) == 8
    w = np.fromfile(str(models / blobs[0]), dtype=np.float32)
    # Keras get_weights() layout: 25 583 592 trainable (conv biases as zeros) + 53 120 stats
    assert w.size == 25636712 and np.isfinite(w).all()
    jobs = [j for ep in json.loads((logs / "jobs_info.json").read_text()).values()
            for j in ep.values()]
    assert len(jobs) == 64 and all(j["status"] == "SUCCESS" for j in jobs)   # 8 cfg x 8 part.
    assert all(np.isfinite(j["loss_train"]) for j in jobs)


def test_criteo_da_cerebro_standalone_end_to_end(tmp_path):
    """BASELINE config 3 path: the 16-config Criteo confA grid through the
    DA page/pglz reader (one-hot float32 payload -> 39 active ids per row in
    HBM) and MOP on the HIP embedding-bag / linear / loss kernels."""
    from cerebro_ds_kpgi_amd.data import da
    from cerebro_ds_kpgi_amd.ops import _hip
    from cerebro_ds_kpgi_amd.runners import run_da_cerebro_standalone
    _hip.lib()
    root = str(tmp_path / "da")
    da.write_dataset(root, "criteo", 8, n_train=1024, n_valid=512, buffer_size=256)
    logs = tmp_path / "run_logs" / "cerebro-da-criteo"
    run_da_cerebro_standalone.main([
        "--run", "--num_epochs", "1", "--criteo", "--size", "1", "--slots_per_gpu", "8",
        "--da", "--da_root", root, "--train_per_partition", "1024",
        "--valid_per_partition", "512", "--backend", "hip", "--logs_root", str(logs),
        "--models_root", str(tmp_path / "models")])
    summ = json.loads((logs / "summary.json").read_text())
    assert summ["configs"] == 16
    assert summ["train_images"] > 0 and summ["etl_da"]["buffers"] == 8 * (4 + 2)
    assert summ["etl_da"]["decode_GBps"] > 0 and summ["etl_da"]["h2d_GBps"] > 0
    jobs = [j for ep in json.loads((logs / "jobs_info.json").read_text()).values()
            for j in ep.values()]
    assert len(jobs) == 16 * 8 and all(np.isfinite(j["loss_train"]) for j in jobs)
