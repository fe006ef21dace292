"""bench.py contract on CPU: ``--gpus N`` really runs N ranks (gloo here,
RCCL on the GPU node) and reports hop traffic."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_cpu(tmp_path):
    out = _bench("--gpus", "2", "--backend", "torch", "--model", "tinycnn", "--steps", "4",
                 "--warmup", "2", "--steps_per_round", "2", "--train_per_partition", "64",
                 "--logs_root", str(tmp_path))
    assert out["n_gpus"] == 2 and out["world_size"] == 2
    assert out["dist_backend"] == "gloo"
    assert out["hop_bytes"] > 0                  # models hopped between the two ranks
    assert out["metric"].startswith("diag_")     # not the headline model: diagnostic name
    assert out["steps"] == 4 and out["value"] > 0
    # hop telemetry next to the rate: hold time, xGMI bytes (null without amd-smi)
    assert out["hold_ms_max"] >= 0 and "xgmi_write_gb" in out
    recs = [json.loads(l) for l in open(tmp_path / "metrics.jsonl")]
    assert any(r.get("kind") == "hop" for r in recs)
    assert any(r.get("kind") == "hop_hold" for r in recs)
    # the 1 Hz sampler ran beside the ranks
    assert list((tmp_path / "sys_logs").glob("sysmon_*.jsonl"))


def test_bench_one_rank_cpu():
    out = _bench("--backend", "torch", "--model", "tinycnn", "--steps", "2", "--warmup", "1",
                 "--steps_per_round", "2", "--train_per_partition", "64")
    assert out["n_gpus"] == 1 and out["hop_bytes"] == 0


def test_bench_driver_launch_four_ranks_cpu():
    """The driver's N > 1 launch shape (``torch.distributed.run`` starts the
    ranks, bench.py only joins them): 4 ranks, 2 configs each, hops digest-
    checked (CER_HOP_CHECK=1), one JSON line from rank 0."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["CER_HOP_CHECK"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "4", "--backend", "torch", "--model",
           "tinycnn", "--steps", "4", "--warmup", "2", "--steps_per_round", "2",
           "--train_per_partition", "64"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["world_size"] == 4
    assert out["hop_bytes"] > 0 and out["value"] > 0


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port
