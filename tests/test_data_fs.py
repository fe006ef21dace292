"""Filesystem partitions, Criteo / ImageNet preprocessing."""

import json
import os

import numpy as np
import pytest
import torch

os.environ.setdefault("CEREBRO_BACKEND", "torch")


def test_murmur3_matches_mmh3_reference_values():
    from cerebro_ds_kpgi_amd.data import criteo
    # mmh3.hash(...) values (signed MurmurHash3_x86_32, seed 0)
    assert criteo.murmur3_32("foo") == -156908512
    assert criteo.murmur3_32("hello") == 613153351
    assert criteo.murmur3_32("") == 0


def test_criteo_bucket_boundaries():
    from cerebro_ds_kpgi_amd.data import criteo
    bounds = [1.5 ** j - 0.51 for j in range(50)]

    def ref(v):                      # preprocessing_criteo._get_index_bucket
        for i, b in enumerate(bounds):
            if v < b:
                return i
        return i
    for v in [-7, 0, 1, 2, 3, 17, 1000, 10 ** 7, 10 ** 10]:
        assert criteo.bucket(v) == ref(v), v


def test_criteo_featurize_row():
    from cerebro_ds_kpgi_amd.data import criteo
    cont = ["5", "", "3", "0"] + [""] * 8 + ["2"]
    cats = ["foo", "hello"] + [""] * 24
    line = "\t".join(["1"] + cont + cats).encode() + b"\n" + b"0\tshort\n"
    ids, labels = criteo.featurize_lines(line)
    assert labels.tolist() == [1, 0]
    want = sorted([0 * 50 + criteo.bucket(5), 2 * 50 + criteo.bucket(3), 12 * 50 + criteo.bucket(2),
                   650 + 0 * 256 + (-156908512 % 256), 650 + 1 * 256 + (613153351 % 256)])
    got = sorted(int(v) for v in ids[0] if v >= 0)
    assert got == want
    assert (ids[1] == -1).all()
    dense = criteo.ids_to_dense(ids, labels)
    assert dense.shape == (2, 7307) and dense[0, :-1].sum() == 5 and dense[0, -1] == 1


def _tsv(path, n, seed=0):
    rs = np.random.RandomState(seed)
    with open(path, "w") as f:
        for _ in range(n):
            cont = [str(rs.randint(0, 500)) if rs.rand() > 0.2 else "" for _ in range(13)]
            cats = ["{:08x}".format(rs.randint(0, 2 ** 31)) if rs.rand() > 0.1 else ""
                    for _ in range(26)]
            f.write("\t".join([str(rs.randint(0, 2))] + cont + cats) + "\n")


def test_preprocess_criteo_and_fs_training(tmp_path):
    from cerebro_ds_kpgi_amd.tools import preprocess_criteo
    from cerebro_ds_kpgi_amd.data import fs
    src = tmp_path / "day_1"
    _tsv(str(src), 400)
    out = str(tmp_path / "criteo")
    stats = preprocess_criteo.main(["--inputs", str(src), "--out", out, "--partitions", "2"])
    assert stats["train"] + stats["valid"] == 400 and 0 < stats["valid"] < 100
    loader = fs.fs_partition_loader(out, "criteo", "cpu")
    tx, ty, vx, vy = loader(0)
    assert tx.shape[1] == 39 and tx.dtype == torch.int32 and int(tx.max()) < 7306
    assert ((tx >= 0).sum(1) <= 39).all() and set(ty.unique().tolist()) <= {0, 1}
    # dense reference layout round trip
    dense_out = str(tmp_path / "criteo_dense")
    preprocess_criteo.main(["--inputs", str(src), "--out", dense_out, "--partitions", "2",
                            "--dense"])
    ref = fs.input_fn_criteo(os.path.join(dense_out, "train", "train_0.npy"))
    assert ref["images"].shape[1] == 7306 and ref["labels"].shape[1] == 2
    tx2, _, _, _ = fs.fs_partition_loader(dense_out, "criteo", "cpu")(0)
    assert torch.equal(torch.sort(tx2, 1)[0], torch.sort(tx, 1)[0])


def test_fs_imagenet_input_fn_and_loader(tmp_path):
    from cerebro_ds_kpgi_amd.data import fs
    root = str(tmp_path / "imagenet")
    cat = fs.write_fs_dataset(root, "imagenet", 2, 40, 8)
    assert cat["train"][1] == "train/train_1.h5" and cat["train_availability"][1] == [0, 1]
    parts = fs.input_fn(os.path.join(root, cat["train"][0]))
    n = sum(p["images"].shape[0] for p in parts)
    assert n == 40 and parts[0]["images"].shape[1:] == (112, 112, 3)
    assert parts[0]["labels"].shape[1] == 1000 and parts[0]["labels"].sum(1).max() == 1
    tx, ty, vx, vy = fs.fs_partition_loader(root, "imagenet", "cpu")(1)
    assert tx.dtype == torch.uint8 and tuple(tx.shape) == (40, 112, 112, 3) and vx.shape[0] == 8


def test_run_filesystem_cerebro_criteo(tmp_path):
    from cerebro_ds_kpgi_amd.data import fs
    from cerebro_ds_kpgi_amd.runners import run_filesystem_cerebro_standalone as r
    root = str(tmp_path / "criteo")
    fs.write_fs_dataset(root, "criteo", 2, 64, 16)
    logs = tmp_path / "run_logs" / "fs"
    r.main(["--run", "--criteo", "--num_epochs", "1", "--fs_root", root, "--size", "2",
            "--slots_per_gpu", "2", "--compute_dtype", "fp32", "--backend", "torch",
            "--logs_root", str(logs), "--models_root", str(tmp_path / "models")])
    summ = json.loads((logs / "summary.json").read_text())
    assert summ["train_images"] > 0
    assert all(len(s["train_loss"]) == 1 for s in summ["mst_state"].values())


def test_preprocess_imagenet_folders(tmp_path):
    from PIL import Image
    from cerebro_ds_kpgi_amd.tools import preprocess_imagenet
    rs = np.random.RandomState(0)
    for split, n in (("train", 3), ("valid", 2)):
        for syn in ("n01440764", "n01443537"):
            d = tmp_path / split / syn
            d.mkdir(parents=True)
            for i in range(n):
                Image.fromarray(rs.randint(0, 255, (60, 80, 3), dtype=np.uint8)).save(
                    str(d / "{}_{}.JPEG".format(syn, i)))
    out = str(tmp_path / "out")
    res = preprocess_imagenet.main(["--train_dir", str(tmp_path / "train"), "--valid_dir",
                                    str(tmp_path / "valid"), "--out", out, "--partitions", "2",
                                    "--workers", "2"])
    assert res["classes"] == 2 and sum(res["train"]) == 6 and sum(res["valid"]) == 4
    x = np.load(os.path.join(out, "train", "train_0.images.npy"))
    assert x.shape[1:] == (112, 112, 3) and x.dtype == np.uint8
