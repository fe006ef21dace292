"""Serialised weight blobs use the Keras ``get_weights()`` layout
(``serialize_nd_weights``, reference ``madlib_keras_wrapper.py:119-131``):
HWIO conv kernels, (in, out) dense kernels, (kh, kw, c, 1) depthwise
kernels, the conv biases Keras has and we drop, and Keras's layer order.
A hand-built Keras-layout blob loads element-wise into our storage."""

import numpy as np
import torch

from cerebro_ds_kpgi_amd.models import create_model_from_mst
from cerebro_ds_kpgi_amd.runtime import Arena
from cerebro_ds_kpgi_amd.runtime import serialize as S
from cerebro_ds_kpgi_amd.runtime.arena import KerasBias


def _names(layout):
    return [e.name for e in layout.keras_entries]


def test_resnet50_blob_matches_keras_counts_and_order():
    net = create_model_from_mst({"model": "resnet50"})
    L = net.layout
    shapes = S.model_shapes(L)
    # Keras ResNet50: 25 583 592 trainable + 53 120 moving statistics
    assert sum(int(np.prod(s)) for s in shapes) == 25636712
    assert shapes[0] == (7, 7, 3, 64) and shapes[1] == (64,)
    assert shapes[-2:] == [(2048, 1000), (1000,)]
    n = _names(L)
    i = n.index("res2a_branch2c/kernel")
    assert n[i:i + 6] == ["res2a_branch2c/kernel", "res2a_branch2c/bias",
                          "res2a_branch1/kernel", "res2a_branch1/bias",
                          "bn2a_branch2c/gamma", "bn2a_branch2c/beta"]
    assert n[i + 8:i + 10] == ["bn2a_branch1/gamma", "bn2a_branch1/beta"]
    j = n.index("res2b_branch2c/kernel")
    assert n[j:j + 3] == ["res2b_branch2c/kernel", "res2b_branch2c/bias", "bn2b_branch2c/gamma"]


def test_hand_built_keras_blob_loads_elementwise():
    net = create_model_from_mst({"model": "resnet50"})
    L = net.layout
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal(s).astype(np.float32) for s in S.model_shapes(L)]
    blob = S.serialize_nd_weights(arrays)
    arena = Arena(L, 1, "cpu", torch.float32, trainable=False)
    arena.load_row_weights_f32(0, np.frombuffer(blob, np.float32))
    ents = L.keras_entries
    byname = {e.name: a for e, a in zip(ents, arrays)}
    # conv: ours (cout, kh, kw, cin) vs Keras HWIO
    w = arena.master_view(L.by_name["res3a_branch2b/kernel"])[0]
    k = byname["res3a_branch2b/kernel"]
    for co, kh, kw, ci in [(0, 0, 0, 0), (5, 2, 1, 7), (127, 1, 2, 100)]:
        assert w[co, kh, kw, ci].item() == k[kh, kw, ci, co]
    # dense: ours (cout, cin) vs Keras (cin, cout)
    d = arena.master_view(L.by_name["fc1000/kernel"])[0]
    kd = byname["fc1000/kernel"]
    assert d[3, 2047].item() == kd[2047, 3] and d[999, 0].item() == kd[0, 999]
    # the dropped bias folds into the BN moving mean
    rm = arena.master_view(L.by_name["bn3a_branch2b/moving_mean"])[0].numpy()
    np.testing.assert_allclose(rm, byname["bn3a_branch2b/moving_mean"] -
                               byname["res3a_branch2b/bias"], rtol=0, atol=1e-6)
    # and the unchanged tensors round-trip exactly
    back = S.arena_to_nd_weights(arena, 0)
    for e, a, b in zip(ents, arrays, back):
        if isinstance(e, KerasBias):
            assert not b.any()
        elif "moving_mean" not in e.name:
            np.testing.assert_array_equal(a, b)


def test_blob_round_trip_every_family():
    for arch in ("resnet50", "vgg16", "mobilenetv2", "nasnetmobile", "confA", "resnet50_nobn"):
        net = create_model_from_mst({"model": arch})
        L = net.layout
        arena = Arena(L, 1, "cpu", torch.float32, trainable=False)
        arena.init_model(0, 7)
        blob = arena.row_weights_f32(0)
        assert blob.size == sum(int(np.prod(s)) for s in S.model_shapes(L))
        other = Arena(L, 1, "cpu", torch.float32, trainable=False)
        other.load_row_weights_f32(0, blob)
        torch.testing.assert_close(other.master, arena.master, rtol=0, atol=0)


def test_depthwise_keras_shape():
    net = create_model_from_mst({"model": "mobilenetv2"})
    dw = [e for e in net.layout.keras_entries if e.name.endswith("depthwise_kernel")]
    assert dw and all(len(e.keras_shape) == 4 and e.keras_shape[-1] == 1 for e in dw)
