"""Flat float32 weight blobs.

Byte-compatible with the reference's MADlib wrapper formats
(``cerebro_gpdb/madlib_keras_wrapper.py:63-160``):

* ``serialize_nd_weights(list of arrays)`` -> float32 bytes of every array
  flattened and concatenated in layer order (the CTQ checkpoint file);
* ``serialize_state_with_nd_weights(image_count, arrays)`` /
  ``serialize_state_with_1d_weights(image_count, flat)`` -> the same blob
  prefixed by ``image_count`` as one float32 (the MA merge state);
* ``deserialize_as_image_1d_weights(state)`` -> (image_count, flat);
* ``deserialize_as_nd_weights(blob, shapes)`` -> list of arrays.

``arena_to_nd_weights`` / ``nd_weights_to_arena`` move one configuration's
row of a packed arena to and from that list in the Keras ``get_weights()``
layout (``master_to_keras`` / ``keras_to_master``): HWIO conv kernels,
(in, out) dense kernels, (kh, kw, c, 1) depthwise kernels, the architecture's
Keras layer order and the conv biases Keras has and we drop (zeros), so
blobs interoperate with ``runtime.checkpoint`` files, with MA merging and
with a Keras model of the same architecture.  The layer order of
``keras.applications`` ResNet-50 is pinned by hand (there is no TF here to
check it against: parity unpinned beyond the element count).
"""

import numpy as np
import torch


def serialize_nd_weights(model_weights):
    if model_weights is None:
        return None
    return np.concatenate([np.asarray(w, np.float32).reshape(-1) for w in model_weights]) \
        .astype(np.float32).tobytes()


def serialize_state_with_nd_weights(image_count, model_weights):
    if model_weights is None:
        return None
    flat = [np.array([image_count], np.float32)] + \
        [np.asarray(w, np.float32).reshape(-1) for w in model_weights]
    return np.concatenate(flat).astype(np.float32).tobytes()


def serialize_state_with_1d_weights(image_count, model_weights):
    if model_weights is None:
        return None
    return np.concatenate([np.array([image_count], np.float32),
                           np.asarray(model_weights, np.float32).reshape(-1)]).tobytes()


def deserialize_as_image_1d_weights(state):
    if not state:
        return None
    arr = np.frombuffer(state, dtype=np.float32)
    return float(arr[0]), arr[1:]


def deserialize_as_nd_weights(blob, model_shapes):
    if not blob or not model_shapes:
        return None
    arr = np.frombuffer(blob, dtype=np.float32)
    total = sum(int(np.prod(s)) for s in model_shapes)
    if total != arr.size:
        raise ValueError("Number of elements in model weights({}) doesn't match model({})."
                         .format(arr.size, total))
    out, i = [], 0
    for s in model_shapes:
        n = int(np.prod(s))
        out.append(np.array(arr[i:i + n]).reshape(s))
        i += n
    return out


def model_shapes(layout):
    """Keras ``get_weights()`` shapes of one configuration (blob order)."""
    return [tuple(e.keras_shape) for e in layout.keras_entries]


def master_to_keras(layout, master):
    """One configuration's master section (flat numpy, our storage order:
    trainable params then BN statistics) -> the list of Keras arrays
    (``get_weights()`` order and shapes; dropped conv biases as zeros)."""
    from .arena import KerasBias
    out = []
    for e in layout.keras_entries:
        if isinstance(e, KerasBias):
            out.append(np.zeros(e.shape, np.float32))
        else:
            out.append(e.to_keras(master[e.offset:e.offset + e.numel]).astype(np.float32))
    return out


def keras_to_master(layout, weights):
    """Inverse of ``master_to_keras``: a flat numpy master section.  A
    non-zero dropped bias is folded into its BatchNorm's moving mean (Keras
    accumulated the biased conv output there; our conv output lacks it)."""
    from .arena import KerasBias
    ents = layout.keras_entries
    if len(weights) != len(ents):
        raise ValueError("expected {} arrays, got {}".format(len(ents), len(weights)))
    out = np.zeros(layout.n_master, np.float32)
    folds = []
    for e, w in zip(ents, weights):
        if isinstance(e, KerasBias):
            w = np.asarray(w, np.float32)
            if tuple(w.shape) != e.shape:
                raise ValueError("{}: shape {} != {}".format(e.name, w.shape, e.shape))
            if np.any(w):
                folds.append((e.fold_into, w))
            continue
        out[e.offset:e.offset + e.numel] = e.from_keras(w)
    for name, b in folds:
        s = layout.by_name[name]
        out[s.offset:s.offset + s.numel] -= b
    return out


def weights_blob(layout, master):
    """``serialize_nd_weights`` blob of one master section (numpy)."""
    return serialize_nd_weights(master_to_keras(layout, master))


def blob_to_master(layout, blob):
    if isinstance(blob, np.ndarray):
        blob = blob.astype("<f4").tobytes()
    return keras_to_master(layout, deserialize_as_nd_weights(blob, model_shapes(layout)))


def arena_to_nd_weights(arena, row):
    """One configuration's weights (trainable + BN statistics) as the list
    of Keras arrays."""
    master = arena.state[row, :arena.layout.n_master].detach().to("cpu").numpy()
    return master_to_keras(arena.layout, master)


def nd_weights_to_arena(arena, row, weights):
    out = torch.from_numpy(keras_to_master(arena.layout, weights))
    arena.state[row, :arena.layout.n_master].copy_(out.to(arena.state.device))
    arena.sync_work(row)
