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
row of a packed arena to and from that list, in the layout's spec order
(which is the Keras ``get_weights()`` order of the architecture), so blobs
interoperate with ``runtime.checkpoint`` files and with MA merging.
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
    return [tuple(s.shape) for s in layout.specs]


def arena_to_nd_weights(arena, row):
    """One configuration's weights (trainable + BN statistics) as a list of
    arrays in spec order."""
    master = arena.state[row].detach().to("cpu")
    return [master[s.offset:s.offset + s.numel].numpy().reshape(s.shape).copy()
            for s in arena.layout.specs]


def nd_weights_to_arena(arena, row, weights):
    specs = arena.layout.specs
    if len(weights) != len(specs):
        raise ValueError("expected {} arrays, got {}".format(len(specs), len(weights)))
    out = torch.zeros(arena.layout.n_master, dtype=torch.float32)
    for s, w in zip(specs, weights):
        w = np.asarray(w, np.float32)
        if tuple(w.shape) != tuple(s.shape):
            raise ValueError("{}: shape {} != {}".format(s.name, w.shape, s.shape))
        out[s.offset:s.offset + s.numel] = torch.from_numpy(w.reshape(-1))
    arena.state[row, :arena.layout.n_master].copy_(out.to(arena.state.device))
    arena.sync_work(row)
