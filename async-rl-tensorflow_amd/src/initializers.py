"""Parameter initialisers of the reference (host side, numpy).

* conv weights: ``tf.truncated_normal_initializer(0, 0.02)`` (agent.py:214, network.py:10,
  passed to ops.conv2d ops.py:21) -- re-draw outside 2 sigma;
* linear ``Matrix``: ``tf.random_normal_initializer(stddev=0.02)`` (ops.py:36-37);
* biases: ``tf.constant_initializer(0.0)`` / ``bias_start`` (ops.py:24,38-39).
TF's own op RNG is not reproducible outside TF, so draws come from numpy's PCG64 seeded by
``random_seed`` (main.py:35).
"""
import numpy as np


def truncated_normal(rng, shape, mean=0.0, stddev=0.02):
    v = rng.standard_normal(shape)
    bad = np.abs(v) > 2.0
    while bad.any():
        v[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(v) > 2.0
    return (mean + v * stddev).astype(np.float32)


def random_normal(rng, shape, stddev=0.02):
    return (rng.standard_normal(shape) * stddev).astype(np.float32)


def init_params(names_shapes, seed=123, stddev=0.02, bias_start=0.0):
    """dict name -> float32 array, in the flat order of ``names_shapes``."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shp in names_shapes:
        if name.endswith('_b'):
            out[name] = np.full(shp, bias_start, np.float32)
        elif len(shp) == 4:
            out[name] = truncated_normal(rng, shp, 0.0, stddev)
        else:
            out[name] = random_normal(rng, shp, stddev)
    return out


def flatten_host(names_shapes, offsets, total, params):
    flat = np.zeros(total, np.float32)
    for (name, shp), off in zip(names_shapes, offsets):
        v = np.asarray(params[name], np.float32).reshape(-1)
        flat[off:off + v.size] = v
    return flat
