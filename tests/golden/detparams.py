"""Deterministic parameters and input states for the large golden updates (test infrastructure).

make_golden.py loads these values into the *reference* modules before running the reference's
update, and the GPU tests regenerate the same values for the modules under test, so a
production-size golden (about 0.9 M parameters) stores no parameter or state arrays, only the
reference's inputs that compress well and its outputs. Every tensor is drawn from numpy's legacy
RandomState (a fixed, version-stable stream) seeded by (seed, crc32 of the state_dict key), so the
values do not depend on the order in which a module registers its parameters.
"""
import zlib

import numpy as np


def _rs(seed, key):
    return np.random.RandomState((seed * 1000003 + zlib.crc32(key.encode())) & 0x7FFFFFFF)


def det_tensor(seed, key, shape):
    """torch-default-like init: U(-1/sqrt(fan), 1/sqrt(fan)) with fan = in-features of a matrix and
    the length of a vector; LayerNorm weights (`ln_*.weight`) 1 + U(-0.1, 0.1), LayerNorm biases
    U(-0.1, 0.1) (away from the identity so that their gradients matter)."""
    rs = _rs(seed, key)
    shape = tuple(int(s) for s in shape)
    if ".ln_" in key or key.startswith("ln_"):
        u = rs.uniform(-0.1, 0.1, size=shape)
        return (1.0 + u if key.endswith("weight") else u).astype(np.float32)
    fan = shape[1] if len(shape) == 2 else shape[0]
    b = 1.0 / np.sqrt(fan)
    return rs.uniform(-b, b, size=shape).astype(np.float32)


def det_state_dict(seed, shapes):
    """{key: float32 array} for {key: shape}."""
    return {k: det_tensor(seed, k, s) for k, s in shapes.items()}


def det_perturb(seed, key, base, scale=0.01):
    """base + scale * N(0, 1) (the target network of a golden update)."""
    return (base + scale * _rs(seed + 7, key).standard_normal(base.shape)).astype(np.float32)


def det_state(seed, shape, scale=0.1):
    """Initial NetMon state of a golden update: scale * N(0, 1)."""
    return (scale * np.random.RandomState(seed).standard_normal(shape)).astype(np.float32)


def sample_index(numel, count, seed):
    """Sorted distinct flat indices at which a large golden array is stored."""
    if numel <= count:
        return np.arange(numel, dtype=np.int64)
    return np.sort(np.random.RandomState(seed).choice(numel, count, replace=False)).astype(np.int64)
