"""Deterministic RandLA-Net parameters keyed by state_dict name (shared by the
golden generator and the tests, so no weights need to be stored)."""
import zlib

import numpy as np


def fill(name, shape):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    if name.endswith("num_batches_tracked"):
        return np.zeros(shape, np.int64)
    if name.endswith("running_var"):
        return (1.0 + 0.5 * rng.random(shape)).astype(np.float32)
    if name.endswith("running_mean"):
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if "batch_norm" in name or name.startswith("bn0") or name.endswith(".bn.weight") or name.endswith(".bn.bias"):
        base = 1.0 if name.endswith("weight") else 0.0
        return (base + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    if name.endswith("bias"):
        return (0.05 * rng.standard_normal(shape)).astype(np.float32)
    if name.endswith("offset"):  # SparseConv offsets are structural, never filled
        return None
    fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    if ".conv." in name and "decoder" in name:  # ConvTranspose2d: weight [in, out, 1, 1]
        fan_in = shape[0]
    if name.endswith("kernel"):  # SparseConv kernel [k, k, k, Cin, Cout]
        fan_in = int(np.prod(shape[:-1]))
    return (rng.standard_normal(shape) / np.sqrt(max(fan_in, 1))).astype(np.float32)


def state_dict_for(keys_shapes, base=None):
    """Deterministic values for every entry; entries fill() leaves alone (None)
    keep their value from `base` (a state_dict)."""
    import torch
    out = {}
    for k, s in keys_shapes:
        v = fill(k, tuple(s))
        out[k] = base[k].clone() if v is None else torch.from_numpy(v)
    return out
