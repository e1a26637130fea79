"""Deterministic synthetic parameter values shared by the golden-vector generator and the tests.

Golden fixtures do not store model weights (they would be megabytes of random floats). Instead
every parameter is regenerated from its state-dict *name* and shape with numpy's PCG64 uniform
doubles (`Generator.random`, whose bit stream numpy keeps stable), so the generator (which loads
these values into the reference models) and the tests (which load them into the oracle and into
the HIP path) see bit-identical float32 weights. A per-fixture checksum guards against drift.
"""
from __future__ import annotations

import zlib

import numpy as np


def synth_param(name: str, shape, seed: int = 1234) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    rng = np.random.Generator(np.random.PCG64(seed * 1_000_003 + zlib.crc32(name.encode())))
    u = rng.random(n) * 2.0 - 1.0  # U[-1, 1) float64
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "weight" and len(shape) >= 2:
        if "embedding" in name:
            vals = u
        else:
            fan_in = int(np.prod(shape[1:]))
            vals = u / np.sqrt(fan_in)
    elif leaf == "weight":  # GroupNorm gamma
        vals = 1.0 + 0.2 * u
    elif leaf == "bias":
        vals = 0.05 * u
    else:
        vals = u
    return vals.astype(np.float32).reshape(shape)


def synth_state(named_shapes, seed: int = 1234) -> dict:
    return {k: synth_param(k, s, seed) for k, s in named_shapes}


def state_checksum(state: dict) -> float:
    tot = 0.0
    for k in sorted(state):
        a = np.asarray(state[k], dtype=np.float64)
        tot += float(np.sum(a * a)) + float(np.sum(a))
    return tot
