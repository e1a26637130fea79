"""Helpers to load golden fixtures (tests/golden/*.npz + *.json) -- data only, no pickles."""
import json
import os

import numpy as np
import torch

from weights import synth_state, state_checksum

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_case(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        meta = json.load(f)
    data = dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
    return meta, data


def golden_state(meta):
    state = synth_state([(k, tuple(s)) for k, s in meta["params"]])
    assert abs(state_checksum(state) - meta["weight_checksum"]) <= 1e-9 * max(1.0, abs(meta["weight_checksum"]))
    return {k: torch.from_numpy(v) for k, v in state.items()}


def rel_err(a, b):
    a = torch.as_tensor(a).double().flatten()
    b = torch.as_tensor(b).double().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def max_rel(a, b):
    a = torch.as_tensor(a).double().flatten()
    b = torch.as_tensor(b).double().flatten()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
