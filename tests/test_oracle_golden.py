"""The CPU oracle (oracle/torch_ref.py) against the reference's own golden vectors.

Tolerances: the oracle evaluates the same fp32 arithmetic as the reference, through different but
equivalent torch calls (functional ops, matmul instead of bmm), so agreement is ~1e-6 relative;
we require <= 1e-5 (norm-wise relative) for tensors and 1e-6 relative for scalar loss terms.
"""
import json
import os

import numpy as np
import pytest
import torch

from cases import CASES, FULL_GRADS
from golden_io import GOLDEN, golden_state, load_case, rel_err
from oracle import torch_ref as R


def _cond(case, data):
    if case["cond"] == "onehot":
        return torch.from_numpy(data["in.cond"])
    if case["cond"] == "idx":
        return torch.from_numpy(data["in.cond"]).long()
    return None


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference(name):
    meta, data = load_case(name)
    case = CASES[name]
    a = R.make_arch(case["cls"], case["kwargs"])
    assert [[k, list(s)] for k, s in R.param_shapes(a)] == meta["params"] or \
        sorted(map(tuple, [(k, tuple(s)) for k, s in R.param_shapes(a)])) == \
        sorted((k, tuple(s)) for k, s in meta["params"])
    P = golden_state(meta)
    x = torch.from_numpy(data["in.x"])
    eps = torch.from_numpy(data["in.eps"])
    res = R.train_step(P, a, x, _cond(case, data), eps, case["loss"], case["optimizer"], case["clip"])
    out = res["out"]
    for k in ("reconstruction", "mean", "logvar", "z"):
        assert rel_err(out[k].detach(), data[f"out.{k}"]) < 1e-5, k
    for k, v in res["loss"].items():
        ref = float(data[f"loss.{k}"])
        assert abs(float(v) - ref) <= 1e-6 * max(1.0, abs(ref)) + 1e-9, (k, float(v), ref)
    assert abs(float(res["total_norm"]) - float(data["clip.total_norm"])) < 1e-5 * float(data["clip.total_norm"])
    # every parameter that received a gradient in the reference receives one here, and only those
    has = {k for k, v in meta["param_has_grad"].items() if v}
    assert set(res["grads"]) == has
    for k in has:
        s = data[f"gradsum.{k}"]
        g = res["grads"][k].double()
        assert abs(float((g * g).sum()) - s[1]) <= 1e-4 * s[1] + 1e-12, k
    for k in FULL_GRADS[name]:
        assert rel_err(res["grads"][k], data[f"grad.{k}"]) < 1e-5, k
        assert rel_err(res["params"][k], data[f"step.{k}"]) < 1e-6, k
    for k in P:
        s = data[f"stepsum.{k}"]
        v = res["params"][k].double()
        assert abs(float((v * v).sum()) - s[1]) <= 1e-6 * s[1] + 1e-12, k


def test_known_answer_anchor_shapes():
    """SURVEY 8(c) anchor values were reproduced by the generator on the reference itself."""
    with open(os.path.join(GOLDEN, "kat_anchor.json")) as f:
        kat = json.load(f)
    assert abs(kat["recon_loss"] - 0.45200789) < 1e-7
    assert abs(kat["kl_loss"] - 0.09072405) < 1e-7
