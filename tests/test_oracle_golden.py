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


def _disc_inputs():
    meta, data = load_case("disc")
    W = golden_state(meta)
    return meta, data, W


def test_oracle_discriminator_matches_reference():
    """oracle.discriminator (restating src/models/discriminator.py) against the reference's own
    NLayerDiscriminator run by make_golden.py (train-mode BatchNorm, three forwards, hinge loss, adaptive weight)."""
    import torch.nn.functional as F
    meta, data, W = _disc_inputs()
    from weights import synth_param
    running = {}
    for k, s in meta["params"]:
        if k.endswith(".weight") and len(s) == 1:  # BatchNorm affine weight -> its running buffers
            base = k[: -len(".weight")]
            running[f"{base}.running_mean"] = torch.zeros(s[0])
            running[f"{base}.running_var"] = torch.ones(s[0])
    Wr = {k: v.clone().requires_grad_() for k, v in W.items()}
    x = torch.from_numpy(data["in.x"])
    feat = torch.from_numpy(data["in.feat"])
    w_last = torch.from_numpy(synth_param("last.weight", (3, 8, 3, 3))).requires_grad_()
    b_last = torch.from_numpy(synth_param("last.bias", (3,)))
    rec = F.conv2d(feat, w_last, b_last, padding=1)
    nll = F.mse_loss(rec, x)
    lg = R.discriminator(Wr, rec, running=running)
    g_loss = -lg.mean()
    ng = torch.autograd.grad(nll, w_last, retain_graph=True)[0]
    gg = torch.autograd.grad(g_loss, w_last, retain_graph=True)[0]
    dw = torch.clamp(ng.norm() / (gg.norm() + 1e-4), 0.0, 1e4)
    for v in Wr.values():
        v.grad = None
    lr_ = R.discriminator(Wr, x, running=running)
    lf = R.discriminator(Wr, rec.detach(), running=running)
    d_loss = R.hinge_d_loss(lr_, lf)
    d_loss.backward()
    assert rel_err(lg.detach(), data["out.logits_g"]) < 1e-5
    assert rel_err(lr_.detach(), data["out.logits_real"]) < 1e-5
    assert rel_err(lf.detach(), data["out.logits_fake"]) < 1e-5
    for k, tol in (("g_loss", 1e-5), ("d_weight", 1e-5), ("d_loss", 1e-6)):
        ref = float(data[f"loss.{k}"])
        got = {"g_loss": g_loss, "d_weight": dw, "d_loss": d_loss}[k]
        assert abs(float(got) - ref) <= tol * max(1.0, abs(ref)), (k, float(got), ref)
    for k in meta["full_grads"]:
        assert rel_err(Wr[k].grad, data[f"grad.{k}"]) < 1e-5, k
    for k in W:
        s = data[f"gradsum.{k}"]
        g = Wr[k].grad.double()
        assert abs(float((g * g).sum()) - s[1]) <= 1e-4 * s[1] + 1e-12, k
    for k, v in running.items():
        assert rel_err(v, data[f"buf.{k}"]) < 1e-5, k
