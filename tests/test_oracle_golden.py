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


@pytest.mark.parametrize("tag,dt", [("f32", torch.float32), ("f64", torch.float64)])
def test_oracle_latent_losses_b512(tag, dt):
    """The oracle's separation / contrastive terms against the reference's own methods at the c3 bench batch
    (tests/golden/latent_b512.npz, make_golden.latent_case): B = 512, ids 0..4 plus out-of-range 7 / 9 / 17."""
    data = dict(np.load(os.path.join(GOLDEN, "latent_b512.npz"), allow_pickle=False))
    a = R.make_arch("DisentangledConditionalVAE", dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8,
                                                       hidden_channels=32, ch_mult=[1, 2, 4], num_res_blocks=1,
                                                       attn_resolutions=[], dropout=0.0, resolution=28))
    idx = torch.from_numpy(data["in.idx"])
    tol = 1e-6 if tag == "f32" else 1e-12
    for term, fn in (("sep", R.separation_loss), ("con", R.contrastive_loss)):
        z = torch.from_numpy(data["in.z"]).to(dt).requires_grad_()
        v = fn(a, z, idx)
        v.backward()
        ref = float(data[f"{term}.{tag}"])
        assert abs(float(v) - ref) <= tol * abs(ref), (term, float(v), ref)
        g = z.grad.reshape(z.shape[0], -1)
        assert rel_err(g[:, :16], data[f"grad_{term}.{tag}"]) < (1e-5 if tag == "f32" else 1e-12), term
        assert float(g[:, 16:].abs().max()) == float(data[f"grad_{term}_rest_max.{tag}"]) == 0.0
