"""End-to-end parity of the MI355X training step against the REFERENCE's golden vectors.

For every golden case (tests/golden, produced from the reference's own src.models by
make_golden.py) the HIP path runs one full Lightning-style optimisation step -- forward, loss,
backward, non-finite zeroing, global-norm clip, Adam/AdamW -- on the same weights / batch / eps,
and is compared with the reference's outputs, loss terms, gradients and updated parameters.

Tolerance (BASELINE.json north star): 1e-3 relative (fp32 budget); tensors are compared norm-wise,
gradients of every parameter through their sum of squares, selected gradients/parameters in full.
The index routing of the disentangled model is exact (selection, no arithmetic).
"""
import json
import math
import os

import pytest
import torch

from cases import CASES, FULL_GRADS
from golden_io import golden_state, load_case, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _batch(case, data, dev):
    x = torch.from_numpy(data["in.x"]).to(dev)
    B = x.shape[0]
    labels = torch.zeros(B, 1, dtype=torch.long, device=dev)
    if case["cond"] == "onehot":
        return (x, labels, torch.from_numpy(data["in.cond"]).to(dev))
    if case["cond"] == "idx":
        idx = torch.from_numpy(data["in.cond"]).long().to(dev)
        oh = torch.zeros(B, 12, device=dev)
        oh[torch.arange(B, device=dev), idx.clamp_max(11)] = 1.0
        return (x, labels, oh, idx)
    return (x, labels)


@pytest.mark.parametrize("name", sorted(CASES))
def test_training_step_matches_reference(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check_step(name)


@pytest.mark.parametrize("name", ["cvae_c4_full", "beta_c2_full"])
def test_training_step_winograd_matches_reference(name, monkeypatch):
    """The same step with the Winograd F(4x4, 3x3) convs the bench runs at B = 256 forced on at the golden B = 2 (the
    size rule would keep the implicit GEMM there): c4's 8x8 / 16x16 / 32x32 levels, c2's 7x7 level."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from medvae_disentangled_multimodal_amd import _lib, ops
    monkeypatch.setattr(ops, "WINOGRAD_MIN_MACS", 0.0)
    seen = set()
    orig = _lib.call

    def spy(fn, *args):
        seen.add(fn)
        return orig(fn, *args)
    monkeypatch.setattr(_lib, "call", spy)
    _check_step(name)
    assert {"mvae_winograd_gemm", "mvae_winograd_wgrad_gemm"} <= seen


def _check_step(name):
    import medvae_disentangled_multimodal_amd as M
    dev = torch.device("cuda:0")
    meta, data = load_case(name)
    case = CASES[name]
    model = getattr(M, case["cls"])(**case["kwargs"])
    model.load_state_dict(golden_state(meta))
    model = model.to(dev)
    mod = M.VAELightningModule(model, case["optimizer"], {"type": "none"}, case["loss"],
                               gradient_clip_val=case["clip"])
    mod.configure_optimizers()
    batch = _batch(case, data, dev)
    eps = torch.from_numpy(data["in.eps"]).to(dev)

    mod.optimizer.zero_grad()
    loss = mod.training_step(batch, 0, eps=eps)
    out = mod._last_outputs
    for k in ("reconstruction", "mean", "logvar", "z"):
        assert rel_err(out[k].detach().cpu(), data[f"out.{k}"]) < TOL, k
    report = {k: rel_err(out[k].detach().cpu(), data[f"out.{k}"]) for k in ("reconstruction", "mean", "logvar", "z")}
    terms = [k for k in ("recon_loss", "kl_loss", "separation_loss", "contrastive_loss") if f"loss.{k}" in data]
    w = {"recon_loss": case["loss"].get("recon_weight", 1.0), "kl_loss": case["loss"].get("kl_weight", 1.0),
         "separation_loss": case["loss"].get("separation_weight", 0.1),
         "contrastive_loss": case["loss"].get("contrastive_weight", 0.05)}
    scale_total = sum(abs(w[k] * float(data[f"loss.{k}"])) for k in terms)
    for k in terms + ["loss"]:
        ref = float(data[f"loss.{k}"])
        got = float(mod.logged[f"train/{k}"])
        denom = scale_total if k == "loss" else abs(ref)
        report[f"loss.{k}"] = abs(got - ref) / max(denom, 1e-12)
        assert abs(got - ref) <= TOL * max(denom, 1e-6), (k, got, ref)
    loss.backward()
    torch.cuda.synchronize()
    names = mod.flat.names
    has = {k for k, v in meta["param_has_grad"].items() if v}
    for k in has:
        g = mod.flat.params[names.index(k)]._mvae_main_grad.double().cpu()
        ss = float((g * g).sum())
        ref = float(data[f"gradsum.{k}"][1])
        assert abs(ss - ref) <= 2 * TOL * ref + 1e-12, (k, ss, ref)
    for k in FULL_GRADS[name]:
        g = mod.flat.params[names.index(k)]._mvae_main_grad.cpu()
        assert rel_err(g, data[f"grad.{k}"]) < TOL, k
    p_before = mod.flat.data.detach().clone().cpu()
    g_before = mod.flat.grad.detach().clone().cpu()
    used = mod._used_mask()
    mod.optimizer.step(used=used)
    torch.cuda.synchronize()
    tn = float(mod.optimizer.last_total_norm)
    # The global norm of the reference's own gradients, summed in float64 from the fixture's per-tensor sums of
    # squares. torch's CPU fp32 clip_grad_norm_ (the fixture's clip.total_norm) accumulates in fp32 and drifts
    # from it by 1.1e-3 at the 927 M-parameter c4 architecture (9.7718 vs 9.7828; float64 oracle: 9.78283),
    # so the exact norm is the target and the fp32 value is held to 2x the budget.
    exact = math.sqrt(sum(float(data[f"gradsum.{k}"][1]) for k in has))
    report["clip.total_norm_vs_exact"] = abs(tn - exact) / exact
    assert abs(tn - exact) < TOL * exact
    assert abs(tn - float(data["clip.total_norm"])) < 2 * TOL * float(data["clip.total_norm"])
    # (a) the fused step equals torch.optim applied to OUR gradients (per-tensor non-finite zeroing,
    #     global clip, Adam/AdamW, params without a gradient skipped)
    used_l = used.tolist() if used is not None else [1] * len(names)
    ref_params, ref_grads = [], []
    for i, (k, p) in enumerate(zip(names, mod.flat.params)):
        if not used_l[i]:
            continue
        off, n = mod.flat.offsets[i], p.numel()
        ref_params.append(p_before[off:off + n].clone().requires_grad_())
        ref_grads.append(g_before[off:off + n].clone())
    for rp, rg in zip(ref_params, ref_grads):
        rp.grad = rg if torch.isfinite(rg).all() else torch.zeros_like(rg)
    # clip_grad_norm_'s arithmetic with the norm summed in float64 (torch's CPU fp32 norm drifts by 1e-3 at the
    # 927 M-parameter c4 architecture -- see the total-norm check above)
    tn64 = math.sqrt(sum(float((rp.grad.double() ** 2).sum()) for rp in ref_params))
    coef = min(1.0, case["clip"] / (tn64 + 1e-6))
    for rp in ref_params:
        rp.grad.mul_(coef)
    oc = case["optimizer"]
    O = torch.optim.AdamW if oc["type"] == "adamw" else torch.optim.Adam
    O(ref_params, lr=oc["lr"], betas=tuple(oc["betas"]), weight_decay=oc["weight_decay"]).step()
    after = mod.flat.data.detach().cpu()
    j = 0
    worst = 0.0
    for i, (k, p) in enumerate(zip(names, mod.flat.params)):
        off, n = mod.flat.offsets[i], p.numel()
        if not used_l[i]:
            assert torch.equal(after[off:off + n], p_before[off:off + n]), f"unused {k} changed"
            continue
        d = float((after[off:off + n] - ref_params[j].detach()).abs().max())
        worst = max(worst, d)
        assert d <= 1e-6 * float(ref_params[j].detach().abs().max()) + 1e-9, k
        j += 1
    report["step.vs_torch_optim_maxabs"] = worst
    # (b) against the reference's own post-step values: Adam's first step moves each element by
    #     ~lr*sign(g), so an element whose reference gradient is rounding noise (e.g. a conv bias in
    #     front of a 1-channel-per-group GroupNorm: exact gradient 0) may step the other way on ANY
    #     platform. Bound: |dp| <= 2*lr everywhere and < 0.01*lr for >= 98% of the elements.
    lr = oc["lr"]
    for k in FULL_GRADS[name]:
        p = mod.flat.params[names.index(k)].detach().cpu()
        d = (p - torch.from_numpy(data[f"step.{k}"])).abs()
        assert float(d.max()) <= 2.0 * lr * 1.001 + 1e-7, k
        assert float((d > 0.01 * lr).float().mean()) < 0.02, k
    out_dir = os.environ.get("MVAE_PARITY_REPORT")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"parity_{name}.json"), "w") as f:
            json.dump(report, f, indent=1, sort_keys=True)


def test_state_dict_roundtrip_and_names():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import medvae_disentangled_multimodal_amd as M
    meta, _ = load_case("cvae_c4")
    case = CASES["cvae_c4"]
    m = getattr(M, case["cls"])(**case["kwargs"]).cuda()
    m.load_state_dict(golden_state(meta))
    mod = M.VAELightningModule(m, case["optimizer"], {}, case["loss"], gradient_clip_val=1.0)
    mod.configure_optimizers()  # params re-homed into the flat buffer (channels_last conv weights)
    sd = {k: v.cpu() for k, v in m.state_dict().items()}
    ref = golden_state(meta)
    assert list(sd) == [k for k, _ in meta["params"]]
    for k in sd:
        assert torch.equal(sd[k], ref[k]), k


@pytest.mark.parametrize("wino", [False, True], ids=["direct", "winograd"])
@pytest.mark.parametrize("name", ["cvae_c4_full", "beta_c2_full", "dis_c3_b16", "base_c1_full"])
def test_training_step_exact_fp32_matches_reference(name, wino, monkeypatch):
    """The trainer's "32-exact" precision (every conv / bmm on the f32-input MFMA, no operand rounding -- the
    arithmetic of the bench's c4x line) against the reference at the exact BASELINE architectures: outputs, loss
    terms, the global gradient norm and the selected full gradients, 1e-4 relative (only the summation order
    differs from the reference's CPU fp32). winograd: the F(4x4, 3x3) convs the c4x bench runs at B = 256 forced on at
    the golden B = 2 (fp32 transforms, bit-split GEMM operands: ~5e-7 per conv)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import _lib, ops
    seen = set()
    if wino:
        if name not in ("cvae_c4_full", "beta_c2_full", "base_c1_full"):
            pytest.skip("no Winograd-eligible conv (the channel floor) in this architecture")
        monkeypatch.setattr(ops, "WINOGRAD_MIN_MACS", 0.0)
        orig = _lib.call

        def spy(fn, *args):
            seen.add(fn)
            return orig(fn, *args)
        monkeypatch.setattr(_lib, "call", spy)
    dev = torch.device("cuda:0")
    meta, data = load_case(name)
    case = CASES[name]
    model = getattr(M, case["cls"])(**case["kwargs"])
    model.load_state_dict(golden_state(meta))
    model = model.to(dev)
    mod = M.VAELightningModule(model, case["optimizer"], {"type": "none"}, case["loss"],
                               gradient_clip_val=case["clip"], precision="32-exact")
    mod.configure_optimizers()
    prev = ops.set_precision("32-exact")
    try:
        mod.optimizer.zero_grad()
        loss = mod.training_step(_batch(case, data, dev), 0, eps=torch.from_numpy(data["in.eps"]).to(dev))
        loss.backward()
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
    tol = 1e-4
    out = mod._last_outputs
    for k in ("reconstruction", "mean", "logvar", "z"):
        assert rel_err(out[k].detach().cpu(), data[f"out.{k}"]) < tol, (k, rel_err(out[k].detach().cpu(),
                                                                                    data[f"out.{k}"]))
    for k in ("recon_loss", "kl_loss"):
        ref = float(data[f"loss.{k}"])
        assert abs(float(mod.logged[f"train/{k}"]) - ref) <= tol * abs(ref), k
    names = mod.flat.names
    has = [k for k, v in meta["param_has_grad"].items() if v]
    exact = math.sqrt(sum(float(data[f"gradsum.{k}"][1]) for k in has))
    got = math.sqrt(sum(float((mod.flat.params[names.index(k)]._mvae_main_grad.double() ** 2).sum()) for k in has))
    assert abs(got - exact) <= tol * exact, (got, exact)
    for k in FULL_GRADS[name]:
        g = mod.flat.params[names.index(k)]._mvae_main_grad.cpu()
        assert rel_err(g, data[f"grad.{k}"]) < 10 * tol, (k, rel_err(g, data[f"grad.{k}"]))
    if wino:
        assert {"mvae_winograd_gemm", "mvae_winograd_wgrad_gemm", "mvae_winograd_input_transform_gn"} <= seen
