#!/usr/bin/env python3
"""Generate golden input/output vectors from the REFERENCE implementation (run in the build
container only; /root/reference does not exist on the GPU box).

    python3 -B tests/golden/make_golden.py

For every case in cases.py this script
  1. imports the reference's own model classes (`src.models`, reference commit mounted read-only
     at /root/reference) and instantiates the case's model with its constructor kwargs,
  2. loads the deterministic synthetic weights of weights.py (no weights are stored),
  3. runs the reference training-step semantics on a synthetic MedMNIST-shaped batch:
       forward (src/lightning_module.py:115-128) with an injected reparameterization eps,
       loss (VAELoss src/losses/vae_losses.py:17-64 -- restated here with the same two torch
       calls because src.losses needs lpips/open_clip, which are not installed --, or the
       reference's own DisentangledVAELoss src/models/disentangled_conditional_vae.py:485-573),
       backward, zero non-finite grads (src/lightning_module.py:468-477), global-norm clip
       (:452-466, torch.nn.utils.clip_grad_norm_) and one Adam/AdamW step (:390-408),
  4. writes tests/golden/<case>.npz (plain arrays, allow_pickle=False) + <case>.json (metadata).

Only data leaves this script: inputs, outputs, loss terms, gradient and post-step checksums, and a
few full gradient tensors. No reference source is copied.
"""
from __future__ import annotations

import contextlib
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
REF = os.environ.get("MEDVAE_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.distributions import kl_divergence  # noqa: E402

import src.models as ref_models  # noqa: E402  (the reference)
from cases import CASES, FULL_GRADS  # noqa: E402
from weights import synth_param, synth_state, state_checksum  # noqa: E402


@contextlib.contextmanager
def injected_randn_like(eps: torch.Tensor):
    """BaseVAE.reparameterize (src/models/base_vae.py:83-87) draws eps with torch.randn_like;
    replace it by the fixture's eps so the CPU reference is deterministic."""
    orig = torch.randn_like

    def fake(t, *a, **k):
        assert tuple(t.shape) == tuple(eps.shape), (t.shape, eps.shape)
        return eps.clone()

    torch.randn_like = fake
    try:
        yield
    finally:
        torch.randn_like = orig


def make_inputs(case_name, case, model):
    rng = np.random.Generator(np.random.PCG64(2024 + len(case_name)))
    B = case["batch"]
    res = case["kwargs"]["resolution"]
    if case["cls"] == "DisentangledConditionalVAE":
        C = 3
    else:
        C = case["kwargs"]["input_channels"]
    x = rng.integers(0, 256, size=(B, C, res, res)).astype(np.float32) / np.float32(255.0)
    x = x * np.float32(2.0) - np.float32(1.0)
    ins = {"x": x}
    if case["cond"] == "onehot":
        idx = rng.integers(0, 12, size=(B,))
        oh = np.zeros((B, 12), np.float32)
        oh[np.arange(B), idx] = 1.0
        ins["cond"] = oh
    elif case["cond"] == "idx":
        idx = np.asarray(case["idx"], np.int64)
        # mixed_modality_collate_fn (src/data/medmnist_data.py:16-72): 1-channel modalities are
        # zero-padded to 3 channels.
        for b, m in enumerate(idx):
            mm = min(int(m), 4)
            if mm in (0, 3):
                x[b, 1:] = 0.0
        ins["cond"] = idx
    lat = model.latent_dim
    r = model.encoder_out_res
    ins["eps"] = rng.standard_normal(size=(B, lat, r, r)).astype(np.float32)
    return ins


def vae_loss(cfg, x, out):
    """VAELoss.forward, src/losses/vae_losses.py:37-64 (mse branch)."""
    rec = F.mse_loss(out["reconstruction"], x, reduction="mean")
    kl = kl_divergence(out["posterior"], out["prior"]).mean()
    loss = cfg.get("recon_weight", 1.0) * rec + cfg.get("kl_weight", 1.0) * kl
    return {"loss": loss, "recon_loss": rec, "kl_loss": kl}


def run_case(name, case):
    torch.manual_seed(0)
    cls = getattr(ref_models, case["cls"])
    kw = dict(case["kwargs"])
    if "ch_mult" in kw:
        kw["ch_mult"] = tuple(kw["ch_mult"])
    model = cls(**kw)
    model.train()
    seeded_init = {k: (float(v.double().sum()), float((v.double() ** 2).sum()))
                   for k, v in model.state_dict().items()}
    named = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    state = synth_state(named)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})

    ins = make_inputs(name, case, model)
    x = torch.from_numpy(ins["x"])
    eps = torch.from_numpy(ins["eps"])
    with injected_randn_like(eps):
        if case["cond"] == "none":
            out = model(x)
        elif case["cond"] == "onehot":
            out = model(x, torch.from_numpy(ins["cond"]))
        else:
            out = model(x, torch.from_numpy(ins["cond"]))

    cond_rec = {}
    if case["cond"] == "onehot":
        # the one-hot conditioning path of ConditionalVAE.encode (src/models/conditional_vae.py:107-136), from
        # the reference's own modules: the projection (Linear -> W[:, idx] + b for a one-hot row), its ReLU'd
        # [C, 8, 8] map and the bilinear condition map at the image size
        with torch.no_grad():
            c = torch.from_numpy(ins["cond"])
            cond_rec["out.cond_proj"] = model.condition_proj[0](c).numpy().copy()
            cond_rec["out.cond_map"] = model.create_condition_map(c, ins["x"].shape[2], ins["x"].shape[3]).numpy().copy()
    lcfg = case["loss"]
    if lcfg["type"] == "vae":
        ld = vae_loss(lcfg, x, out)
    else:
        crit = ref_models.DisentangledVAELoss(
            recon_loss_type=lcfg["recon_loss_type"], kl_weight=lcfg["kl_weight"],
            recon_weight=lcfg["recon_weight"], separation_weight=lcfg["separation_weight"],
            contrastive_weight=lcfg["contrastive_weight"])
        ld = crit(out, x)
    loss = ld["loss"]

    params = dict(model.named_parameters())
    for p in params.values():
        p.grad = None
    loss.backward()
    # on_before_optimizer_step: zero non-finite grads per tensor (lightning_module.py:468-477)
    for p in params.values():
        if p.grad is not None and (torch.isnan(p.grad).any() or torch.isinf(p.grad).any()):
            p.grad.zero_()
    rec = {}
    meta_grads = {}
    for k, p in params.items():
        if p.grad is None:
            meta_grads[k] = None
            continue
        g = p.grad.double()
        rec[f"gradsum.{k}"] = np.array([float(g.sum()), float((g * g).sum())])
        if k in FULL_GRADS.get(name, []):
            rec[f"grad.{k}"] = p.grad.numpy().copy()
        meta_grads[k] = True
    grads_with = [p for p in params.values() if p.grad is not None]
    total_norm = torch.nn.utils.clip_grad_norm_(grads_with, case["clip"])
    o = case["optimizer"]
    if o["type"] == "adam":
        opt = torch.optim.Adam(params.values(), lr=o["lr"], weight_decay=o["weight_decay"],
                               betas=tuple(o["betas"]))
    else:
        opt = torch.optim.AdamW(params.values(), lr=o["lr"], weight_decay=o["weight_decay"],
                                betas=tuple(o["betas"]))
    opt.step()
    for k, p in params.items():
        v = p.detach().double()
        rec[f"stepsum.{k}"] = np.array([float(v.sum()), float((v * v).sum())])
        if k in FULL_GRADS.get(name, []):
            rec[f"step.{k}"] = p.detach().numpy().copy()

    for k, v in ins.items():
        rec[f"in.{k}"] = v
    rec.update(cond_rec)
    for k in ("reconstruction", "mean", "logvar", "z"):
        rec[f"out.{k}"] = out[k].detach().numpy().copy()
    for k in ("separation_loss", "contrastive_loss"):
        if k in out:
            rec[f"out.{k}"] = np.array(float(out[k]))
    for k, v in ld.items():
        rec[f"loss.{k}"] = np.array(float(v))
    rec["clip.total_norm"] = np.array(float(total_norm))
    np.savez(os.path.join(HERE, f"{name}.npz"), **rec)
    meta = dict(case=case, params=[[k, list(s)] for k, s in named],
                param_has_grad={k: bool(v) for k, v in meta_grads.items()},
                weight_checksum=state_checksum(state), seeded_init_torch_seed0=seeded_init,
                reference="parsakzr/medvae-disentangled-multimodal @ 2025-08-24",
                torch=torch.__version__)
    with open(os.path.join(HERE, f"{name}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(f"{name}: loss={float(loss):.8f} recon={float(ld['recon_loss']):.8f} "
          f"kl={float(ld['kl_loss']):.8f} |g|={float(total_norm):.6f}")


DISC_FULL = ["main.0.weight", "main.0.bias", "main.3.weight", "main.3.bias", "main.11.weight", "main.11.bias"]


def disc_case():
    """Adversarial branch pinned on the reference's own NLayerDiscriminator (src/models/discriminator.py:11-82,
    default config: input_nc 3, ndf 64, n_layers 3, BatchNorm) in train mode, with the generator / discriminator
    objective arithmetic of LPIPSWithDiscriminator (src/losses/vae_losses.py:297-382; src.losses itself needs
    lpips, so its few torch calls are restated): g_loss = -mean(D(rec)), the adaptive weight
    |dNLL/dW| / (|dG/dW| + 1e-4) clamped to [0, 1e4] w.r.t. the last decoder layer W (here a conv3x3 8 -> 3
    producing rec; NLL = mse(rec, x) stands in for the perceptual term), and the hinge loss
    0.5 * (mean(relu(1 - D(x))) + mean(relu(1 + D(rec.detach())))). Three train-mode forwards in the training
    step's order (generator D(rec), then D(x), D(rec)) update the BatchNorm running statistics three times."""
    torch.manual_seed(0)
    D = ref_models.NLayerDiscriminator(input_nc=3, ndf=64, n_layers=3)
    D.train()
    named = [(k, tuple(v.shape)) for k, v in D.named_parameters()]
    state = synth_state(named)
    with torch.no_grad():
        for k, p in D.named_parameters():
            p.copy_(torch.from_numpy(state[k]))
    rng = np.random.Generator(np.random.PCG64(77))
    x = torch.from_numpy((rng.random((2, 3, 64, 64)) * 2 - 1).astype(np.float32))
    feat = torch.from_numpy(rng.standard_normal((2, 8, 64, 64)).astype(np.float32))
    w_last = torch.from_numpy(synth_param("last.weight", (3, 8, 3, 3))).requires_grad_()
    b_last = torch.from_numpy(synth_param("last.bias", (3,))).requires_grad_()
    rec = F.conv2d(feat, w_last, b_last, padding=1)
    nll = F.mse_loss(rec, x)
    logits_g = D(rec)
    g_loss = -torch.mean(logits_g)
    nll_grads = torch.autograd.grad(nll, w_last, retain_graph=True)[0]
    g_grads = torch.autograd.grad(g_loss, w_last, retain_graph=True)[0]
    d_weight = torch.clamp(torch.norm(nll_grads) / (torch.norm(g_grads) + 1e-4), 0.0, 1e4).detach()
    D.zero_grad()
    logits_real = D(x.detach())
    logits_fake = D(rec.detach())
    d_loss = 0.5 * (torch.mean(F.relu(1.0 - logits_real)) + torch.mean(F.relu(1.0 + logits_fake)))
    d_loss.backward()
    rec_arr = {"in.x": x.numpy(), "in.feat": feat.numpy(), "out.rec": rec.detach().numpy(),
               "out.logits_g": logits_g.detach().numpy(),
               "out.logits_real": logits_real.detach().numpy(), "out.logits_fake": logits_fake.detach().numpy(),
               "loss.g_loss": np.array(float(g_loss)), "loss.nll": np.array(float(nll)),
               "loss.d_weight": np.array(float(d_weight)), "loss.d_loss": np.array(float(d_loss)),
               "grad.nll_last": nll_grads.numpy(), "grad.g_last": g_grads.numpy()}
    for k, p in D.named_parameters():
        g = p.grad.double()
        rec_arr[f"gradsum.{k}"] = np.array([float(g.sum()), float((g * g).sum())])
        if k in DISC_FULL:
            rec_arr[f"grad.{k}"] = p.grad.numpy().copy()
    for k, b in D.named_buffers():
        if b.is_floating_point():
            rec_arr[f"buf.{k}"] = b.numpy().copy()
    np.savez(os.path.join(HERE, "disc.npz"), **rec_arr)
    meta = dict(params=[[k, list(s)] for k, s in named], weight_checksum=state_checksum(state),
                config=dict(input_nc=3, ndf=64, n_layers=3), full_grads=DISC_FULL,
                reference="parsakzr/medvae-disentangled-multimodal @ 2025-08-24", torch=torch.__version__)
    with open(os.path.join(HERE, "disc.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(f"disc: g_loss={float(g_loss):.8f} d_weight={float(d_weight):.6f} d_loss={float(d_loss):.8f}")


LATENT_B = 512  # the c3 bench batch (BASELINE config 3: bs 512, z [16, 7, 7])


def latent_case():
    """The batch-coupled latent losses at the c3 bench batch, on the reference's own
    DisentangledConditionalVAE.modality_separation_loss / contrastive_loss (src/models/
    disentangled_conditional_vae.py:305-386, partition_latent :195-206) -- a fixed z [512, 16, 7, 7] with ids uniform
    over the 5 modalities plus a few out-of-range ids (each its own centroid: the losses take the raw ids). Values and
    dL/dz of each term, in the reference's fp32 and with the same reference methods on float64 tensors. Only the
    partition's 8 + 8 elements (flat NCHW 0..15) can carry gradient: the fixture stores that [B, 16] slice and the
    largest magnitude elsewhere (0)."""
    torch.manual_seed(0)
    m = ref_models.DisentangledConditionalVAE(
        num_modalities=5, shared_latent_dim=8, modality_latent_dim=8, input_channels=3, latent_dim=16,
        hidden_channels=32, ch_mult=(1, 2, 4), num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28)
    rng = np.random.Generator(np.random.PCG64(512))
    z = rng.standard_normal(size=(LATENT_B, 16, 7, 7)).astype(np.float32)
    ids = rng.integers(0, 5, size=(LATENT_B,)).astype(np.int64)
    ids[[5, 77, 301]] = [7, 9, 17]
    rec = {"in.z": z, "in.idx": ids}
    for tag, dt in (("f32", torch.float32), ("f64", torch.float64)):
        for term, fn in (("sep", m.modality_separation_loss), ("con", m.contrastive_loss)):
            zt = torch.from_numpy(z).to(dt).requires_grad_()
            v = fn(zt, torch.from_numpy(ids))
            v.backward()
            g = zt.grad.reshape(LATENT_B, -1)
            rec[f"{term}.{tag}"] = np.array(float(v))
            rec[f"grad_{term}.{tag}"] = g[:, :16].numpy().astype(np.float64 if tag == "f64" else np.float32).copy()
            rec[f"grad_{term}_rest_max.{tag}"] = np.array(float(g[:, 16:].abs().max()))
    np.savez(os.path.join(HERE, "latent_b512.npz"), **rec)
    print(f"latent_b512: sep={float(rec['sep.f32']):.8f} ({float(rec['sep.f64']):.10f} f64) "
          f"con={float(rec['con.f32']):.8f} ({float(rec['con.f64']):.10f} f64)")


def known_answer_anchor():
    """SURVEY.md section 8(c) known-answer anchor, run on the reference itself."""
    torch.manual_seed(0)
    m = ref_models.BaseVAE(input_channels=3, latent_dim=16, hidden_channels=32, ch_mult=(1, 2, 4),
                           num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28)
    m.train()
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (4, 3, 28, 28), generator=g).float() / 255 * 2 - 1
    eps = torch.randn(4, 16, 7, 7, generator=g)
    with injected_randn_like(eps):
        out = m(x)
    ld = vae_loss({}, x, out)
    res = {k: float(v) for k, v in ld.items()}
    with open(os.path.join(HERE, "kat_anchor.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("anchor", res)


if __name__ == "__main__":
    torch.set_num_threads(8)
    sel = sys.argv[1:] or list(CASES) + ["disc", "latent"]
    for n in sel:
        if n == "disc":
            disc_case()
        elif n == "latent":
            latent_case()
        else:
            run_case(n, CASES[n])
    known_answer_anchor()
