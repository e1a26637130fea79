"""VAE objectives on the fused HIP reduction kernels.

VAELoss mirrors src/losses/vae_losses.py:17-64 (same constructor kwargs, forward signature and
returned keys). When the posterior comes from this package's models, the KL term runs on the fused
kernel straight from (mean, logvar) slices of the encoder output; any other Normal pair falls back to
torch.distributions (not on the hot path).
"""
from __future__ import annotations

import os
from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal, kl_divergence

from . import ops

# DisentangledVAELoss's term guards + weighted total as one fused launch (ops.loss_combine); MVAE_NO_FUSED_COMBINE=1
# keeps the torch where / isfinite chain
FUSED_COMBINE = os.environ.get("MVAE_NO_FUSED_COMBINE") is None


def _recon(kind: str, rec: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    if kind == "mse":
        return ops.mse_mean(rec, x)
    if kind == "l1":
        return ops.l1_mean(rec, x)
    if kind == "bce":
        return F.binary_cross_entropy_with_logits(rec, x.to(rec.dtype), reduction="mean")
    raise ValueError(f"Unknown reconstruction loss type: {kind}")


class VAELoss(nn.Module):
    def __init__(self, recon_loss_type: str = "mse", kl_weight: float = 1.0, recon_weight: float = 1.0):
        super().__init__()
        self.recon_loss_type = recon_loss_type
        self.kl_weight = kl_weight
        self.recon_weight = recon_weight

    def forward(self, inputs, reconstructions, posteriors: Normal, priors: Normal, **kwargs) -> Dict[str, torch.Tensor]:
        recon = _recon(self.recon_loss_type, reconstructions, inputs)
        if hasattr(posteriors, "_mvae_logvar") and getattr(priors, "_mvae_standard", False):
            kl = ops.kl_standard_normal_mean(posteriors._mvae_mean, posteriors._mvae_logvar)
        else:
            kl = kl_divergence(posteriors, priors).mean()
        total = self.recon_weight * recon + self.kl_weight * kl
        return {"loss": total, "recon_loss": recon, "kl_loss": kl}


def _finite_or_zero(v: torch.Tensor) -> torch.Tensor:
    # device-side replacement of the reference's `if isnan(v).any(): v = 0` (no host sync); the term's own
    # gradient is gated by ops.finite_gated where it is computed, so a non-finite term contributes nothing
    return torch.where(torch.isfinite(v), v, 0.0)


class DisentangledVAELoss(nn.Module):
    """src/models/disentangled_conditional_vae.py:485-573."""

    def __init__(self, recon_loss_type: str = "mse", kl_weight: float = 1.0, recon_weight: float = 1.0,
                 separation_weight: float = 0.1, contrastive_weight: float = 0.05):
        super().__init__()
        if recon_loss_type not in ("mse", "l1"):
            raise ValueError(f"Unknown reconstruction loss: {recon_loss_type}")
        self.recon_loss_type = recon_loss_type
        self.kl_weight, self.recon_weight = kl_weight, recon_weight
        self.separation_weight, self.contrastive_weight = separation_weight, contrastive_weight

    def forward(self, outputs: Dict[str, torch.Tensor], targets: torch.Tensor) -> Dict[str, torch.Tensor]:
        kind, n = self.recon_loss_type, targets.numel()
        recon = ops.finite_gated(lambda r, t: _recon(kind, r, t), outputs["reconstruction"], targets)
        kl = ops.finite_gated(lambda m, lv: ops.kl_closed_form_sum(m, lv, n), outputs["mu"], outputs["logvar"])
        sep, con = outputs["separation_loss"], outputs["contrastive_loss"]
        if FUSED_COMBINE and recon.is_cuda:  # finite-or-zero terms + weighted total + its guard: one launch each way
            total, recon, kl, sep, con = ops.loss_combine(
                [recon, kl, sep, con],
                [self.recon_weight, self.kl_weight, self.separation_weight, self.contrastive_weight])
            return {"loss": total, "recon_loss": recon, "kl_loss": kl, "separation_loss": sep,
                    "contrastive_loss": con}
        recon, kl = _finite_or_zero(recon), _finite_or_zero(kl)
        sep, con = _finite_or_zero(sep), _finite_or_zero(con)
        total = (self.recon_weight * recon + self.kl_weight * kl + self.separation_weight * sep +
                 self.contrastive_weight * con)
        total = torch.where(torch.isfinite(total), total, 1e6)
        return {"loss": total, "recon_loss": recon, "kl_loss": kl, "separation_loss": sep,
                "contrastive_loss": con}


class LPIPSLoss(nn.Module):
    """Perceptual loss of the reference (vae_losses.py:67-94): LPIPS(x*2-1, rec*2-1).mean(), gray
    inputs repeated to 3 channels. Backed by `lpips.LPIPS` (AlexNet) on the HIP kernels; the
    pretrained weights come from `weights=` / MVAE_LPIPS_WEIGHTS (see lpips.py)."""

    def __init__(self, net: str = "alex", use_gpu: bool = True, weights=None, allow_synthetic: bool = False,
                 seed: int = 0):
        super().__init__()
        from .lpips import LPIPS
        self.lpips = LPIPS(net=net, weights=weights, allow_synthetic=allow_synthetic, seed=seed)
        if use_gpu and torch.cuda.is_available():
            self.lpips = self.lpips.cuda()

    def forward(self, inputs: torch.Tensor, reconstructions: torch.Tensor) -> torch.Tensor:
        if inputs.shape[1] == 1:
            inputs = inputs.repeat(1, 3, 1, 1)
        if reconstructions.shape[1] == 1:
            reconstructions = reconstructions.repeat(1, 3, 1, 1)
        return self.lpips(inputs, reconstructions, pre_a=2.0, pre_b=-1.0).mean()


class LPIPSWithDiscriminator(nn.Module):
    """The reference's combined objective (vae_losses.py:214-382) on the HIP kernels.

    optimizer_idx 0 (generator): perceptual_factor * LPIPS + kl_factor * KL(q || N(0, I)).sum() / B
    + d_weight * g_loss, g_loss = -mean(D(rec)) and the adaptive d_weight = |dNLL/dW| / (|dG/dW| + 1e-4)
    (clamped to [0, 1e4], times discriminator_factor) w.r.t. the decoder's last conv, once global_step
    >= discriminator_iter_start. optimizer_idx 1 (discriminator): hinge loss
    0.5 * (mean(relu(1 - D(x))) + mean(relu(1 + D(rec)))) once active, else 0.
    The reference calls `posteriors.kl()`, which a torch Normal does not have; the closed-form KL is
    used."""

    def __init__(self, discriminator_factor: float = 1.0, perceptual_factor: float = 1.0, kl_factor: float = 1.0,
                 discriminator_iter_start: int = 50001, use_biomedclip_loss: bool = False,
                 biomedclip_factor: float = 1.0, discriminator_config=None, lpips_weights=None,
                 allow_synthetic_lpips: bool = False, lpips_net: str = "alex"):
        super().__init__()
        if use_biomedclip_loss:
            raise NotImplementedError("BiomedCLIP loss is outside the MI355X hot path")
        from .discriminator import NLayerDiscriminator
        self.discriminator_factor = discriminator_factor
        self.perceptual_factor = perceptual_factor
        self.kl_factor = kl_factor
        self.discriminator_iter_start = discriminator_iter_start
        self.perceptual_loss = LPIPSLoss(net=lpips_net, weights=lpips_weights, allow_synthetic=allow_synthetic_lpips)
        if discriminator_config is None:
            discriminator_config = {"input_nc": 3, "ndf": 64, "n_layers": 3}
        self.discriminator = NLayerDiscriminator(**discriminator_config)

    def calculate_adaptive_weight(self, nll_loss, g_loss, last_layer):
        with ops.autograd_weight_grads():  # the probes must not touch the flat gradient buffer
            nll_grads = torch.autograd.grad(nll_loss, last_layer.weight, retain_graph=True)[0]
            g_grads = torch.autograd.grad(g_loss, last_layer.weight, retain_graph=True)[0]
        d_weight = torch.norm(nll_grads) / (torch.norm(g_grads) + 1e-4)
        return torch.clamp(d_weight, 0.0, 1e4).detach()

    def forward(self, inputs, reconstructions, latent=None, posteriors=None, optimizer_idx: int = 0,
                global_step: int = 0, last_layer=None, split: str = "train", **kwargs):
        bsz = inputs.shape[0]
        d_valid = global_step >= self.discriminator_iter_start
        zero = torch.zeros((), device=inputs.device)
        if optimizer_idx == 0:
            p_loss = self.perceptual_loss(inputs, reconstructions)
            kl_loss = ops.kl_closed_form_sum(posteriors._mvae_mean, posteriors._mvae_logvar, bsz)
            d_weight, g_loss = zero, zero
            if d_valid:
                rec = reconstructions.repeat(1, 3, 1, 1) if reconstructions.shape[1] == 1 else reconstructions
                dparams = list(self.discriminator.parameters())
                flags = [p.requires_grad for p in dparams]
                for p in dparams:  # the generator step updates only the VAE: skip D's weight gradients
                    p.requires_grad_(False)
                try:
                    g_loss = ops.neg_mean(self.discriminator(rec))
                finally:
                    for p, f in zip(dparams, flags):
                        p.requires_grad_(f)
                try:
                    d_weight = self.calculate_adaptive_weight(p_loss, g_loss, last_layer) if last_layer is not None \
                        else zero
                except RuntimeError:
                    d_weight = zero
                d_weight = d_weight * self.discriminator_factor
            loss = self.perceptual_factor * p_loss + self.kl_factor * kl_loss + d_weight * g_loss
            log = {f"{split}/total_loss": loss.detach(), f"{split}/kl_loss": kl_loss.detach(),
                   f"{split}/p_loss": p_loss.detach(), f"{split}/d_weight": d_weight.detach(),
                   f"{split}/g_loss": g_loss.detach()}
            return loss, log
        if d_valid:
            x = inputs.repeat(1, 3, 1, 1) if inputs.shape[1] == 1 else inputs
            r = reconstructions.repeat(1, 3, 1, 1) if reconstructions.shape[1] == 1 else reconstructions
            logits_real = self.discriminator(x.contiguous().detach())
            logits_fake = self.discriminator(r.contiguous().detach())
            d_loss = 0.5 * (ops.hinge_real(logits_real) + ops.hinge_fake(logits_fake))
        else:
            d_loss = zero
        return d_loss, {f"{split}/d_loss": d_loss.detach()}
