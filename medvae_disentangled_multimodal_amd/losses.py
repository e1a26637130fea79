"""VAE objectives on the fused HIP reduction kernels.

VAELoss mirrors src/losses/vae_losses.py:17-64 (same constructor kwargs, forward signature and
returned keys). When the posterior comes from this package's models, the KL term runs on the fused
kernel straight from (mean, logvar) slices of the encoder output; any other Normal pair falls back to
torch.distributions (not on the hot path).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal, kl_divergence

from . import ops


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
    # device-side replacement of the reference's `if isnan(v).any(): v = 0` (no host sync)
    return torch.where(torch.isfinite(v), v, torch.zeros_like(v))


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
        recon = _finite_or_zero(_recon(self.recon_loss_type, outputs["reconstruction"], targets))
        kl = _finite_or_zero(ops.kl_closed_form_sum(outputs["mu"], outputs["logvar"], targets.numel()))
        sep = _finite_or_zero(outputs["separation_loss"])
        con = _finite_or_zero(outputs["contrastive_loss"])
        total = (self.recon_weight * recon + self.kl_weight * kl + self.separation_weight * sep +
                 self.contrastive_weight * con)
        total = torch.where(torch.isfinite(total), total, torch.full_like(total, 1e6))
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
    """Generator objective of the reference's combined loss (vae_losses.py:214-362):
    perceptual_factor * LPIPS + kl_factor * KL(q || N(0, I)).sum() / B (+ d_weight * g_loss once
    global_step >= discriminator_iter_start). The reference calls `posteriors.kl()`, which a
    torch Normal does not have; the closed-form KL is used. The
    adversarial branch (NLayerDiscriminator, adaptive weight) is the next scope row and raises."""

    def __init__(self, discriminator_factor: float = 1.0, perceptual_factor: float = 1.0, kl_factor: float = 1.0,
                 discriminator_iter_start: int = 50001, use_biomedclip_loss: bool = False,
                 biomedclip_factor: float = 1.0, discriminator_config=None, lpips_weights=None,
                 allow_synthetic_lpips: bool = False, lpips_net: str = "alex"):
        super().__init__()
        if use_biomedclip_loss:
            raise NotImplementedError("BiomedCLIP loss is outside the MI355X hot path")
        self.discriminator_factor = discriminator_factor
        self.perceptual_factor = perceptual_factor
        self.kl_factor = kl_factor
        self.discriminator_iter_start = discriminator_iter_start
        self.perceptual_loss = LPIPSLoss(net=lpips_net, weights=lpips_weights, allow_synthetic=allow_synthetic_lpips)

    def forward(self, inputs, reconstructions, latent=None, posteriors=None, optimizer_idx: int = 0,
                global_step: int = 0, last_layer=None, split: str = "train", **kwargs):
        bsz = inputs.shape[0]
        d_valid = global_step >= self.discriminator_iter_start
        if d_valid:
            raise NotImplementedError("adversarial branch (NLayerDiscriminator) is not built yet")
        if optimizer_idx == 1:
            zero = torch.zeros((), device=inputs.device)
            return zero, {f"{split}/d_loss": zero}
        p_loss = self.perceptual_loss(inputs, reconstructions)
        kl_loss = ops.kl_closed_form_sum(posteriors._mvae_mean, posteriors._mvae_logvar, bsz)
        zero = torch.zeros((), device=inputs.device)
        loss = self.perceptual_factor * p_loss + self.kl_factor * kl_loss
        log = {f"{split}/total_loss": loss.detach(), f"{split}/kl_loss": kl_loss.detach(),
               f"{split}/p_loss": p_loss.detach(), f"{split}/d_weight": zero, f"{split}/g_loss": zero}
        return loss, log
