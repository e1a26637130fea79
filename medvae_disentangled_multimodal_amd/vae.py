"""BaseVAE / BetaVAE / ConditionalVAE on the MI355X kernels.

Constructor kwargs, methods, forward-dict keys and state-dict names follow the reference
(src/models/base_vae.py:14-153, beta_vae.py:13-43, conditional_vae.py:14-203), so a Hydra config can
swap `_target_: src.models.BaseVAE` for `medvae_disentangled_multimodal_amd.BaseVAE`.
Extra (keyword-only) argument: `eps=` on forward/reparameterize injects the reparameterization
noise (used by the parity tests; the reference draws it with torch.randn_like).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal, kl_divergence

from . import ops
from .encoder_decoder import Conv2d, Decoder, Encoder


def _posterior(mean, logvar, std=None):
    post = Normal(mean, torch.exp(0.5 * logvar) if std is None else std, validate_args=False)
    post._mvae_mean = mean        # fast path for the fused KL kernel (losses.VAELoss)
    post._mvae_logvar = logvar
    return post


_UNIT = {}


def _prior(mean, logvar):
    # N(0, I) of the latent's shape as expanded views of cached per-device 0-d constants: the same distribution as
    # the reference's Normal(zeros_like(mu), ones_like(logvar)) without two fill launches per step
    key = (mean.device, mean.dtype)
    if key not in _UNIT:
        _UNIT[key] = (torch.zeros((), device=mean.device, dtype=mean.dtype),
                      torch.ones((), device=mean.device, dtype=mean.dtype))
    zero, one = _UNIT[key]
    prior = Normal(zero.expand(mean.shape), one.expand(logvar.shape), validate_args=False)
    prior._mvae_standard = True
    return prior


class BaseVAE(nn.Module):
    def __init__(self, input_channels: int = 1, latent_dim: int = 128, hidden_channels: int = 128,
                 ch_mult: Tuple[int, ...] = (1, 2, 4, 8), num_res_blocks: int = 2, attn_resolutions: list = [16],
                 dropout: float = 0.0, resolution: int = 224, use_linear_attn: bool = False,
                 attn_type: str = "vanilla", double_z: bool = True, **kwargs):
        super().__init__()
        self.latent_dim = latent_dim
        self.input_channels = input_channels
        self.encoder_out_res = resolution // (2 ** (len(ch_mult) - 1))
        common = dict(ch=hidden_channels, out_ch=input_channels, ch_mult=tuple(ch_mult),
                      num_res_blocks=num_res_blocks, attn_resolutions=list(attn_resolutions), dropout=dropout,
                      resamp_with_conv=True, in_channels=input_channels, resolution=resolution,
                      z_channels=latent_dim, use_linear_attn=use_linear_attn, attn_type=attn_type)
        self.encoder = Encoder(double_z=double_z, **common)
        self.decoder = Decoder(**common)

    # -- reference API --------------------------------------------------------------------
    def encode(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        h = self.encoder(ops.nhwc(x))
        mean, logvar = torch.chunk(h, 2, dim=1)  # channel slices of the NHWC output: views, no copy
        return mean, logvar

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        return self.decoder(z)

    def reparameterize(self, mean: torch.Tensor, logvar: torch.Tensor, *, eps: Optional[torch.Tensor] = None):
        if eps is None:
            eps = torch.randn(mean.shape, device=mean.device, dtype=mean.dtype).contiguous(
                memory_format=torch.channels_last)
        return ops.reparameterize(mean, logvar, eps)

    def _pack(self, mean, logvar, z, rec, return_latents, extra=None):
        out = {"reconstruction": rec, "mean": mean, "logvar": logvar, "z": z,
               "prior": _prior(mean, logvar), "posterior": _posterior(mean, logvar)}
        if extra:
            out.update(extra)
        if return_latents:
            out["latents"] = z
        return out

    def forward(self, x: torch.Tensor, return_latents: bool = False, *, eps=None) -> Dict[str, torch.Tensor]:
        mean, logvar = self.encode(x)
        z = self.reparameterize(mean, logvar, eps=eps)
        rec = self.decode(z)
        return self._pack(mean, logvar, z, rec, return_latents)

    def sample(self, num_samples: int, device) -> torch.Tensor:
        z = torch.randn(num_samples, self.latent_dim, self.encoder_out_res, self.encoder_out_res, device=device)
        return self.decode(z)

    def compute_loss(self, x, reconstruction, prior, posterior, **kwargs):
        from .losses import VAELoss
        d = VAELoss()(x, reconstruction, posterior, prior)
        return {"loss": d["loss"], "recon_loss": d["recon_loss"], "kl_loss": d["kl_loss"]}


class BetaVAE(BaseVAE):
    def __init__(self, beta: float = 1.0, **kwargs):
        super().__init__(**kwargs)
        self.beta = beta

    def compute_loss(self, x, reconstruction, prior, posterior, **kwargs):
        d = super().compute_loss(x, reconstruction, prior, posterior)
        total = d["recon_loss"] + self.beta * d["kl_loss"]
        return {"loss": total, "recon_loss": d["recon_loss"], "kl_loss": d["kl_loss"],
                "weighted_kl_loss": self.beta * d["kl_loss"]}


DEFAULT_MODALITIES = ["chest_xray", "pathology", "oct", "pneumonia", "dermatoscope", "blood_cell", "tissue",
                      "retina", "breast_ultrasound", "abdominal_ct_a", "abdominal_ct_c", "abdominal_ct_s"]


class FiLMLayer(nn.Module):
    def __init__(self, condition_dim: int, feature_dim: int):
        super().__init__()
        self.scale_transform = nn.Linear(condition_dim, feature_dim)
        self.shift_transform = nn.Linear(condition_dim, feature_dim)

    def forward(self, features, condition):
        return features * self.scale_transform(condition)[..., None, None] + \
            self.shift_transform(condition)[..., None, None]


class ConditionalVAE(BaseVAE):
    """Concat-conditioned VAE: one-hot -> Linear -> ReLU -> [C,8,8] -> bilinear -> concat with x."""

    def __init__(self, modalities: List[str] = None, condition_dim: int = None, condition_method: str = "concat",
                 **kwargs):
        super().__init__(**kwargs)
        self.modalities = list(modalities) if modalities is not None else list(DEFAULT_MODALITIES)
        self.num_modalities = len(self.modalities)
        self.condition_dim = condition_dim or self.num_modalities
        self.condition_method = condition_method
        if condition_method == "concat":
            self.condition_proj = nn.Sequential(nn.Linear(self.condition_dim, self.input_channels * 64), nn.ReLU(),
                                                nn.Unflatten(1, (self.input_channels, 8, 8)))
            self.encoder.conv_in = Conv2d(self.input_channels * 2, self.encoder.ch, 3, 1, 1)
        elif condition_method == "inject":
            # parameters exist in the reference but are never used by its forward (conditional_vae.py:80-89)
            self.condition_embedding = nn.Sequential(nn.Linear(self.condition_dim, 512), nn.ReLU(),
                                                     nn.Linear(512, 512))
        elif condition_method == "film":
            self.film_layers = nn.ModuleList(
                [FiLMLayer(self.condition_dim, self.encoder.ch * (2 ** i)) for i in range(len(self.encoder.down))])

    def encode_condition(self, condition):
        return condition.unsqueeze(0) if condition.dim() == 1 else condition

    def create_condition_map(self, condition, height: int, width: int):
        cmap = self.condition_proj(condition)
        return F.interpolate(cmap, size=(height, width), mode="bilinear", align_corners=False)

    def encode(self, x, condition):
        # one fused conditioning op (csrc/condition.hip) up to 256 x 256 (every reference config: <= 224); larger
        # images take the module path (Linear + ReLU + bilinear interpolate + cat, conditional_vae.py:107-127)
        if self.condition_method == "concat" and ops.condition_concat_fits(x):
            lin = self.condition_proj[0]
            x_cond, _ = ops.condition_concat(x, condition, lin.weight, lin.bias)
            return super().encode(x_cond)
        if self.condition_method == "concat":
            cmap = self.create_condition_map(condition.to(x.dtype), x.shape[2], x.shape[3])
            x_cond = torch.cat([x, cmap], dim=1).contiguous(memory_format=torch.channels_last)
            return super().encode(x_cond)
        return super().encode(x)

    def forward(self, x, condition, return_latents: bool = False, *, eps=None):
        mean, logvar = self.encode(x, condition)
        z = self.reparameterize(mean, logvar, eps=eps)
        rec = self.decode(z)
        return self._pack(mean, logvar, z, rec, return_latents, {"condition": condition})

    def conditional_sample(self, num_samples: int, condition, device):
        return self.sample(num_samples, device)

    def get_modality_condition(self, modality: str) -> torch.Tensor:
        if modality not in self.modalities:
            raise ValueError(f"Unknown modality: {modality}")
        c = torch.zeros(self.num_modalities)
        c[self.modalities.index(modality)] = 1.0
        return c
