"""DisentangledConditionalVAE on the MI355X kernels
(reference: src/models/disentangled_conditional_vae.py:14-482).

The reference routes every sample through a Python loop (`.item()` per sample, per-sample conv
launches: :137-169, :255-301). Here the routing is batched and stays on the device: ONE launch routes
the batch through the input projectors and ONE through the modality heads (csrc/routing.hip): each
sample reads its modality id on the device and runs only that modality's layers (no host sync, no
work on the other heads). Images too large for the kernels' LDS tiles use the grouped form: every
head over the whole batch on the HIP conv kernel, then an exact per-sample index select.
Semantics kept: out-of-range indices clamp to the last modality (:142-146, :258-265), 1-channel
modalities use only channel 0 of the (collate-padded) input, NaN scrubbing (:132-191), mu/logvar clamp
to [-10, 10] (:409-412), `partition_latent`'s NCHW flatten order (:195-206), separation loss over the
sorted unique (unclamped) modality ids (:305-349), masked InfoNCE contrastive loss (:351-386).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

from . import ops
from .encoder_decoder import Conv2d
from .vae import BaseVAE, _posterior, _prior

# batched per-sample routing kernels (csrc/routing.hip); MVAE_NO_ROUTING=1 selects the grouped-conv form
ROUTING_KERNELS = os.environ.get("MVAE_NO_ROUTING") is None
# fused latent side of the forward (ops.latent_prep); MVAE_NO_LATENT_PREP=1 keeps the torch clamp / reparam chain
LATENT_PREP = os.environ.get("MVAE_NO_LATENT_PREP") is None


def _nan_to_zero(t):
    return torch.where(torch.isnan(t), 0.0, t)


class DisentangledConditionalVAE(BaseVAE):
    def __init__(self, num_modalities: int = 5, shared_latent_dim: int = 8, modality_latent_dim: int = 8,
                 modality_separation_weight: float = 1.0, contrastive_weight: float = 0.5, resolution: int = 28,
                 hidden_channels: int = 128, ch_mult: Tuple[int, ...] = (1, 2, 4, 8), num_res_blocks: int = 2,
                 attn_resolutions: list = [16], dropout: float = 0.0, use_linear_attn: bool = False,
                 attn_type: str = "vanilla", **kwargs):
        self.num_modalities = num_modalities
        self.shared_latent_dim = shared_latent_dim
        self.modality_latent_dim = modality_latent_dim
        self.modality_separation_weight = modality_separation_weight
        self.contrastive_weight = contrastive_weight
        self.modality_channels = self._get_modality_channel_map()
        max_channels = max(self.modality_channels.values())
        kwargs.update(latent_dim=shared_latent_dim + modality_latent_dim, resolution=resolution,
                      input_channels=max_channels, hidden_channels=hidden_channels, ch_mult=ch_mult,
                      num_res_blocks=num_res_blocks, attn_resolutions=attn_resolutions, dropout=dropout,
                      use_linear_attn=use_linear_attn, attn_type=attn_type)
        super().__init__(**kwargs)
        self.resolution = resolution
        self.modality_input_projectors = nn.ModuleDict()
        for m, c in self.modality_channels.items():
            if c != max_channels:
                self.modality_input_projectors[str(m)] = Conv2d(c, max_channels, 1, 1, 0)
        self.modality_output_projectors = nn.ModuleDict()
        for m, c in self.modality_channels.items():
            if c != max_channels:
                self.modality_output_projectors[str(m)] = Conv2d(max_channels, c, 1, 1, 0)
        self.modality_embedding = nn.Embedding(num_modalities, 64)  # unused by the reference forward
        self.modality_decoders = nn.ModuleList([
            nn.Sequential(Conv2d(max_channels, max_channels, 3, 1, 1), nn.ReLU(),
                          Conv2d(max_channels, max_channels, 3, 1, 1)) for _ in range(num_modalities)])

    @staticmethod
    def _get_modality_channel_map() -> Dict[int, int]:
        return {0: 1, 1: 3, 2: 3, 3: 1, 4: 3}

    @staticmethod
    def _clamp(idx: torch.Tensor, n: int) -> torch.Tensor:
        return torch.where(idx >= n, torch.full_like(idx, n - 1), idx)

    # -- parameter usage (optimizer skips parameters without a gradient, like torch.optim) ----
    def parameter_modality(self, name: str) -> int:
        """-1: always used; -2: never used (dead parameter); m >= 0: used iff modality m is present."""
        if name.startswith("modality_embedding."):
            return -2
        for pfx in ("modality_input_projectors.", "modality_output_projectors.", "modality_decoders."):
            if name.startswith(pfx):
                return int(name[len(pfx):].split(".")[0])
        return -1

    def modality_presence(self, modality_indices: torch.Tensor) -> torch.Tensor:
        idx = self._clamp(modality_indices.long(), self.num_modalities)
        return (idx[:, None] == torch.arange(self.num_modalities, device=idx.device)[None, :]).any(0)

    # -- routing ------------------------------------------------------------------------------
    def _route_in_params(self):
        ps = []
        for m in range(len(self.modality_channels)):
            proj = self.modality_input_projectors[str(m)] if str(m) in self.modality_input_projectors else None
            ps += [proj.weight, proj.bias] if proj is not None else [None, None]
        return ps

    def _head_params(self):
        ps = []
        for m, head in enumerate(self.modality_decoders):
            proj = self.modality_output_projectors[str(m)] if str(m) in self.modality_output_projectors else None
            ps += [head[0].weight, head[0].bias, head[2].weight, head[2].bias]
            ps += [proj.weight, proj.bias] if proj is not None else [None, None]
        return ps

    def _routing_kernel_ok(self, t: torch.Tensor) -> bool:
        mx = max(self.modality_channels.values())
        return (t.is_cuda and ROUTING_KERNELS and len(self.modality_channels) == len(self.modality_decoders) and
                all(c in (1, mx) for c in self.modality_channels.values()) and
                ops.routing_fits(t.shape[2], t.shape[3], mx, len(self.modality_decoders)))

    def _encode_routed_raw(self, x: torch.Tensor, modality_indices: torch.Tensor) -> torch.Tensor:
        """The encoder output [B, 2 z, r, r] of the routed batch before the chunk / NaN scrub (routing-kernel path)."""
        mx = max(self.modality_channels.values())
        routed = ops.modality_route_in(x, modality_indices, mx, len(self.modality_channels), self._route_in_params())
        return self.encoder(ops.nhwc(routed))

    def encode(self, x: torch.Tensor, modality_indices: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        mx = max(self.modality_channels.values())
        if self._routing_kernel_ok(x):  # one launch: each sample through its own input projector (csrc/routing.hip)
            mu, logvar = torch.chunk(self._encode_routed_raw(x, modality_indices), 2, dim=1)
            return _nan_to_zero(mu), _nan_to_zero(logvar)
        x = _nan_to_zero(x)
        idx = self._clamp(modality_indices.to(x.device).long(), len(self.modality_channels))
        sel = idx.view(-1, 1, 1, 1)
        if x.shape[1] >= mx:
            routed = x[:, :mx]
        else:  # fewer channels than the colour modalities take (a 1-channel batch): zero-padded, as the collate
            # pads gray images (medmnist_data.py:16-72) and as the routing kernel reads them (the reference errors)
            routed = torch.cat([x, x.new_zeros((x.shape[0], mx - x.shape[1]) + tuple(x.shape[2:]))], 1)
        gray = x[:, :1]
        for key, proj in self.modality_input_projectors.items():
            p = _nan_to_zero(proj(gray))
            routed = torch.where(sel == int(key), p, routed)
        mu, logvar = BaseVAE.encode(self, _nan_to_zero(routed))
        return _nan_to_zero(mu), _nan_to_zero(logvar)

    def _decode_routed(self, z, modality_indices, out_channels: Optional[int]):
        rec = BaseVAE.decode(self, z)
        idx = self._clamp(modality_indices.to(rec.device).long(), len(self.modality_decoders))
        if out_channels is None:
            colour = [m for m, c in self.modality_channels.items() if c == max(self.modality_channels.values())]
            out_channels = 3 if bool(torch.isin(idx, torch.tensor(colour, device=idx.device)).any()) else 1
        if self._routing_kernel_ok(rec):  # one launch: each sample through its own head + projector
            return ops.modality_heads(rec, modality_indices, out_channels, len(self.modality_decoders),
                                      self._head_params())
        sel = idx.view(-1, 1, 1, 1)
        heads = torch.zeros_like(rec)
        for m, head in enumerate(self.modality_decoders):
            heads = torch.where(sel == m, head(rec), heads)
        out = heads[:, :out_channels] if out_channels <= heads.shape[1] else heads
        for key, proj in self.modality_output_projectors.items():
            o = proj(heads)  # [B, c_m, H, W]
            if o.shape[1] < out_channels:
                o = torch.cat([o, o.new_zeros((o.shape[0], out_channels - o.shape[1]) + tuple(o.shape[2:]))], 1)
            out = torch.where(sel == int(key), o, out)
        return out

    def decode(self, z: torch.Tensor, modality_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        if modality_indices is None:
            return BaseVAE.decode(self, z)
        hint = None
        if not modality_indices.is_cuda:
            mx = max(self.modality_channels.values())
            idx = self._clamp(modality_indices.long(), len(self.modality_decoders))
            hint = max(self.modality_channels[int(m)] for m in idx.tolist())
            hint = mx if hint == mx else hint
        return self._decode_routed(z, modality_indices, hint)

    # -- latent partition and auxiliary losses ---------------------------------------------------
    def partition_latent(self, z: torch.Tensor):
        flat = z.reshape(z.shape[0], -1)  # logical NCHW flatten order
        return (flat[:, :self.shared_latent_dim],
                flat[:, self.shared_latent_dim:self.shared_latent_dim + self.modality_latent_dim])

    def reconstruct_latent(self, z_shared, z_modality):
        rem = self.latent_dim - self.shared_latent_dim - self.modality_latent_dim
        parts = [z_shared, z_modality]
        if rem > 0:
            parts.append(torch.zeros(z_shared.shape[0], rem, device=z_shared.device))
        z_full = torch.cat(parts, 1)
        r = self.encoder_out_res
        spatial = int((z_full.shape[1] / (r ** 2)) ** 0.5)
        if spatial ** 2 * r ** 2 != z_full.shape[1]:
            return z_full.view(z_full.shape[0], -1, r, r)
        return z_full.view(z_full.shape[0], spatial, r, r)

    def modality_separation_loss(self, z: torch.Tensor, modality_indices: torch.Tensor) -> torch.Tensor:
        """-mean pdist of the centroids of every distinct (unclamped) modality id, :305-349. The ids of
        `torch.unique` become segment numbers of the sorted ids (any id value, no host sync): B segment
        slots, of which the first (#distinct) are present."""
        _, zm = self.partition_latent(z)
        idx = modality_indices.to(z.device).long().view(-1)
        nb = idx.shape[0]
        srt, perm = torch.sort(idx, stable=True)
        new = torch.ones_like(srt, dtype=torch.bool)
        new[1:] = srt[1:] != srt[:-1]
        seg = torch.empty_like(idx)
        seg[perm] = torch.cumsum(new.long(), 0) - 1
        oh = (seg[:, None] == torch.arange(nb, device=z.device)[None, :]).to(zm.dtype)  # [B, B]
        cnt = oh.sum(0)
        present = cnt > 0
        cent = (oh.t() @ zm) / cnt.clamp_min(1.0)[:, None]
        # direct-difference distances without a [B, B, D] tensor (torch.pdist's arithmetic; cdist's backward gives
        # the zero-distance pairs of absent slots a zero gradient, and they are masked out anyway)
        d = torch.cdist(cent[None], cent[None], compute_mode="donot_use_mm_for_euclid_dist")[0]
        iu = torch.triu(torch.ones(nb, nb, dtype=torch.bool, device=z.device), diagonal=1)
        pair = iu & present[:, None] & present[None, :]
        dist = torch.where(pair, d, torch.zeros_like(d))
        npair = pair.sum()
        loss = -dist.sum() / npair.clamp_min(1).to(zm.dtype)
        return torch.where(present.sum() >= 2, loss, torch.zeros_like(loss))

    def contrastive_loss(self, z: torch.Tensor, modality_indices: torch.Tensor, temperature: float = 0.1):
        _, zm = self.partition_latent(z)
        idx = modality_indices.to(z.device)
        zn = F.normalize(zm, p=2, dim=1)
        sim = zn @ zn.t() / temperature
        pos = idx[None, :] == idx[:, None]
        pos = pos & ~torch.eye(pos.shape[0], dtype=torch.bool, device=z.device)
        e = torch.exp(sim)
        ps = (e * pos.to(e.dtype)).sum(1)
        tot = e.sum(1) - torch.diagonal(e)
        l = -torch.log(ps / tot + 1e-8)
        has = ps > 0
        n = has.sum()
        loss = torch.where(has, l, torch.zeros_like(l)).sum() / n.clamp_min(1).to(l.dtype)
        return torch.where(n > 0, loss, torch.zeros_like(loss))

    def forward(self, x: torch.Tensor, modality_indices: torch.Tensor, return_latents: bool = False, *, eps=None):
        std = None
        if LATENT_PREP and self._routing_kernel_ok(x):
            # NaN scrub + clamps + reparameterization + posterior std: one launch per direction (csrc/loss.hip)
            h = self._encode_routed_raw(x, modality_indices)
            zc = h.shape[1] // 2
            if eps is None:
                eps = torch.randn((h.shape[0], zc) + tuple(h.shape[2:]), device=h.device,
                                  dtype=torch.float32).contiguous(memory_format=torch.channels_last)
            mu, logvar, std, z = ops.latent_prep(h, zc, eps)
        else:
            mu, logvar = self.encode(x, modality_indices)
            logvar = torch.clamp(logvar, min=-10.0, max=10.0)
            mu = torch.clamp(mu, min=-10.0, max=10.0)
            z = self.reparameterize(mu, logvar, eps=eps)
        hint = 1 if x.shape[1] == 1 else max(self.modality_channels.values())
        rec = self._decode_routed(z, modality_indices, hint)
        # gated terms: a NaN/Inf value drops the term's gradient (DisentangledVAELoss replaces it by 0, :540-550)
        if ops.latent_aux_fits(z, self.modality_latent_dim) and modality_indices.is_cuda:
            sep, con = ops.latent_aux_losses(z, modality_indices, self.shared_latent_dim, self.modality_latent_dim)
        else:
            sep = ops.finite_gated(lambda zz: self.modality_separation_loss(zz, modality_indices), z)
            con = ops.finite_gated(lambda zz: self.contrastive_loss(zz, modality_indices), z)
        if std is None:
            std = torch.clamp(torch.exp(0.5 * logvar), min=1e-6, max=10.0)
        out = {"reconstruction": rec, "mean": mu, "logvar": logvar, "mu": mu, "z": z,
               "prior": _prior(mu, std), "posterior": _posterior(mu, logvar, std),
               "separation_loss": sep, "contrastive_loss": con}
        if return_latents:
            zs, zmod = self.partition_latent(z)
            out.update(z_shared=zs, z_modality=zmod)
        return out

    def sample_conditional(self, num_samples: int, modality_indices: torch.Tensor, device):
        z = torch.randn(num_samples, self.latent_dim, self.encoder_out_res, self.encoder_out_res, device=device)
        with torch.no_grad():
            shift = (modality_indices.to(device).float() - 2.0) * 0.3
            z = z + shift.view(-1, 1, 1, 1)
        return self.decode(z, modality_indices)
