"""Validation metrics on the device (src/utils/metrics.py:14-73, used by
VAELightningModule.validation_step, src/lightning_module.py:220-300).

`compute_reconstruction_metrics` / `compute_kl_metrics` keep the reference's names, arguments and
returned keys (floats, like the reference's `.item()` values); the `*_device` variants return 0-d
device tensors so a validation loop can log without a host sync per batch. MSE / MAE reuse the
fused loss reductions, PSNR follows torchmetrics' `peak_signal_noise_ratio(data_range=1.0)`, SSIM
and the KL statistics run on `csrc/metrics.hip`.
"""
from __future__ import annotations

import math
from typing import Dict

import torch

from . import _lib, ops


def ssim_per_image(preds: torch.Tensor, target: torch.Tensor, data_range: float = 1.0) -> torch.Tensor:
    ops._check(preds, "ssim input")
    p = ops.nhwc(preds.float())
    t = ops.nhwc(target.to(device=p.device, dtype=torch.float32))
    n, c, h, w = p.shape
    out = torch.empty(n, device=p.device, dtype=torch.float32)
    _lib.call("mvae_ssim", p.data_ptr(), t.data_ptr(), n, h, w, c, float(data_range), out.data_ptr(),
              ops._stream(p))
    return out


def compute_reconstruction_metrics_device(original: torch.Tensor, reconstructed: torch.Tensor) -> Dict[str, torch.Tensor]:
    with torch.no_grad():
        mse = ops.mse_mean(reconstructed, original)
        mae = ops.l1_mean(reconstructed, original)
        psnr = -10.0 * torch.log10(mse)  # torchmetrics PSNR, data_range = 1.0, over the whole batch
        ssim = ssim_per_image(reconstructed, original, 1.0).mean()
    return {"mse": mse, "mae": mae, "psnr": psnr, "ssim": ssim}


def compute_kl_metrics_device(mean: torch.Tensor, logvar: torch.Tensor) -> Dict[str, torch.Tensor]:
    ld_m = ops._pixel_ld(mean) if mean.dim() == 4 else None
    ld_l = ops._pixel_ld(logvar) if logvar.dim() == 4 else None
    if ld_m is not None and ld_m == ld_l:
        mu, lv, ld = mean, logvar, ld_m  # channel slices of the encoder output, read in place
        npix, zc = mean.shape[0] * mean.shape[2] * mean.shape[3], mean.shape[1]
    else:  # [B, D] latents (or any layout): per-sample sums over dim 1
        mu = mean.detach().float().reshape(mean.shape[0], mean.shape[1], -1).transpose(1, 2).contiguous()
        lv = logvar.detach().float().reshape(logvar.shape[0], logvar.shape[1], -1).transpose(1, 2).contiguous()
        npix, zc = mu.shape[0] * mu.shape[1], mu.shape[2]
        ld = zc
    out = torch.empty(4, device=mean.device, dtype=torch.float32)
    ws = ops.ARENA.get("klstats", _lib.query("mvae_kl_stats_workspace_bytes", npix), mean.device)
    _lib.call("mvae_kl_stats", mu.data_ptr(), lv.data_ptr(), ld, npix, zc, out.data_ptr(), ws.data_ptr(),
              ws.numel(), ops._stream(mean))
    return {"kl_total": out[0], "kl_mean": out[1], "kl_std": out[2], "kl_per_dim_mean": out[3]}


def compute_reconstruction_metrics(original: torch.Tensor, reconstructed: torch.Tensor) -> Dict[str, float]:
    return {k: float(v) for k, v in compute_reconstruction_metrics_device(original, reconstructed).items()}


def compute_kl_metrics(mean: torch.Tensor, logvar: torch.Tensor) -> Dict[str, float]:
    return {k: float(v) for k, v in compute_kl_metrics_device(mean, logvar).items()}
