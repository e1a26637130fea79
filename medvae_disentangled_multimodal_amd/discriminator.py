"""PatchGAN discriminator of the adversarial branch on the HIP kernels.

Mirrors src/models/discriminator.py:11-82 -- same constructor kwargs (input_nc, ndf, n_layers,
use_actnorm), the same `main` Sequential and therefore the same state-dict names
(`main.0.weight`, `main.3.running_mean`, ...): 4x4 convs (stride 2 ... 2, 1, 1; padding 1) on the
implicit-GEMM kernel, BatchNorm2d fused with the in-place LeakyReLU(0.2) that follows it
(csrc/disc.hip), the first LeakyReLU as its own kernel. The convolutions run in exact fp32 (f32-input MFMA)
by default: see NLayerDiscriminator.__init__.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .encoder_decoder import Conv2d, GroupNorm


class LeakyReLU(nn.Module):
    def __init__(self, negative_slope: float = 0.2, inplace: bool = False):
        super().__init__()
        self.negative_slope = negative_slope

    def forward(self, x):
        return ops.leaky_relu(x, self.negative_slope)


class BatchNorm2d(nn.Module):
    """nn.BatchNorm2d-compatible parameters/buffers; `fuse_leaky` folds the following LeakyReLU."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, affine: bool = True):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self.fuse_slope = -1.0

    def forward(self, x):
        if self.training:
            self.num_batches_tracked.add_(1)
        return ops.batch_norm(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                              self.momentum, self.eps, self.fuse_slope)


class _Fused(nn.Module):
    """LeakyReLU whose work was folded into the preceding BatchNorm (keeps the module index)."""

    def __init__(self, negative_slope: float = 0.2):
        super().__init__()
        self.negative_slope = negative_slope

    def forward(self, x):
        return x


class NLayerDiscriminator(nn.Module):
    def __init__(self, input_nc: int = 3, ndf: int = 64, n_layers: int = 3, use_actnorm: bool = False,
                 exact_fp32: bool = True):
        """exact_fp32: the discriminator's convolutions run on the exact f32-input MFMA whatever the trainer's
        precision (its BatchNorm backward removes the per-channel mean of near-constant hinge gradients, which
        amplifies the 3xBF16 operand rounding of the layer above by ~300x: 3.6e-3 relative on main.0's
        gradient vs 1e-5 in exact fp32; tests/test_gpu_adversarial.py)."""
        super().__init__()
        self.n_layers = n_layers
        self.exact_fp32 = exact_fp32
        kw, padw = 4, 1
        use_bias = not use_actnorm

        def norm(planes):
            return GroupNorm(32, planes, eps=1e-5) if use_actnorm else BatchNorm2d(planes)

        seq = [Conv2d(input_nc, ndf, kw, stride=2, padding=padw, bias=use_bias), LeakyReLU(0.2, True)]
        nf_mult = 1
        for n in range(1, n_layers):
            nf_prev, nf_mult = nf_mult, min(2 ** n, 8)
            seq += [Conv2d(ndf * nf_prev, ndf * nf_mult, kw, stride=2, padding=padw, bias=use_bias),
                    norm(ndf * nf_mult), LeakyReLU(0.2, True)]
        nf_prev, nf_mult = nf_mult, min(2 ** n_layers, 8)
        seq += [Conv2d(ndf * nf_prev, ndf * nf_mult, kw, stride=1, padding=padw, bias=use_bias),
                norm(ndf * nf_mult), LeakyReLU(0.2, True)]
        seq += [Conv2d(ndf * nf_mult, 1, kw, stride=1, padding=padw)]
        # fold each BatchNorm's following LeakyReLU into the BatchNorm kernel
        for i in range(len(seq) - 1):
            if isinstance(seq[i], BatchNorm2d) and isinstance(seq[i + 1], LeakyReLU):
                seq[i].fuse_slope = seq[i + 1].negative_slope
                seq[i + 1] = _Fused(seq[i + 1].negative_slope)
        self.main = nn.Sequential(*seq)

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        with ops.math_scope(2 if self.exact_fp32 else None):
            return self.main(input)
