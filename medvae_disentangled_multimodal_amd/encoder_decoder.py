"""Encoder / Decoder of the conv-VAE on the MI355X kernels.

Module tree, parameter names and constructor kwargs mirror the reference
(src/models/encoder_decoder.py:212-451) so `state_dict`s interchange and `_target_` configs keep
working; parameters are created in the reference's construction order with torch's own
initialisers, so a given `torch.manual_seed` yields the reference's initial weights.
The forward composes the fused HIP ops of `ops.py`:
  ResnetBlock  = GN+SiLU -> conv3x3 -> GN+SiLU(+dropout) -> conv3x3 with the skip add (or the
                 1x1 nin_shortcut output) fused into the second conv's epilogue
  AttnBlock    = GN -> q/k/v 1x1 GEMMs -> attention core -> proj_out GEMM (+x fused)
  Downsample   = stride-2 conv whose zero fill covers the (0,1,0,1) F.pad
  Upsample     = conv whose gather reads the nearest-x2 upsampled image without materialising it
"""
from __future__ import annotations

import itertools
import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .ops import ConvGeom

_seed_counter = itertools.count(1)
_seed_base = [0x5EED_0000_1234]


def set_dropout_seed(seed: int):
    """Seed of the fused (counter-based) dropout masks."""
    global _seed_counter
    _seed_base[0] = int(seed) * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF
    _seed_counter = itertools.count(1)


def _next_seed() -> int:
    return (_seed_base[0] + next(_seed_counter) * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF


class Conv2d(nn.Module):
    """nn.Conv2d-compatible parameters (weight [out, in, k, k], bias [out]) on the HIP conv."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 padding: int = 0, bias: bool = True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (kernel_size, kernel_size)
        self.stride = (stride, stride)
        self.padding = (padding, padding)
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()
        self.geom = ConvGeom(kernel_size, kernel_size, stride, padding, padding, padding, padding)

    def reset_parameters(self):
        # identical to torch.nn.modules.conv._ConvNd.reset_parameters (same RNG consumption)
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.weight.shape[1] * self.weight.shape[2] * self.weight.shape[3]
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, residual=None, geom: Optional[ConvGeom] = None, res_sink=None, x_sink=None,
                gn_stats: bool = False, gn_bias: bool = False, dx_sum=None):
        # gn_stats: the output feeds a Normalize; its statistics come out of the conv's epilogue
        return ops.conv2d(x, self.weight, self.bias, geom or self.geom, residual, res_sink, x_sink, gn_stats, gn_bias,
                          dx_sum)


class GroupNorm(nn.Module):
    """nn.GroupNorm-compatible parameters; forward optionally fuses SiLU and dropout."""

    def __init__(self, num_groups: int, num_channels: int, eps: float = 1e-6, affine: bool = True):
        super().__init__()
        self.num_groups, self.num_channels, self.eps = num_groups, num_channels, eps
        self.weight = nn.Parameter(torch.ones(num_channels))
        self.bias = nn.Parameter(torch.zeros(num_channels))

    def forward(self, x, silu: bool = False, drop_p: float = 0.0, for_conv: bool = False, grad_sink=None,
                conv_dy_only: bool = False):
        seed = _next_seed() if drop_p > 0.0 else 0
        return ops.group_norm(x, self.weight, self.bias, self.num_groups, self.eps, silu, drop_p, seed, for_conv,
                              grad_sink, conv_dy_only)


def Normalize(in_channels: int, num_groups: int = 32) -> GroupNorm:
    # encoder_decoder.py:28-33
    return GroupNorm(min(num_groups, in_channels), in_channels, eps=1e-6, affine=True)


class ResnetBlock(nn.Module):
    def __init__(self, in_channels: int, out_channels: Optional[int] = None, conv_shortcut: bool = False,
                 dropout: float = 0.0, temb_channels: int = 512):
        super().__init__()
        out_channels = in_channels if out_channels is None else out_channels
        self.in_channels, self.out_channels = in_channels, out_channels
        self.use_conv_shortcut = conv_shortcut
        self.norm1 = Normalize(in_channels)
        self.conv1 = Conv2d(in_channels, out_channels, 3, 1, 1)
        if temb_channels > 0:
            self.temb_proj = nn.Linear(temb_channels, out_channels)
        self.norm2 = Normalize(out_channels)
        self.dropout = nn.Dropout(dropout)
        self.conv2 = Conv2d(out_channels, out_channels, 3, 1, 1)
        if in_channels != out_channels:
            if conv_shortcut:
                self.conv_shortcut = Conv2d(in_channels, out_channels, 3, 1, 1)
            else:
                self.nin_shortcut = Conv2d(in_channels, out_channels, 1, 1, 0)

    def forward(self, x, temb=None):
        if temb is not None:
            raise NotImplementedError("timestep embeddings are not used by the VAE (temb_channels=0)")
        # x's two gradient branches (norm1 and the residual / shortcut) are summed inside norm1's backward
        sink = ops.GradSink() if torch.is_grad_enabled() and x.requires_grad else None
        # for_conv = the consuming conv's output channels (bf16-mixed: packed bf16 GroupNorm outputs, ops.group_norm)
        h = self.conv1(self.norm1(x, silu=True, for_conv=self.out_channels, grad_sink=sink), gn_stats=True)
        p = self.dropout.p if self.training else 0.0
        # (conv1's output has no other consumer: its gradient is norm2's dx alone -- conv_dy_only)
        h = self.norm2(h, silu=True, drop_p=p, for_conv=self.out_channels, conv_dy_only=True)
        if self.in_channels != self.out_channels:
            sc = self.conv_shortcut if self.use_conv_shortcut else self.nin_shortcut
            return self.conv2(h, residual=sc(x, x_sink=sink), gn_stats=True)
        return self.conv2(h, residual=x, res_sink=sink, gn_stats=True)


class AttnBlock(nn.Module):
    def __init__(self, in_channels: int):
        super().__init__()
        self.in_channels = in_channels
        self.norm = Normalize(in_channels)
        self.q = Conv2d(in_channels, in_channels, 1)
        self.k = Conv2d(in_channels, in_channels, 1)
        self.v = Conv2d(in_channels, in_channels, 1)
        self.proj_out = Conv2d(in_channels, in_channels, 1)

    def forward(self, x):
        sink = ops.GradSink() if torch.is_grad_enabled() and x.requires_grad else None
        h = self.norm(x, grad_sink=sink)
        acc = ops.DxSum(3) if torch.is_grad_enabled() and x.requires_grad else None  # (h's gradient: one buffer)
        o = ops.attention_core(self.q(h, dx_sum=acc), self.k(h, dx_sum=acc), self.v(h, dx_sum=acc))
        return self.proj_out(o, residual=x, res_sink=sink)


def make_attn(in_channels: int, attn_type: str = "vanilla") -> nn.Module:
    if attn_type == "vanilla":
        return AttnBlock(in_channels)
    raise NotImplementedError(f"attention type {attn_type!r} is not on the MI355X path (only 'vanilla')")


class Downsample(nn.Module):
    def __init__(self, in_channels: int, with_conv: bool = True):
        super().__init__()
        if not with_conv:
            raise NotImplementedError("avg-pool Downsample is not used by the reference models")
        self.with_conv = True
        self.conv = Conv2d(in_channels, in_channels, 3, 2, 0)
        # pad (left 0, right 1, top 0, bottom 1) then 3x3 stride 2 valid (encoder_decoder.py:184-188)
        self.geom = ConvGeom(3, 3, 2, 0, 0, 1, 1)

    def forward(self, x):
        return self.conv(x, geom=self.geom, gn_stats=True)


class Upsample(nn.Module):
    def __init__(self, in_channels: int, with_conv: bool = True):
        super().__init__()
        if not with_conv:
            raise NotImplementedError("conv-less Upsample is not used by the reference models")
        self.with_conv = True
        self.conv = Conv2d(in_channels, in_channels, 3, 1, 1)
        self.geom = ConvGeom(3, 3, 1, 1, 1, 1, 1, upsample=True)

    def forward(self, x):
        # (the output feeds the next level's ResnetBlock Normalize: gn_bias lets its backward give the bias gradient)
        return self.conv(x, geom=self.geom, gn_bias=True)


class Encoder(nn.Module):
    def __init__(self, *, ch: int, out_ch: int, ch_mult: Tuple[int, ...] = (1, 2, 4, 8), num_res_blocks: int,
                 attn_resolutions: List[int], dropout: float = 0.0, resamp_with_conv: bool = True,
                 in_channels: int, resolution: int, z_channels: int, double_z: bool = True,
                 use_linear_attn: bool = False, attn_type: str = "vanilla", **ignore_kwargs):
        super().__init__()
        if use_linear_attn:
            attn_type = "linear"
        self.ch, self.temb_ch = ch, 0
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.resolution, self.in_channels = resolution, in_channels
        self.conv_in = Conv2d(in_channels, ch, 3, 1, 1)
        curr_res = resolution
        in_ch_mult = (1,) + tuple(ch_mult)
        self.in_ch_mult = in_ch_mult
        self.down = nn.ModuleList()
        block_in = ch
        for i_level in range(self.num_resolutions):
            block, attn = nn.ModuleList(), nn.ModuleList()
            block_in = ch * in_ch_mult[i_level]
            block_out = ch * ch_mult[i_level]
            for _ in range(num_res_blocks):
                block.append(ResnetBlock(block_in, block_out, dropout=dropout, temb_channels=0))
                block_in = block_out
                if curr_res in attn_resolutions:
                    attn.append(make_attn(block_in, attn_type))
            down = nn.Module()
            down.block, down.attn = block, attn
            if i_level != self.num_resolutions - 1:
                down.downsample = Downsample(block_in, resamp_with_conv)
                curr_res //= 2
            self.down.append(down)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in, dropout=dropout, temb_channels=0)
        self.mid.attn_1 = make_attn(block_in, attn_type)
        self.mid.block_2 = ResnetBlock(block_in, block_in, dropout=dropout, temb_channels=0)
        self.norm_out = Normalize(block_in)
        self.conv_out = Conv2d(block_in, 2 * z_channels if double_z else z_channels, 3, 1, 1)

    def forward(self, x):
        h = self.conv_in(x, gn_stats=True)
        for i_level in range(self.num_resolutions):
            lvl = self.down[i_level]
            for i_block in range(self.num_res_blocks):
                h = lvl.block[i_block](h)
                if len(lvl.attn) > 0:
                    h = lvl.attn[i_block](h)
            if i_level != self.num_resolutions - 1:
                h = lvl.downsample(h)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        return self.conv_out(self.norm_out(h, silu=True, for_conv=self.conv_out.out_channels))


class Decoder(nn.Module):
    def __init__(self, *, ch: int, out_ch: int, ch_mult: Tuple[int, ...] = (1, 2, 4, 8), num_res_blocks: int,
                 attn_resolutions: List[int], dropout: float = 0.0, resamp_with_conv: bool = True,
                 in_channels: int, resolution: int, z_channels: int, give_pre_end: bool = False,
                 tanh_out: bool = False, use_linear_attn: bool = False, attn_type: str = "vanilla",
                 **ignorekwargs):
        super().__init__()
        if use_linear_attn:
            attn_type = "linear"
        self.ch, self.temb_ch = ch, 0
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.resolution, self.in_channels = resolution, in_channels
        self.give_pre_end, self.tanh_out = give_pre_end, tanh_out
        block_in = ch * ch_mult[self.num_resolutions - 1]
        curr_res = resolution // 2 ** (self.num_resolutions - 1)
        self.z_shape = (1, z_channels, curr_res, curr_res)
        self.conv_in = Conv2d(z_channels, block_in, 3, 1, 1)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in, dropout=dropout, temb_channels=0)
        self.mid.attn_1 = make_attn(block_in, attn_type)
        self.mid.block_2 = ResnetBlock(block_in, block_in, dropout=dropout, temb_channels=0)
        self.up = nn.ModuleList()
        for i_level in reversed(range(self.num_resolutions)):
            block, attn = nn.ModuleList(), nn.ModuleList()
            block_out = ch * ch_mult[i_level]
            for _ in range(num_res_blocks + 1):
                block.append(ResnetBlock(block_in, block_out, dropout=dropout, temb_channels=0))
                block_in = block_out
                if curr_res in attn_resolutions:
                    attn.append(make_attn(block_in, attn_type))
            up = nn.Module()
            up.block, up.attn = block, attn
            if i_level != 0:
                up.upsample = Upsample(block_in, resamp_with_conv)
                curr_res *= 2
            self.up.insert(0, up)
        self.norm_out = Normalize(block_in)
        self.conv_out = Conv2d(block_in, out_ch, 3, 1, 1)

    def forward(self, z):
        h = self.conv_in(z, gn_stats=True)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        for i_level in reversed(range(self.num_resolutions)):
            lvl = self.up[i_level]
            for i_block in range(self.num_res_blocks + 1):
                h = lvl.block[i_block](h)
                if len(lvl.attn) > 0:
                    h = lvl.attn[i_block](h)
            if i_level != 0:
                h = lvl.upsample(h)
        if self.give_pre_end:
            return h
        h = self.conv_out(self.norm_out(h, silu=True, for_conv=self.conv_out.out_channels))
        if self.tanh_out:
            h = torch.tanh(h)
        return h
