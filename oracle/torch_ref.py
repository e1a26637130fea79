"""CPU oracle: a functional fp32 restatement of the reference conv-VAE training step.

TEST INFRASTRUCTURE ONLY. Nothing in the product package imports this module; only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use it, and only as the checker /
CPU baseline. The product path (medvae_disentangled_multimodal_amd) runs the HIP kernels and fails
loudly if they are missing.

Pinned against the reference: tests/test_oracle_golden.py checks this file against the golden
vectors that tests/golden/make_golden.py produced by running the reference's own `src.models`
(parsakzr/medvae-disentangled-multimodal @ 2025-08-24) in the build container, and against the
SURVEY.md section 8(c) known-answer anchor.

Layout: logical NCHW fp32 on the CPU (what the reference runs). Parameters live in a flat dict keyed
by the reference's state-dict names (e.g. ``encoder.down.0.block.1.norm2.weight``) so the same
dict loads into the reference, the oracle and the HIP path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# src/models/disentangled_conditional_vae.py:112-122 (modality index -> channel count)
MODALITY_CHANNELS = {0: 1, 1: 3, 2: 3, 3: 1, 4: 3}


# --------------------------------------------------------------------------------------------
# architecture description (names/shapes follow the reference's module tree)
# --------------------------------------------------------------------------------------------
@dataclass
class Arch:
    cls: str
    input_channels: int
    latent_dim: int
    ch: int
    ch_mult: Tuple[int, ...]
    num_res_blocks: int
    attn_resolutions: Tuple[int, ...]
    resolution: int
    dropout: float = 0.0
    double_z: bool = True
    # ConditionalVAE
    condition_dim: int = 12
    # DisentangledConditionalVAE
    num_modalities: int = 5
    shared_latent_dim: int = 8
    modality_latent_dim: int = 8
    extra: dict = field(default_factory=dict)

    @property
    def levels(self) -> int:
        return len(self.ch_mult)

    @property
    def enc_res(self) -> int:
        # base_vae.py:37
        return self.resolution // (2 ** (self.levels - 1))


def make_arch(cls: str, kwargs: dict) -> Arch:
    kw = dict(kwargs)
    if cls == "DisentangledConditionalVAE":
        # disentangled_conditional_vae.py:48-74: latent = shared + modality, input = max channels
        lat = kw.get("shared_latent_dim", 8) + kw.get("modality_latent_dim", 8)
        return Arch(cls=cls, input_channels=max(MODALITY_CHANNELS.values()), latent_dim=lat,
                    ch=kw.get("hidden_channels", 128), ch_mult=tuple(kw.get("ch_mult", (1, 2, 4, 8))),
                    num_res_blocks=kw.get("num_res_blocks", 2),
                    attn_resolutions=tuple(kw.get("attn_resolutions", [16])),
                    resolution=kw.get("resolution", 28), dropout=kw.get("dropout", 0.0),
                    num_modalities=kw.get("num_modalities", 5),
                    shared_latent_dim=kw.get("shared_latent_dim", 8),
                    modality_latent_dim=kw.get("modality_latent_dim", 8))
    cond_dim = 12
    if cls == "ConditionalVAE":
        mods = kw.get("modalities")
        cond_dim = kw.get("condition_dim") or (len(mods) if mods else 12)
    return Arch(cls=cls, input_channels=kw.get("input_channels", 1),
                latent_dim=kw.get("latent_dim", 128), ch=kw.get("hidden_channels", 128),
                ch_mult=tuple(kw.get("ch_mult", (1, 2, 4, 8))),
                num_res_blocks=kw.get("num_res_blocks", 2),
                attn_resolutions=tuple(kw.get("attn_resolutions", [16])),
                resolution=kw.get("resolution", 224), dropout=kw.get("dropout", 0.0),
                double_z=kw.get("double_z", True), condition_dim=cond_dim)


def _conv_shapes(name, cin, cout, k):
    return [(f"{name}.weight", (cout, cin, k, k)), (f"{name}.bias", (cout,))]


def _gn_shapes(name, c):
    return [(f"{name}.weight", (c,)), (f"{name}.bias", (c,))]


def _resblock_shapes(p, cin, cout):
    s = _gn_shapes(f"{p}.norm1", cin) + _conv_shapes(f"{p}.conv1", cin, cout, 3)
    s += _gn_shapes(f"{p}.norm2", cout) + _conv_shapes(f"{p}.conv2", cout, cout, 3)
    if cin != cout:
        s += _conv_shapes(f"{p}.nin_shortcut", cin, cout, 1)
    return s


def _attn_shapes(p, c):
    s = _gn_shapes(f"{p}.norm", c)
    for n in ("q", "k", "v", "proj_out"):
        s += _conv_shapes(f"{p}.{n}", c, c, 1)
    return s


def param_shapes(a: Arch) -> List[Tuple[str, Tuple[int, ...]]]:
    """State-dict names and shapes in the reference's registration order
    (encoder_decoder.py:212-451, base_vae.py:14-70, conditional_vae.py:59-78,
    disentangled_conditional_vae.py:76-109)."""
    s: List[Tuple[str, Tuple[int, ...]]] = []
    cin0 = a.input_channels * 2 if a.cls == "ConditionalVAE" else a.input_channels
    # ---- encoder
    s += _conv_shapes("encoder.conv_in", cin0, a.ch, 3)
    res = a.resolution
    in_mult = (1,) + a.ch_mult
    bin_ = a.ch
    for i in range(a.levels):
        bin_ = a.ch * in_mult[i]
        bout = a.ch * a.ch_mult[i]
        for j in range(a.num_res_blocks):
            s += _resblock_shapes(f"encoder.down.{i}.block.{j}", bin_, bout)
            bin_ = bout
        if res in a.attn_resolutions:
            for j in range(a.num_res_blocks):
                s += _attn_shapes(f"encoder.down.{i}.attn.{j}", bin_)
        if i != a.levels - 1:
            s += _conv_shapes(f"encoder.down.{i}.downsample.conv", bin_, bin_, 3)
            res //= 2
    s += _resblock_shapes("encoder.mid.block_1", bin_, bin_)
    s += _attn_shapes("encoder.mid.attn_1", bin_)
    s += _resblock_shapes("encoder.mid.block_2", bin_, bin_)
    s += _gn_shapes("encoder.norm_out", bin_)
    zc = 2 * a.latent_dim if a.double_z else a.latent_dim
    s += _conv_shapes("encoder.conv_out", bin_, zc, 3)
    # ---- decoder
    bin_ = a.ch * a.ch_mult[-1]
    res = a.resolution // 2 ** (a.levels - 1)
    s += _conv_shapes("decoder.conv_in", a.latent_dim, bin_, 3)
    s += _resblock_shapes("decoder.mid.block_1", bin_, bin_)
    s += _attn_shapes("decoder.mid.attn_1", bin_)
    s += _resblock_shapes("decoder.mid.block_2", bin_, bin_)
    up: Dict[int, list] = {}
    for i in reversed(range(a.levels)):
        lst = []
        bout = a.ch * a.ch_mult[i]
        for j in range(a.num_res_blocks + 1):
            lst += _resblock_shapes(f"decoder.up.{i}.block.{j}", bin_, bout)
            bin_ = bout
        if res in a.attn_resolutions:
            for j in range(a.num_res_blocks + 1):
                lst += _attn_shapes(f"decoder.up.{i}.attn.{j}", bin_)
        if i != 0:
            lst += _conv_shapes(f"decoder.up.{i}.upsample.conv", bin_, bin_, 3)
            res *= 2
        up[i] = lst
    for i in range(a.levels):  # self.up.insert(0, ...) -> state_dict lists level 0 first
        s += up[i]
    s += _gn_shapes("decoder.norm_out", bin_)
    s += _conv_shapes("decoder.conv_out", bin_, a.input_channels, 3)
    # ---- heads
    if a.cls == "ConditionalVAE":
        s += [("condition_proj.0.weight", (a.input_channels * 64, a.condition_dim)),
              ("condition_proj.0.bias", (a.input_channels * 64,))]
    if a.cls == "DisentangledConditionalVAE":
        mx = max(MODALITY_CHANNELS.values())
        for m, c in MODALITY_CHANNELS.items():
            if c != mx:
                s += _conv_shapes(f"modality_input_projectors.{m}", c, mx, 1)
        for m, c in MODALITY_CHANNELS.items():
            if c != mx:
                s += _conv_shapes(f"modality_output_projectors.{m}", mx, c, 1)
        s += [("modality_embedding.weight", (a.num_modalities, 64))]
        for m in range(a.num_modalities):
            s += _conv_shapes(f"modality_decoders.{m}.0", mx, mx, 3)
            s += _conv_shapes(f"modality_decoders.{m}.2", mx, mx, 3)
    return s


# --------------------------------------------------------------------------------------------
# forward restatement
# --------------------------------------------------------------------------------------------
def silu(x: Tensor) -> Tensor:
    # encoder_decoder.py:13-15 (x * sigmoid(x))
    return x * torch.sigmoid(x)


def gn(P, name, x):
    # encoder_decoder.py:28-33: GroupNorm(min(32, C), C, eps=1e-6, affine=True)
    c = x.shape[1]
    return F.group_norm(x, min(32, c), P[f"{name}.weight"], P[f"{name}.bias"], eps=1e-6)


def conv(P, name, x, stride=1, padding=None):
    w = P[f"{name}.weight"]
    k = w.shape[-1]
    if padding is None:
        padding = k // 2
    return F.conv2d(x, w, P[f"{name}.bias"], stride=stride, padding=padding)


def _dropout(x, p, train, gen):
    if not train or p == 0.0:
        return x
    keep = (torch.rand(x.shape, generator=gen) >= p).to(x.dtype)
    return x * keep / (1.0 - p)


def resblock(P, p, x, dropout=0.0, train=True, gen=None):
    # encoder_decoder.py:148-170
    h = conv(P, f"{p}.conv1", silu(gn(P, f"{p}.norm1", x)))
    h = _dropout(silu(gn(P, f"{p}.norm2", h)), dropout, train, gen)
    h = conv(P, f"{p}.conv2", h)
    if f"{p}.nin_shortcut.weight" in P:
        x = conv(P, f"{p}.nin_shortcut", x)
    return x + h


def attnblock(P, p, x):
    # encoder_decoder.py:83-107: softmax over keys of q.k / sqrt(C), out = x + proj(v @ attn^T)
    h = gn(P, f"{p}.norm", x)
    q = conv(P, f"{p}.q", h)
    k = conv(P, f"{p}.k", h)
    v = conv(P, f"{p}.v", h)
    b, c, hh, ww = q.shape
    n = hh * ww
    qt = q.reshape(b, c, n).transpose(1, 2)          # [b, n, c]
    s = torch.matmul(qt, k.reshape(b, c, n)) * (c ** -0.5)   # [b, nq, nk]
    a = torch.softmax(s, dim=2)
    o = torch.matmul(v.reshape(b, c, n), a.transpose(1, 2))  # [b, c, nq]
    return x + conv(P, f"{p}.proj_out", o.reshape(b, c, hh, ww))


def downsample(P, p, x):
    # encoder_decoder.py:184-188: pad right/bottom by one, 3x3 stride-2 valid conv
    return conv(P, f"{p}.conv", F.pad(x, (0, 1, 0, 1)), stride=2, padding=0)


def upsample(P, p, x):
    # encoder_decoder.py:205-209: nearest x2 then 3x3 conv
    return conv(P, f"{p}.conv", F.interpolate(x, scale_factor=2.0, mode="nearest"))


def encoder(P, a: Arch, x, train=True, gen=None):
    # encoder_decoder.py:303-328
    h = conv(P, "encoder.conv_in", x)
    res = a.resolution
    for i in range(a.levels):
        for j in range(a.num_res_blocks):
            h = resblock(P, f"encoder.down.{i}.block.{j}", h, a.dropout, train, gen)
            if res in a.attn_resolutions:
                h = attnblock(P, f"encoder.down.{i}.attn.{j}", h)
        if i != a.levels - 1:
            h = downsample(P, f"encoder.down.{i}.downsample", h)
            res //= 2
    h = resblock(P, "encoder.mid.block_1", h, a.dropout, train, gen)
    h = attnblock(P, "encoder.mid.attn_1", h)
    h = resblock(P, "encoder.mid.block_2", h, a.dropout, train, gen)
    return conv(P, "encoder.conv_out", silu(gn(P, "encoder.norm_out", h)))


def decoder(P, a: Arch, z, train=True, gen=None):
    # encoder_decoder.py:421-451
    h = conv(P, "decoder.conv_in", z)
    h = resblock(P, "decoder.mid.block_1", h, a.dropout, train, gen)
    h = attnblock(P, "decoder.mid.attn_1", h)
    h = resblock(P, "decoder.mid.block_2", h, a.dropout, train, gen)
    res = a.enc_res
    for i in reversed(range(a.levels)):
        for j in range(a.num_res_blocks + 1):
            h = resblock(P, f"decoder.up.{i}.block.{j}", h, a.dropout, train, gen)
            if res in a.attn_resolutions:
                h = attnblock(P, f"decoder.up.{i}.attn.{j}", h)
        if i != 0:
            h = upsample(P, f"decoder.up.{i}.upsample", h)
            res *= 2
    return conv(P, "decoder.conv_out", silu(gn(P, "decoder.norm_out", h)))


def condition_map(P, a: Arch, onehot, H, W):
    # conditional_vae.py:107-119: Linear -> ReLU -> [C, 8, 8] -> bilinear (align_corners=False)
    m = F.relu(F.linear(onehot, P["condition_proj.0.weight"], P["condition_proj.0.bias"]))
    m = m.reshape(onehot.shape[0], a.input_channels, 8, 8)
    return F.interpolate(m, size=(H, W), mode="bilinear", align_corners=False)


def _fma32(a, b, c):
    """Correctly rounded float32 fma(a, b, c) in numpy: the float32 product is exact in float64, TwoSum gives the
    exact error of the float64 sum, and a float64 sum lying exactly on a float32 rounding midpoint is resolved
    by that error's sign (no double rounding)."""
    import numpy as np
    f32, f64 = np.float32, np.float64
    a, b, c = (np.asarray(v, f32).astype(f64) for v in (a, b, c))
    p = a * b
    s = p + c
    bb = s - p
    e = (p - (s - bb)) + (c - bb)
    r = s.astype(f32)
    bits = np.ascontiguousarray(s).view(np.uint64)
    tie = ((bits & np.uint64((1 << 29) - 1)) == np.uint64(1 << 28)) & (e != 0)
    if np.any(tie):
        lo = np.where(s.astype(f32).astype(f64) > s, np.nextafter(s.astype(f32), f32(-np.inf)), s.astype(f32))
        hi = np.nextafter(lo, f32(np.inf))
        r = np.where(tie, np.where(e > 0, hi, lo), r)
    return r.astype(f32)


def _lerp_exact(in_size: int, out_size: int):
    """UpSample.h compute_source_index_and_lambda (align_corners=False) in float32, the source index taken with
    one fma as torch's compiled CPU kernel does: src = fma(in/out, dst + 0.5, -0.5)."""
    import numpy as np
    f32 = np.float32
    d = np.arange(out_size, dtype=f32)
    if in_size == out_size:
        i = np.arange(out_size)
        return i, i, np.ones(out_size, f32), np.zeros(out_size, f32)
    scale = f32(f32(in_size) / f32(out_size))
    src = _fma32(np.full_like(d, scale), (d + f32(0.5)).astype(f32), np.full_like(d, f32(-0.5)))
    src = np.where(src < 0, f32(0), src).astype(f32)
    i0 = np.minimum(np.floor(src).astype(np.int64), in_size - 1)
    l1 = np.clip((src - i0.astype(f32)).astype(f32), f32(0), f32(1)).astype(f32)
    i1 = np.where(i0 < in_size - 1, i0 + 1, i0)
    return i0, i1, (f32(1) - l1).astype(f32), l1


def condition_map_exact(weight, bias, cond, channels: int, H: int, W: int):
    """Bit-exact float32 restatement of ConditionalVAE.create_condition_map on the reference's CPU path
    (src/models/conditional_vae.py:65-69 Linear + ReLU + Unflatten(C, 8, 8), :107-127 F.interpolate bilinear,
    align_corners=False). Returns (projection [B, C*64] before the ReLU, map [B, C, H, W]) as numpy float32.
    The projection is the fma chain over the condition entries plus the bias (exactly W[:, idx] + b for a one-hot
    row, torch's addmm result); the interpolation is torch's CPU bilinear kernel for H + W <= 128 (the path it
    takes for these sizes): corner weights w00 = hl0*wl0, ... and fma(w11, v11, fma(w10, v10, fma(w00, v00,
    w01*v01))). Pinned bitwise against torch and the reference's own condition maps (tests/test_condition_cpu.py)."""
    import numpy as np
    f32 = np.float32
    w = np.asarray(weight, f32)
    b = np.asarray(bias, f32)
    c = np.asarray(cond, f32)
    B, K = c.shape
    acc = np.zeros((B, w.shape[0]), f32)
    for j in range(K):
        acc = _fma32(np.broadcast_to(c[:, j:j + 1], acc.shape), np.broadcast_to(w[None, :, j], acc.shape), acc)
    pre = (acc + b[None, :]).astype(f32)
    m = np.where(np.isnan(pre), pre, np.maximum(pre, f32(0))).reshape(B, channels, 8, 8)
    h0, h1, hl0, hl1 = _lerp_exact(8, H)
    w0, w1, wl0, wl1 = _lerp_exact(8, W)
    v00, v01 = m[:, :, h0][:, :, :, w0], m[:, :, h0][:, :, :, w1]
    v10, v11 = m[:, :, h1][:, :, :, w0], m[:, :, h1][:, :, :, w1]
    shp = v00.shape
    w00 = np.broadcast_to((hl0[:, None] * wl0[None, :]).astype(f32), shp)
    w01 = np.broadcast_to((hl0[:, None] * wl1[None, :]).astype(f32), shp)
    w10 = np.broadcast_to((hl1[:, None] * wl0[None, :]).astype(f32), shp)
    w11 = np.broadcast_to((hl1[:, None] * wl1[None, :]).astype(f32), shp)
    out = _fma32(w11, v11, _fma32(w10, v10, _fma32(w00, v00, (w01 * v01).astype(f32))))
    return pre, out


def clamp_modality(idx: Tensor, n: int) -> Tensor:
    # disentangled_conditional_vae.py:142-146 and :258-265 (out-of-range -> last modality)
    return torch.where(idx >= n, torch.full_like(idx, n - 1), idx)


def dis_route_in(P, a: Arch, x, idx):
    # disentangled_conditional_vae.py:124-193 (batched restatement of the per-sample loop)
    x = torch.nan_to_num(x, nan=0.0, posinf=float("inf"), neginf=float("-inf"))
    idx = clamp_modality(idx, len(MODALITY_CHANNELS))
    outs = []
    for b in range(x.shape[0]):
        m = int(idx[b])
        c = MODALITY_CHANNELS[m]
        s = x[b:b + 1, :c] if x.shape[1] > c else x[b:b + 1]
        if f"modality_input_projectors.{m}.weight" in P:
            s = conv(P, f"modality_input_projectors.{m}", s)
            s = torch.where(torch.isnan(s), torch.zeros_like(s), s)
        outs.append(s)
    return torch.cat(outs, 0)


def dis_route_out(P, a: Arch, rec, idx):
    # disentangled_conditional_vae.py:241-303
    idx = clamp_modality(idx, a.num_modalities)
    outs = []
    for b in range(rec.shape[0]):
        m = int(idx[b])
        s = rec[b:b + 1]
        s = conv(P, f"modality_decoders.{m}.2", F.relu(conv(P, f"modality_decoders.{m}.0", s)))
        if f"modality_output_projectors.{m}.weight" in P:
            s = conv(P, f"modality_output_projectors.{m}", s)
        outs.append(s)
    cmax = max(o.shape[1] for o in outs)
    outs = [torch.cat([o, o.new_zeros(1, cmax - o.shape[1], *o.shape[2:])], 1)
            if o.shape[1] < cmax else o for o in outs]
    return torch.cat(outs, 0)


def partition_latent(a: Arch, z):
    # disentangled_conditional_vae.py:195-206 (NCHW flatten order)
    f = z.reshape(z.shape[0], -1)
    return f[:, :a.shared_latent_dim], f[:, a.shared_latent_dim:a.shared_latent_dim + a.modality_latent_dim]


def separation_loss(a: Arch, z, idx):
    # disentangled_conditional_vae.py:305-349 (non-MPS branch)
    _, zm = partition_latent(a, z)
    cents = [zm[idx == m].mean(0) for m in torch.unique(idx)]
    if len(cents) < 2:
        return z.new_zeros(())
    d = torch.pdist(torch.stack(cents), p=2)
    return -d.mean()


def contrastive_loss(a: Arch, z, idx, temperature=0.1):
    # disentangled_conditional_vae.py:351-386
    _, zm = partition_latent(a, z)
    zn = F.normalize(zm, p=2, dim=1)
    e = torch.exp(zn @ zn.t() / temperature)
    pos = (idx[None, :] == idx[:, None])
    pos.fill_diagonal_(False)
    ps = (e * pos.float()).sum(1)
    tot = e.sum(1) - torch.diagonal(e)
    l = -torch.log(ps / tot + 1e-8)
    l = l[ps > 0]
    return l.mean() if l.numel() > 0 else z.new_zeros(())


def forward(P, a: Arch, x, cond=None, eps=None, train=True, gen=None):
    """Model forward (base_vae.py:89-118, conditional_vae.py:134-164,
    disentangled_conditional_vae.py:388-454). `eps` replaces randn_like in reparameterize."""
    out = {}
    if a.cls == "ConditionalVAE":
        xin = torch.cat([x, condition_map(P, a, cond, x.shape[2], x.shape[3])], 1)
    elif a.cls == "DisentangledConditionalVAE":
        xin = dis_route_in(P, a, x, cond)
    else:
        xin = x
    h = encoder(P, a, xin, train, gen)
    mean, logvar = torch.chunk(h, 2, dim=1)
    if a.cls == "DisentangledConditionalVAE":
        mean = torch.nan_to_num(mean, nan=0.0, posinf=float("inf"), neginf=float("-inf"))
        logvar = torch.nan_to_num(logvar, nan=0.0, posinf=float("inf"), neginf=float("-inf"))
        logvar = torch.clamp(logvar, -10.0, 10.0)
        mean = torch.clamp(mean, -10.0, 10.0)
    if eps is None:
        eps = torch.randn(mean.shape, generator=gen)
    z = mean + eps * torch.exp(0.5 * logvar)   # base_vae.py:83-87
    rec = decoder(P, a, z, train, gen)
    if a.cls == "DisentangledConditionalVAE":
        rec = dis_route_out(P, a, rec, cond)
        out["separation_loss"] = separation_loss(a, z, cond)
        out["contrastive_loss"] = contrastive_loss(a, z, cond)
        out["mu"] = mean
    out.update(reconstruction=rec, mean=mean, logvar=logvar, z=z)
    return out


def vae_loss(out, x, recon_weight=1.0, kl_weight=1.0, recon_loss_type="mse"):
    # vae_losses.py:37-64; KL(N(mu, e^{lv/2}) || N(0,1)) as torch.distributions computes it
    rec = out["reconstruction"]
    if recon_loss_type == "mse":
        r = F.mse_loss(rec, x)
    elif recon_loss_type == "l1":
        r = F.l1_loss(rec, x)
    else:
        r = F.binary_cross_entropy_with_logits(rec, x)
    s = torch.exp(0.5 * out["logvar"])
    vr = s * s
    kl = (0.5 * (vr + out["mean"] ** 2 - 1 - torch.log(vr))).mean()
    return {"loss": recon_weight * r + kl_weight * kl, "recon_loss": r, "kl_loss": kl}


def _finite_or_zero(v):
    return v if bool(torch.isfinite(v).all()) else torch.zeros_like(v)


def disentangled_loss(out, x, recon_weight=1.0, kl_weight=1.0, separation_weight=0.1,
                      contrastive_weight=0.05, recon_loss_type="mse"):
    # disentangled_conditional_vae.py:510-573
    rec = out["reconstruction"]
    r = F.mse_loss(rec, x) if recon_loss_type == "mse" else F.l1_loss(rec, x)
    mu, lv = out["mu"], out["logvar"]
    kl = -0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp()) / x.numel()
    r, kl = _finite_or_zero(r), _finite_or_zero(kl)
    sep = _finite_or_zero(out["separation_loss"])
    con = _finite_or_zero(out["contrastive_loss"])
    tot = recon_weight * r + kl_weight * kl + separation_weight * sep + contrastive_weight * con
    if not bool(torch.isfinite(tot).all()):
        tot = torch.full_like(tot, 1e6)
    return {"loss": tot, "recon_loss": r, "kl_loss": kl, "separation_loss": sep,
            "contrastive_loss": con}


# --------------------------------------------------------------------------------------------
# optimizer step restatement (torch.optim.Adam/AdamW single-tensor path, clip_grad_norm_)
# --------------------------------------------------------------------------------------------
def clip_grads(grads: Dict[str, Tensor], max_norm: float) -> Tensor:
    norms = torch.stack([torch.linalg.vector_norm(g, 2) for g in grads.values()])
    total = torch.linalg.vector_norm(norms, 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads.values():
        g.mul_(coef)
    return total


def adam_step(p, g, m, v, step, lr, betas, eps, wd, decoupled):
    b1, b2 = betas
    if decoupled:
        p.mul_(1 - lr * wd)
    elif wd != 0:
        g = g.add(p, alpha=wd)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-(lr / bc1))


def train_step(P: Dict[str, Tensor], a: Arch, x, cond, eps, loss_cfg: dict, opt_cfg: dict,
               clip: float, state: Optional[dict] = None, train=True, gen=None):
    """One training step of VAELightningModule (lightning_module.py:98-218, 390-477):
    forward -> loss -> backward -> zero non-finite grads -> clip -> Adam/AdamW."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    out = forward(leaves, a, x, cond, eps, train, gen)
    if loss_cfg.get("type", "vae") == "disentangled_vae":
        ld = disentangled_loss(out, x, loss_cfg.get("recon_weight", 1.0), loss_cfg.get("kl_weight", 1.0),
                               loss_cfg.get("separation_weight", 0.1),
                               loss_cfg.get("contrastive_weight", 0.05),
                               loss_cfg.get("recon_loss_type", "mse"))
    elif loss_cfg.get("type") == "lpips_discriminator":
        # LPIPSWithDiscriminator generator objective before discriminator_iter_start (vae_losses.py:274-323):
        # perceptual_factor * LPIPS(x, rec).mean() + kl_factor * KL.sum() / B (closed-form KL)
        W = loss_cfg["lpips_weights"]
        lp = (lpips_vgg if loss_cfg.get("lpips_net", "alex") == "vgg" else lpips_alex)(W, x, out["reconstruction"])
        mu, lv = out["mean"], out["logvar"]
        kl = -0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp()) / x.shape[0]
        p = lp.mean()
        ld = {"loss": loss_cfg.get("perceptual_factor", 1.0) * p + loss_cfg.get("kl_factor", 1.0) * kl,
              "p_loss": p, "kl_loss": kl}
    else:
        ld = vae_loss(out, x, loss_cfg.get("recon_weight", 1.0), loss_cfg.get("kl_weight", 1.0),
                      loss_cfg.get("recon_loss_type", "mse"))
    loss = ld["loss"]
    if not bool(torch.isfinite(loss)):
        loss = torch.full_like(loss, 1e6)
    loss.backward()
    grads = {k: t.grad.clone() for k, t in leaves.items() if t.grad is not None}
    for k, g in grads.items():
        if not bool(torch.isfinite(g).all()):
            g.zero_()
    raw = {k: g.clone() for k, g in grads.items()}
    total = clip_grads(grads, clip) if clip and clip > 0 else None
    state = state if state is not None else {}
    newP = {k: v.detach().clone() for k, v in P.items()}
    decoupled = opt_cfg["type"] == "adamw"
    wd = opt_cfg.get("weight_decay", 1e-4 if decoupled else 0.0)
    for k, g in grads.items():
        st = state.setdefault(k, {"step": 0, "m": torch.zeros_like(g), "v": torch.zeros_like(g)})
        st["step"] += 1
        adam_step(newP[k], g, st["m"], st["v"], st["step"], opt_cfg["lr"],
                  tuple(opt_cfg.get("betas", (0.9, 0.999))), 1e-8, wd, decoupled)
    return {"out": out, "loss": ld, "grads": raw, "clipped": grads, "total_norm": total,
            "params": newP, "state": state}


# --------------------------------------------------------------------------------------------
# LPIPS (net="alex"): src/losses/vae_losses.py:67-94 wraps the third-party `lpips` 0.1.4
# (uv.lock:1585, not installed here). Restated from that package's published algorithm:
#   lpips.LPIPS.forward (version 0.1): ScalingLayer -> alexnet slices relu1..relu5 ->
#   normalize_tensor (x / (sqrt(sum_c x^2) + 1e-10)) -> (f0 - f1)^2 -> NetLinLayer (1x1, no bias;
#   its Dropout is inactive in eval mode) -> spatial_average -> sum over layers.
#   AlexNet features = torchvision.models.alexnet().features[0:12].
# Parity against the real package is UNPINNED (no weights / package offline).
# --------------------------------------------------------------------------------------------
LPIPS_SHIFT = (-0.030, -0.088, -0.188)
LPIPS_SCALE = (0.458, 0.448, 0.450)


def lpips_alex(W: Dict[str, Tensor], in0: Tensor, in1: Tensor, pre=(2.0, -1.0)) -> Tensor:
    """W: conv{1..5}.weight/.bias and lins.{0..4} (the HIP module's state-dict names)."""
    shift = torch.tensor(LPIPS_SHIFT, dtype=in0.dtype).view(1, 3, 1, 1)
    scale = torch.tensor(LPIPS_SCALE, dtype=in0.dtype).view(1, 3, 1, 1)

    def feats(x):
        x = (pre[0] * x + pre[1] - shift) / scale
        out = []
        h = F.relu(F.conv2d(x, W["conv1.weight"], W["conv1.bias"], stride=4, padding=2))
        out.append(h)
        h = F.relu(F.conv2d(F.max_pool2d(h, 3, 2), W["conv2.weight"], W["conv2.bias"], padding=2))
        out.append(h)
        h = F.relu(F.conv2d(F.max_pool2d(h, 3, 2), W["conv3.weight"], W["conv3.bias"], padding=1))
        out.append(h)
        h = F.relu(F.conv2d(h, W["conv4.weight"], W["conv4.bias"], padding=1))
        out.append(h)
        h = F.relu(F.conv2d(h, W["conv5.weight"], W["conv5.bias"], padding=1))
        out.append(h)
        return out

    def normalize(f):
        return f / (torch.sqrt(torch.sum(f * f, dim=1, keepdim=True)) + 1e-10)

    score = 0
    for k, (a, b) in enumerate(zip(feats(in0), feats(in1))):
        d = (normalize(a) - normalize(b)) ** 2
        lin = W[f"lins.{k}"].view(1, -1, 1, 1)
        score = score + (d * lin).sum(1, keepdim=True).mean((2, 3), keepdim=True)
    return score


def lpips_vgg(W: Dict[str, Tensor], in0: Tensor, in1: Tensor, pre=(2.0, -1.0)) -> Tensor:
    """lpips net="vgg": torchvision vgg16().features taps relu1_2, relu2_2, relu3_3, relu4_3, relu5_3
    (lpips.pretrained_networks.vgg16 slices [0:4],[4:9],[9:16],[16:23],[23:30]); W: vgg.{0..12}.weight/.bias
    and lins.{0..4}."""
    shift = torch.tensor(LPIPS_SHIFT, dtype=in0.dtype).view(1, 3, 1, 1)
    scale = torch.tensor(LPIPS_SCALE, dtype=in0.dtype).view(1, 3, 1, 1)

    def feats(x):
        h = (pre[0] * x + pre[1] - shift) / scale
        out, i = [], 0
        for block, n in enumerate((2, 2, 3, 3, 3)):
            if block:
                h = F.max_pool2d(h, 2, 2)
            for _ in range(n):
                h = F.relu(F.conv2d(h, W[f"vgg.{i}.weight"], W[f"vgg.{i}.bias"], padding=1))
                i += 1
            out.append(h)
        return out

    def normalize(f):
        return f / (torch.sqrt(torch.sum(f * f, dim=1, keepdim=True)) + 1e-10)

    score = 0
    for k, (a, b) in enumerate(zip(feats(in0), feats(in1))):
        d = (normalize(a) - normalize(b)) ** 2
        score = score + (d * W[f"lins.{k}"].view(1, -1, 1, 1)).sum(1, keepdim=True).mean((2, 3), keepdim=True)
    return score


# --------------------------------------------------------------------------------------------
# validation metrics: src/utils/metrics.py:14-73 (compute_reconstruction_metrics uses torchmetrics
# 1.7.4 psnr/ssim, pinned in uv.lock:4071; not installed here -> restated from its published code:
# functional/image/ssim.py _ssim_update with gaussian_kernel=True, sigma=1.5, k1=0.01, k2=0.03,
# reflect pad (k-1)/2 then the map cropped by the same pad; psnr.py with data_range=1.0, base 10)
# --------------------------------------------------------------------------------------------
def ssim_torchmetrics(preds: Tensor, target: Tensor, data_range: float = 1.0) -> Tensor:
    sigma, k1, k2 = 1.5, 0.01, 0.03
    ks = int(3.5 * sigma + 0.5) * 2 + 1
    pad = (ks - 1) // 2
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    ch = preds.shape[1]
    dist = torch.arange((1 - ks) / 2, (1 + ks) / 2, 1, dtype=preds.dtype)
    gauss = torch.exp(-torch.pow(dist / sigma, 2) / 2)
    g1 = (gauss / gauss.sum()).unsqueeze(0)
    kernel = torch.matmul(g1.t(), g1).expand(ch, 1, ks, ks)
    p = F.pad(preds, (pad, pad, pad, pad), mode="reflect")
    t = F.pad(target, (pad, pad, pad, pad), mode="reflect")
    out = F.conv2d(torch.cat((p, t, p * p, t * t, p * t)), kernel, groups=ch).split(preds.shape[0])
    mu_p_sq, mu_t_sq, mu_pt = out[0].pow(2), out[1].pow(2), out[0] * out[1]
    s_p = torch.clamp(out[2] - mu_p_sq, min=0.0)
    s_t = torch.clamp(out[3] - mu_t_sq, min=0.0)
    s_pt = out[4] - mu_pt
    full = ((2 * mu_pt + c1) * (2 * s_pt + c2)) / ((mu_p_sq + mu_t_sq + c1) * (s_p + s_t + c2))
    return full[..., pad:-pad, pad:-pad].reshape(preds.shape[0], -1).mean(-1).mean()


def reconstruction_metrics(original: Tensor, reconstructed: Tensor) -> Dict[str, float]:
    mse = F.mse_loss(reconstructed, original)
    return {"mse": float(mse), "mae": float(F.l1_loss(reconstructed, original)),
            "psnr": float(-10.0 * torch.log10(mse)), "ssim": float(ssim_torchmetrics(reconstructed, original, 1.0))}


def kl_metrics(mean: Tensor, logvar: Tensor) -> Dict[str, float]:
    kl = 0.5 * (mean.pow(2) + logvar.exp() - logvar - 1)
    per_sample = kl.sum(dim=1)
    return {"kl_total": float(kl.sum()), "kl_mean": float(per_sample.mean()), "kl_std": float(per_sample.std()),
            "kl_per_dim_mean": float(kl.mean(dim=0).mean())}


# --------------------------------------------------------------------------------------------
# adversarial branch: NLayerDiscriminator (src/models/discriminator.py:11-82) and the hinge /
# generator terms + adaptive weight of LPIPSWithDiscriminator (src/losses/vae_losses.py:297-382)
# --------------------------------------------------------------------------------------------
def discriminator(W: Dict[str, Tensor], x: Tensor, n_layers: int = 3, training: bool = True,
                  running: Optional[Dict[str, Tensor]] = None, momentum: float = 0.1) -> Tensor:
    """W: main.{i}.weight/.bias (+ BatchNorm running stats in `running`, updated in place)."""
    i = 0
    h = F.leaky_relu(F.conv2d(x, W["main.0.weight"], W["main.0.bias"], stride=2, padding=1), 0.2)
    i = 2
    for n in range(1, n_layers + 1):
        stride = 2 if n < n_layers else 1
        h = F.conv2d(h, W[f"main.{i}.weight"], W.get(f"main.{i}.bias"), stride=stride, padding=1)
        rm = running[f"main.{i + 1}.running_mean"] if running is not None else None
        rv = running[f"main.{i + 1}.running_var"] if running is not None else None
        h = F.batch_norm(h, rm, rv, W[f"main.{i + 1}.weight"], W[f"main.{i + 1}.bias"], training, momentum, 1e-5)
        h = F.leaky_relu(h, 0.2)
        i += 3
    return F.conv2d(h, W[f"main.{i}.weight"], W[f"main.{i}.bias"], stride=1, padding=1)


def hinge_d_loss(logits_real: Tensor, logits_fake: Tensor) -> Tensor:
    return 0.5 * (torch.mean(F.relu(1.0 - logits_real)) + torch.mean(F.relu(1.0 + logits_fake)))
