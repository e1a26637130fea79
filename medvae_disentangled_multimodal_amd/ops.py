"""Autograd functions over the C-ABI kernels (libmvae_hip.so).

Activations are torch tensors with the reference's logical NCHW shapes stored channels_last
(physical NHWC); conv weights are channels_last OIHW (physical KRSC). Weight / norm-affine
gradients are written straight into the parameter's flat gradient slot (`p._mvae_main_grad`,
attached by `FlatParameters`) and accumulated there (beta = 1), so autograd never materialises
or adds them; without a flat slot the gradient is returned to autograd as usual.
Every op requires CUDA(HIP) tensors: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math
import os
import weakref
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from . import _lib

CL = torch.channels_last


# ------------------------------------------------------------------------------------------
# plumbing
# ------------------------------------------------------------------------------------------
def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _check(t: torch.Tensor, name: str = "tensor"):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: the MI355X path needs device tensors (got {t.device}); no CPU fallback")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name}: expected float32, got {t.dtype}")


def nhwc(t: torch.Tensor) -> torch.Tensor:
    """Return t with channels_last (NHWC) physical layout (no copy when it already is)."""
    if t.dim() == 4:
        return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)
    return t.contiguous()


class _Arena:
    """Per-device scratch buffers reused across launches: the work of one stream is ordered, so a buffer keyed by
    (name, device) is never used by two kernels at once -- the side-stream weight gradient of the two-stream conv
    backward (Conv2dFn._backward) gets buffers of its own (keyed by its stream) whatever names it asks for.

    A buffer that is outgrown is replaced (and its memory returned to the caching allocator). A captured
    HIP graph bakes in the raw pointers of the buffers it used, so while a capture records (`pinning`
    set by VAELightningModule._capture_step) every buffer handed out is also kept in that list: the graph
    holds them for its lifetime and later eager calls that grow the arena cannot free memory a replay
    writes into. `generation` counts replacements."""

    def __init__(self):
        self.bufs = {}
        self.generation = 0
        self.pinning = None

    def get(self, key: str, nbytes: int, device) -> torch.Tensor:
        dev = torch.device(device)
        # (only the backward's side streams get buffers of their own: the default stream and a graph-capture stream
        # never run at once, so they share one set -- two copies of the multi-GB Winograd buffers would otherwise stay
        # allocated for a graphed run)
        s = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
        k = (key, str(dev), s if s in _SIDE_STREAMS else 0)
        t = self.bufs.get(k)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(int(nbytes * 1.25) + 256, 256), dtype=torch.uint8, device=device)
            self.bufs[k] = t
            self.generation += 1
        if self.pinning is not None and not any(p is t for p in self.pinning):
            self.pinning.append(t)
        return t


ARENA = _Arena()
_SIDE_STREAMS = set()  # cuda_stream handles of the conv backward's side streams (_bwd_side)

# Optional live kernel timing (bench.py): when PROFILE is a list, every implicit-GEMM launch is
# bracketed by HIP events on the current stream and recorded as
# (tag, algorithmic_flops, start, end, shape) -- shape = the launch's problem tuple. The HBM-bound
# GroupNorm launches are recorded the same way under HBM_TAGS with algorithmic BYTES in the work slot, and so are the
# loss-side launches (reparameterization, KL, reconstruction MSE / L1 and their backwards: "loss_fwd" / "loss_bwd").
PROFILE = None
HBM_TAGS = ("gn_fwd", "gn_bwd", "loss_fwd", "loss_bwd")


class _timed:
    """HIP-event bracket of one GEMM-family launch (bench.py roofline). `flops` = the algorithmic work of
    the algorithm this launch runs (useful MACs x 2: the sub-pixel Upsample forms count 4/9 of the
    reference conv); `ref_flops` = the reference conv's count for the same result (default: flops)."""
    __slots__ = ("tag", "flops", "s", "shape", "ref_flops")

    def __init__(self, tag: str, flops: float, shape=None, ref_flops=None):
        self.tag, self.flops, self.shape = tag, flops, shape
        self.ref_flops = flops if ref_flops is None else ref_flops

    def __enter__(self):
        if PROFILE is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if PROFILE is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            PROFILE.append((self.tag, self.flops, self.s, e, self.shape, self.ref_flops))
        return False


_WEIGHT_GRADS_TO_AUTOGRAD = [False]


def _main_grad(p: torch.Tensor):
    if _WEIGHT_GRADS_TO_AUTOGRAD[0]:
        return None
    return getattr(p, "_mvae_main_grad", None)


class autograd_weight_grads:
    """Within this context the ops hand parameter gradients back to autograd instead of accumulating
    them into the flat gradient buffer -- for `torch.autograd.grad(loss, param)` probes such as the
    adaptive adversarial weight (vae_losses.py:364-382)."""

    def __enter__(self):
        self.prev = _WEIGHT_GRADS_TO_AUTOGRAD[0]
        _WEIGHT_GRADS_TO_AUTOGRAD[0] = True
        return self

    def __exit__(self, *exc):
        _WEIGHT_GRADS_TO_AUTOGRAD[0] = self.prev
        return False


# Called with each parameter whose flat-slot gradient the backward pass has just finished writing
# (set by ddp.DataParallel to launch bucket all-reduces while the rest of backward runs).
GRAD_HOOK = None


def _grad_done(*params):
    if GRAD_HOOK is not None:
        for p in params:
            if p is not None:
                GRAD_HOOK(p)


# ------------------------------------------------------------------------------------------
# convolution
# ------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class ConvGeom:
    kh: int
    kw: int
    stride: int = 1
    pad_t: int = 0
    pad_l: int = 0
    pad_b: int = 0
    pad_r: int = 0
    upsample: bool = False  # nearest x2 upsample fused into the gather (Upsample, :205-209)

    def out_hw(self, h: int, w: int) -> Tuple[int, int]:
        if self.upsample:
            h, w = 2 * h, 2 * w
        ho = (h + self.pad_t + self.pad_b - self.kh) // self.stride + 1
        wo = (w + self.pad_l + self.pad_r - self.kw) // self.stride + 1
        return ho, wo

    @property
    def pointwise(self) -> bool:
        return self.kh == 1 and self.kw == 1 and self.stride == 1 and not self.upsample and \
            self.pad_t == self.pad_l == self.pad_b == self.pad_r == 0


def _krsc(w: torch.Tensor) -> torch.Tensor:
    return w if w.is_contiguous(memory_format=CL) else w.contiguous(memory_format=CL)


def _subpixel_upsample(g: ConvGeom) -> bool:
    """Upsample's conv (nearest x2 then 3x3 s1 p1, encoder_decoder.py:205-209) runs in sub-pixel form:
    4 parity classes of 2x2 convs on the low-resolution input (4/9 of the MACs)."""
    return g.upsample and g.kh == 3 and g.kw == 3 and g.stride == 1 and \
        g.pad_t == g.pad_l == g.pad_b == g.pad_r == 1 and SUBPIXEL_UPSAMPLE


SUBPIXEL_UPSAMPLE = os.environ.get("MVAE_NO_SUBPIXEL") is None
STRIDE2_CLASSES = os.environ.get("MVAE_NO_STRIDE2_CLASSES") is None
# weight operands handed to the GEMM pre-split into 3xBF16 hi/lo pairs (include/medvae_hip.h MVAE_CONV_WSPLIT):
# the split is done once per step by the weight-prep kernels instead of in every workgroup's staging
WEIGHT_SPLIT = os.environ.get("MVAE_NO_WEIGHT_SPLIT") is None
SMALL_COUT_WGRAD = os.environ.get("MVAE_NO_SMALL_COUT_WGRAD") is None
DIRECT_WGRAD = os.environ.get("MVAE_NO_DIRECT_WGRAD") is None
# output channel counts the direct weight gradient serves (the kernel takes 32 and 64; MVAE_DIRECT_WGRAD_C64=1 adds 64)
DIRECT_WGRAD_COUT = (32, 64) if os.environ.get("MVAE_DIRECT_WGRAD_C64") is not None else (32,)
MVAE_CONV_WSPLIT = 16
MVAE_CONV_XSPLIT = 32
MVAE_CONV_DYSPLIT = 64
MVAE_CONV_DGRAD_DIRECT = 512
# 3x3 / stride-1 / pad-1 convs at 32 -> 32 channels (c3's 28x28 level): the direct stencil kernel
# (mvae_conv2d_direct32_nhwc) for the forward and the input gradient instead of the implicit GEMM
DIRECT32 = os.environ.get("MVAE_NO_DIRECT32") is None


def _direct32(g, c: int, co: int, wd: int) -> bool:
    return (DIRECT32 and c == 32 and co == 32 and g.kh == 3 and g.kw == 3 and g.stride == 1 and not g.upsample and
            (g.pad_t, g.pad_l, g.pad_b, g.pad_r) == (1, 1, 1, 1) and wd <= 62)
# the output gradient of a conv split once into 3xBF16 hi/lo groups (mvae_split_bf16) and handed pre-split to
# both of its GEMMs (input gradient: gathered A operand; weight gradient: dY^T A operand). Off by default: measured
# on c4 (same box, interleaved) the dgrad GEMMs gain 2.5 % but the wgrad GEMMs lose 2.5 % and the split pass
# (8 B/elem over every conv's dy, ~13 ms/step) outweighs the rest (441 -> 433 img/s). MVAE_DY_SPLIT=1 enables it.
DY_SPLIT = os.environ.get("MVAE_DY_SPLIT") is not None
DY_SPLIT_MIN = 1 << 18  # elements: below this the extra launch outweighs the staging work saved


def _al16(*ts) -> bool:
    return all(t.data_ptr() % 16 == 0 for t in ts)


# Winograd F(2x2, 3x3) for the 3x3 / stride-1 / pad-1 convs of the wide, low-resolution levels (c4 / c5's 8x8 x 2048 and
# 16x16 x 1024; csrc/winograd.hip): 4/9 of the GEMM MACs for the input / output transform traffic (4x the input and 4x
# the output in fp32-class words), forward and input gradient, 3xBF16 mode. MVAE_NO_WINOGRAD=1 keeps the implicit GEMM;
# MVAE_WINOGRAD_MIN_C sets the smallest channel count (both sides) it is used for.
WINOGRAD = os.environ.get("MVAE_NO_WINOGRAD") is None
WINOGRAD_MIN_C = int(os.environ.get("MVAE_WINOGRAD_MIN_C", "512"))
# ... and for images at least 32 wide (c4's 64x64x256 level: 665 -> 692 img/s same box; c2's 14x14x256 level lost 3 %
# at 256 channels)
WINOGRAD_MIN_C_WIDE = int(os.environ.get("MVAE_WINOGRAD_MIN_C_WIDE", "256"))
# output tile m of F(m x m, 3x3): 4 (default; 1/4 of the direct MACs, V / M 2.25x the input / output) or 2 (4/9 of the
# MACs, 4x the traffic, ~7x smaller transform error)
WINOGRAD_TILE = int(os.environ.get("MVAE_WINOGRAD_TILE", "4"))
if WINOGRAD_TILE not in (2, 4):
    raise ValueError("MVAE_WINOGRAD_TILE must be 2 or 4")


# The other two GEMM arithmetics. Exact fp32 ("32-exact", mode 2): the transforms write V / U as
# a bit split the f32-input MFMA reassembles exactly, so only the Winograd algorithm's own fp32 rounding differs from the
# direct conv -- F(4x4) errs ~5e-7 against float64 (direct fp32 ~4e-8), far inside the exact mode's 1e-4 step bar;
# MVAE_NO_WINOGRAD_EXACT=1 keeps the direct implicit GEMM there. bf16-mixed (mode 1): V and U rounded to bf16 in the
# transform domain amplify the rounding -- simulated against float64 at 16x16x256 the direct bf16 conv errs 2.4e-3, F(2x2)
# 4.0e-3, F(4x4) 2.7e-2 -- so that mode uses m = 2 (MVAE_WINOGRAD_TILE_BF16), at 4x the input / output transform traffic
# for 4/9 of the MACs: only where the images are small and the channels wide (MVAE_WINOGRAD_BF16_MAX_W, default 16: c5's
# 8x8x2048 and 16x16x1024 levels). The transforms write V, U and D' as packed bf16 (2 B per element: half the transform
# write traffic) and the position / weight-gradient GEMMs run on the LDS-DMA main loop like the mode's other convs.
# MVAE_NO_WINOGRAD_BF16=1 keeps its convs on the LDS-DMA implicit GEMM.
WINOGRAD_EXACT = os.environ.get("MVAE_NO_WINOGRAD_EXACT") is None
WINOGRAD_BF16 = os.environ.get("MVAE_NO_WINOGRAD_BF16") is None
WINOGRAD_TILE_BF16 = int(os.environ.get("MVAE_WINOGRAD_TILE_BF16", "2"))
WINOGRAD_BF16_MAX_W = int(os.environ.get("MVAE_WINOGRAD_BF16_MAX_W", "16"))


def _wtile() -> int:
    """The output tile m of F(m x m, 3x3) in the current GEMM arithmetic."""
    return WINOGRAD_TILE_BF16 if _MATH[0] == 1 else WINOGRAD_TILE


def _wel() -> int:
    """bytes per element of the transformed operands (V, U, D'): the 16-B-per-4 pre-split layouts, or packed bf16 in the
    bf16-mixed mode (the LDS-DMA GEMM's operand)."""
    return 2 if _MATH[0] == 1 else 4


def _wino_alg(ref: float) -> float:
    """GEMM FLOPs of the Winograd form of a conv whose direct form is `ref`: (m+2)^2 / (9 m^2)."""
    m = _wtile()
    return ref * (m + 2) ** 2 / (9.0 * m * m)


# widest image it is used for (the library takes W in {8, 16} and multiples of 32)
WINOGRAD_MAX_W = int(os.environ.get("MVAE_WINOGRAD_MAX_W", "64"))


# smallest conv (direct MACs) it is used for: the four launches of the Winograd form lose to one implicit GEMM on small
# batches (c1's 7x7x512 at B = 32, 3.7 GMAC: 3,607 -> 3,400 img/s; c2's at B = 256, 29.6 GMAC, gains 3.5 %)
WINOGRAD_MIN_MACS = float(os.environ.get("MVAE_WINOGRAD_MIN_MACS", "1e10"))


def _wino_ok(g, n: int, h: int, wd: int, cin: int, cout: int) -> bool:
    """Any image size (edge tiles are zero-filled / cut: c2's 7x7 level in 2x2 tiles of 4x4); the fused GroupNorm
    statistics / partials additionally need _wino_blocks."""
    mode = _MATH[0]
    if mode == 0:  # (3xBF16 on the register-staged loop; the opt-in planar LDS-DMA format has no Winograd form)
        on, maxw = _dma_fmt() == 0, WINOGRAD_MAX_W
    elif mode == 2:
        on, maxw = WINOGRAD_EXACT, WINOGRAD_MAX_W
    else:
        on, maxw = WINOGRAD_BF16, min(WINOGRAD_MAX_W, WINOGRAD_BF16_MAX_W)
    return (WINOGRAD and on and g.kh == 3 and g.kw == 3 and g.stride == 1 and
            not g.upsample and (g.pad_t, g.pad_l, g.pad_b, g.pad_r) == (1, 1, 1, 1) and wd <= maxw and
            cin % (8 if mode == 1 else 4) == 0 and cout % (8 if mode == 1 else 4) == 0 and
            min(cin, cout) >= (WINOGRAD_MIN_C_WIDE if wd >= 32 else WINOGRAD_MIN_C) and
            9.0 * n * h * wd * cin * cout >= WINOGRAD_MIN_MACS and
            # (each transformed operand is addressed through one buffer descriptor, < 4 GiB: batches whose operands
            # exceed it run in image chunks -- at most WINOGRAD_MAX_CHUNKS)
            len(_wino_chunks(n, h, wd, max(cin, cout))) <= WINOGRAD_MAX_CHUNKS)


_MAX_DESC_BYTES = 0xFFFFFF00  # csrc/gemm_core.h MAX_DESC_BYTES

# The Upsample conv (nearest x2 + 3x3 / pad 1, encoder_decoder.py:194-209) on the Winograd form: four class convs on the
# low-resolution input (the sub-pixel form's tap sums as 3x3 class kernels, csrc/winograd.hip wino_ups_weights_kernel)
# sharing one input transform, a position GEMM over N = 4 cout: (m+2)^2 / m^2 MACs per output pixel per channel pair
# instead of the sub-pixel form's 4 (0.56x at m = 4) for the class-interleaving output transform. Same size rules as the
# plain Winograd conv on the low-resolution image. MVAE_NO_WINOGRAD_UPSAMPLE=1: the sub-pixel GEMM.
# Measured (same box, interleaved, profiles/r06_ab_c4_upsample_gnlink.txt, r06_ab_c5.txt): c4 725 -> 740 img/s; in the
# bf16-mixed mode F(2x2) on the Upsample convs lost (c5 964 -> 942), so that mode keeps them on the LDS-DMA sub-pixel
# GEMM (MVAE_WINOGRAD_UPSAMPLE_BF16=1 enables them there).
WINOGRAD_UPSAMPLE = os.environ.get("MVAE_NO_WINOGRAD_UPSAMPLE") is None
WINOGRAD_UPSAMPLE_BF16 = os.environ.get("MVAE_WINOGRAD_UPSAMPLE_BF16") is not None


def _wino_ups_ok(g, n: int, h: int, wd: int, cin: int, cout: int) -> bool:
    """g an Upsample conv geometry, (h, wd) its low-resolution input."""
    # (whole tiles only: c2's 7 -> 14 Upsample at 512 channels, in 2 x 2 tiles of 4 x 4 over a 7 x 7 image, lost 1.4 %,
    # profiles/r06_ab_c2_upsample.txt)
    return (WINOGRAD_UPSAMPLE and (_MATH[0] != 1 or WINOGRAD_UPSAMPLE_BF16) and _subpixel_upsample(g) and
            h % _wtile() == 0 and wd % _wtile() == 0 and cout % 8 == 0 and _wino_ok(G3, n, h, wd, cin, 4 * cout) and
            min(cin, cout) >= (WINOGRAD_MIN_C_WIDE if wd >= 32 else WINOGRAD_MIN_C) and
            4 * n * h * wd * cout * 4 <= _MAX_DESC_BYTES)


def _lazy_wino(lazy, x, w, b, res, g, gn_part, wgrad: bool) -> bool:
    """A deferred GroupNorm output can stay deferred: its conv runs the Winograd forward (normalizing on load) and, when
    the weight gradient is wanted, the Winograd weight gradient on the kept input transform."""
    n, c, h, wd = x.shape
    return (_wino_ok(g, n, h, wd, c, w.shape[0]) and _al16(w, lazy.x) and (b is None or _al16(b)) and
            (res is None or _al16(res)) and (gn_part is None or _wino_blocks(h, wd)) and
            (not wgrad or WINOGRAD_WGRAD))


WINOGRAD_MAX_CHUNKS = 4


def _wino_chunks(n: int, h: int, wd: int, cmax: int):
    """[(b0, b1)] image ranges whose transformed operands ((m+2)^2 x tiles x channels x 4 B) each fit one 4 GiB buffer
    descriptor (c4's 64x64x512 decoder conv at B = 256: two halves)."""
    per_img = (_wtile() + 2) ** 2 * _wino_tiles(1, h, wd) * cmax * 4
    per = max(1, _MAX_DESC_BYTES // per_img) if per_img <= _MAX_DESC_BYTES else 0
    if per == 0:
        return [None] * (WINOGRAD_MAX_CHUNKS + 1)  # (one image alone is too large)
    return [(b0, min(n, b0 + per)) for b0 in range(0, n, per)]


def _wino_blocks(h: int, wd: int) -> bool:
    """The output transform's 32-pixel-block form (GroupNorm statistics / backward partials from it)."""
    return h % 4 == 0 and (wd in (8, 16) or wd % 32 == 0)


def _wino_tiles(n: int, h: int, wd: int) -> int:
    mt = _wtile()
    return n * (-(-h // mt)) * (-(-wd // mt))


WINOGRAD_WGRAD = os.environ.get("MVAE_NO_WINOGRAD_WGRAD") is None
# the conv backward's two passes over dy (the input gradient's input transform, the weight gradient's dy transform) as
# one (mvae_winograd_dy_transforms); MVAE_NO_WINOGRAD_DY2=1: two kernels
WINOGRAD_DY2 = os.environ.get("MVAE_NO_WINOGRAD_DY2") is None
# GroupNorm(+SiLU) -> Winograd conv: the GroupNorm computes its statistics only and the conv's input transform applies
# the normalization on load (mvae_winograd_input_transform_gn), so the GroupNorm output is never written or read
# (SURVEY §7 hard part 4 / VERDICT r4 item 3 on the Winograd form, which reads its input once). The output handed to the
# conv is a deferred placeholder (DeferredGnOutput: an expanded scalar carrying GN_LAZY_ATTR whose values any torch op
# refuses to read), never materialized on this path.
# Default since the transform normalizes in branch-free code after its 36 loads (the first build branched on the SiLU
# flag per element, which serialized the loads: 1.7x the plain transform's time, c4 -0.4 %); now the fused transform
# runs at the plain one's speed and c4 gains 2 % (704-706 -> 717-721 img/s, GroupNorm family 40.5 -> 31.9 ms; same box,
# interleaved, profiles/r05_winograd_gn_ab.txt). MVAE_NO_WINOGRAD_GN=1 writes the GroupNorm output as before.
WINOGRAD_GN = os.environ.get("MVAE_NO_WINOGRAD_GN") is None
# ... and where that GroupNorm's backward streams (the large levels), its partial pass over x and dy can come from the
# conv's Winograd input-gradient output transform instead: the GroupNorm family gets 3.5 ms per c4
# step faster (31.5 -> 28.0 ms). Its first build branched on the SiLU flag per element and summed the partials in fp64,
# one wave per SIMD: 2.1x the plain transform, c4 755 -> 740 img/s (profiles/r06_ab_c4_upsample_gnlink.txt); branch-free
# with fp32 sums per 32-pixel block it runs at two waves per SIMD and c4 gains (752.8 -> 755.1, same box, interleaved,
# profiles/r06_ab_c4_gnlink2.txt). MVAE_NO_WINOGRAD_GN_LINK=1: the GroupNorm backward's own partial pass.
WINOGRAD_GN_LINK = os.environ.get("MVAE_NO_WINOGRAD_GN_LINK") is None
GN_LAZY_ATTR = "_mvae_gn_lazy"
G3 = ConvGeom(3, 3, 1, 1, 1, 1, 1, False)  # the GroupNorm-fed convs' geometry (ResnetBlock conv1 / conv2, conv_out)


class LazyGn:
    """A GroupNorm output deferred to its consuming conv: x (the GroupNorm input), the apply's affine (scale, shift
    [n][c]) and the SiLU flag. materialize() writes y for a consumer that cannot apply it itself."""
    __slots__ = ("x", "scale", "shift", "silu")

    def __init__(self, x, silu: bool):
        self.x, self.silu = x, int(silu)
        self.scale = self.shift = None

    def materialize(self):
        n, c, h, w = self.x.shape
        y = torch.empty_like(self.x, memory_format=CL)
        _lib.call("mvae_group_norm_apply_nhwc", self.x.data_ptr(), self.scale.data_ptr(), self.shift.data_ptr(),
                  y.data_ptr(), n, h * w, c, self.silu, 0, _stream(self.x))
        return y


class DeferredGnOutput(torch.Tensor):
    """The placeholder group_norm hands its consuming conv when the GroupNorm output is deferred (LazyGn): an expanded
    scalar with the output's shape, dtype and device, attached to the GroupNorm's autograd node. Its values are never
    computed, so every read of them raises -- a forward hook, user code on a Normalize output, any torch op -- instead
    of returning the placeholder's bytes. Only metadata queries (shape, device, dtype, data_ptr, version, layout
    checks) pass; ops.conv2d takes the values from the LazyGn record it carries. MVAE_NO_WINOGRAD_GN=1 writes the
    GroupNorm output instead."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        if func in _DEFERRED_META:
            with torch._C.DisableTorchFunctionSubclass():
                return func(*args, **(kwargs or {}))
        name = getattr(func, "__qualname__", None) or getattr(func, "__name__", repr(func))
        raise RuntimeError(f"{name}: this GroupNorm output is deferred to its consuming convolution (the conv's Winograd "
                           "input transform applies the normalization); its values exist nowhere else. Read the conv's "
                           "output instead, or set MVAE_NO_WINOGRAD_GN=1 to have the GroupNorm write its output.")


_DEFERRED_META = {torch.Tensor.shape.__get__, torch.Tensor.size, torch.Tensor.dim, torch.Tensor.ndim.__get__,
                  torch.Tensor.data_ptr, torch.Tensor._version.__get__, torch.Tensor.is_contiguous,
                  torch.Tensor.device.__get__, torch.Tensor.dtype.__get__, torch.Tensor.is_cuda.__get__,
                  torch.Tensor.requires_grad.__get__, torch.Tensor.grad_fn.__get__, torch.Tensor.numel,
                  torch.Tensor.layout.__get__, torch.Tensor.stride, torch.Tensor.is_leaf.__get__,
                  torch.Tensor.__hash__, torch.Tensor.element_size, torch.Tensor.get_device}


def _wino_ups_wgrad_ok(g, x, dy, dw) -> bool:
    n, c, h, wd = x.shape
    return (WINOGRAD_WGRAD and _wino_ups_ok(g, n, h, wd, c, dy.shape[1]) and _al16(x, dy, dw) and
            dy.is_contiguous(memory_format=CL) and dw.is_contiguous(memory_format=CL))


def _wino_wgrad_ok(g, x, dy, dw, dys) -> bool:
    n, c, h, wd = x.shape
    co = dy.shape[1]
    return (WINOGRAD_WGRAD and _wino_ok(g, n, h, wd, c, co) and _al16(x, dy, dw) and (dys is None or _al16(dys)) and
            dy.is_contiguous(memory_format=CL) and dw.is_contiguous(memory_format=CL))


# the forward's Winograd input transform V is kept for the weight gradient (which needs the same V of the same x)
# instead of being recomputed there: one input transform per conv and step less, at (m+2)^2/m^2 x the input's bytes
# of memory held from forward to backward (c4 ≈ 27 GB). MVAE_NO_WINOGRAD_KEEP_V=1 recomputes it.
WINOGRAD_KEEP_V = os.environ.get("MVAE_NO_WINOGRAD_KEEP_V") is None


def _winograd(src, w, n: int, h: int, wd: int, k_in: int, n_out: int, src_split: bool, dgrad: bool, st, keep=None,
              gn=None, key=None, u=None, chunk=(0, 0), dkeep=None):
    """U (filters, unless `u` is given), V (input tiles) and the (m+2)^2 position GEMMs M = V U^T for the n images of
    src; returns (M (arena), U) for an output transform. keep (a list): V is allocated outside the arena and appended
    to it (WINOGRAD_KEEP_V), tagged with `key` (the conv's input tensor; default src) and the image range `chunk`.
    gn (LazyGn): src is a GroupNorm input, normalized on load (its scale / shift rows of these images).
    dkeep (a list; input gradient only): src is dy, and the weight gradient's D' = A dy A^T comes out of the same pass
    over dy (mvae_winograd_dy_transforms), appended like keep's entries for conv2d_wgrad_raw."""
    mt = _wtile()
    t = _wino_tiles(n, h, wd)
    pos = (mt + 2) ** 2
    dev = src.device
    if keep is not None:
        v = torch.empty(_wel() * pos * t * k_in, dtype=torch.uint8, device=dev)
        kt = src if key is None else key
        keep.append((v, mt, kt.data_ptr(), kt._version, tuple(chunk)))
    else:
        v = ARENA.get("wino_v", _wel() * pos * t * k_in, dev)
    m = ARENA.get("wino_m", 4 * pos * t * n_out, dev)
    if u is None:
        u = ARENA.get("wino_u", _wel() * pos * k_in * n_out, dev)
        cin, cout = (n_out, k_in) if dgrad else (k_in, n_out)
        _lib.call("mvae_winograd_weight_transform", w.data_ptr(), u.data_ptr(), cin, cout, int(dgrad), mt, st)
    if dkeep is not None:
        d = torch.empty(_wel() * pos * t * k_in, dtype=torch.uint8, device=dev)
        kt = src if key is None else key
        dkeep.append((d, mt, kt.data_ptr(), kt._version, tuple(chunk)))
        _lib.call("mvae_winograd_dy_transforms", src.data_ptr(), v.data_ptr(), d.data_ptr(), n, h, wd, k_in,
                  int(src_split), mt, st)
    elif gn is not None:
        b0 = chunk[0]
        _lib.call("mvae_winograd_input_transform_gn", src.data_ptr(), gn.scale[b0 * k_in:].data_ptr(),
                  gn.shift[b0 * k_in:].data_ptr(), gn.silu, v.data_ptr(), n, h, wd, k_in, mt, st)
    else:
        _lib.call("mvae_winograd_input_transform", src.data_ptr(), v.data_ptr(), n, h, wd, k_in, int(src_split), mt,
                  st)
    _lib.call("mvae_winograd_gemm", v.data_ptr(), u.data_ptr(), m.data_ptr(), t, k_in, n_out, mt, st)
    return m, u


# Convolutions on DMA-staged operands: the GEMM stages them into LDS by DMA (no staging registers, conversion or
# split). bf16-mixed: packed bf16 (MVAE_CONV_BF16, 64-deep K-tiles; default, MVAE_NO_BF16_DMA=1 keeps the
# register-staged bf16 loop on fp32 operands). fp32-class 3xBF16: planar hi / lo bf16 planes (MVAE_CONV_PLANAR,
# 32-deep K-tiles) -- opt-in (MVAE_PLANAR_DMA=1): measured on c4 (same box) the planar weight gradient runs 10 % faster
# (384 -> 421 TF/s) but fwd / dgrad 5-7 % slower than the hand-pipelined register loop, and the planar dy / x passes
# (8 B per element) cost more than the rest gains: 453 -> 427 img/s.
BF16_DMA = os.environ.get("MVAE_NO_BF16_DMA") is None
PLANAR_DMA = os.environ.get("MVAE_PLANAR_DMA") is not None
MVAE_CONV_BF16 = 128
MVAE_CONV_PLANAR = 256


def _dma_fmt() -> int:
    """operand format of the DMA-staged conv path in the current math mode: 2 = packed bf16, 3 = planar 3xBF16
    (the GroupNorm y_split / weight-prep split codes), 0 = none."""
    if _MATH[0] == 1 and BF16_DMA:
        return 2
    if _MATH[0] == 0 and PLANAR_DMA:
        return 3
    return 0


def _bf16_dma() -> bool:
    return _dma_fmt() != 0


# 3xBF16 mode: the planar DMA path for convolutions of at least this many MACs (the c4 layers; the small layers of the
# 28x28 models keep their tuned register-staged / direct kernels). One rule for the GroupNorm that writes a conv's
# input and for the conv's three GEMMs, so their operand formats agree.
PLANAR_MIN_MACS = 1e11


def _dma_ok(macs: float) -> bool:
    f = _dma_fmt()
    return f == 2 or (f == 3 and macs >= PLANAR_MIN_MACS)


def _dma_flag() -> int:
    return MVAE_CONV_PLANAR if _dma_fmt() == 3 else MVAE_CONV_BF16


def _dma_bytes(numel: int) -> int:
    """bytes of a DMA-staged operand of numel elements (packed bf16: 2 per element; planar: two bf16 planes)"""
    return numel * (4 if _dma_fmt() == 3 else 2)


class _FlatWeights:
    """The conv weights of a step prepared in one launch: fit_step converts the whole flat parameter buffer
    (optim.FlatParameters: every tensor 16-B aligned) into the forward GEMM's weight format -- split4_bf16 in the
    3xBF16 mode, packed bf16 in the bf16-mixed mode -- before the forward, and every conv forward then reads its
    weight's slice instead of converting it (one launch per conv, ~30 per c3 step). Valid until the optimizer step.
    Only the tensors a step actually reads in that format are converted once they are known: `want` records every
    request of a step (data pointer -> elements), the next prep converts just those ranges (merged runs) and `covered`
    holds what this step's copy contains -- a request outside it gets None (the caller converts its own weight) and is
    covered from the next step on. c4: the Winograd convs (~90 % of the 927 M parameters) transform the fp32 weight
    themselves, so the prep moves ~1/10 of the bytes."""
    __slots__ = ("base", "end", "buf", "fmt", "fresh", "want", "covered")

    def __init__(self):
        self.base = self.end = 0
        self.buf = None
        self.fmt = 0
        self.fresh = False
        self.want = {}
        self.covered = None  # None: the whole buffer


_FLATW = _FlatWeights()


class _TransposedWeights:
    """Every dgrad weight re-layout of a step in one launch (mvae_conv_weight_transpose_batched). The (weight, shape,
    format) triples the input-gradient GEMMs ask for are learned on a step that runs them one launch per conv; the
    descriptor table is then uploaded once, and from the next step on fit_step's weight prep (prep_flat_weights)
    re-lays out all of them before the forward, each dgrad reading its slot (~30 launches fewer per c3 step). Valid
    until the optimizer step, like _FlatWeights. Only weights inside the flat parameter buffer are tabled (stable
    addresses); a step graph that bakes in the table and its buffer pins both (ARENA.pinning), so a replaced table
    is freed unless a live graph still uses it."""
    __slots__ = ("slots", "want", "table", "buf", "n", "blocks", "fresh", "base", "end", "tbase", "tend", "seen",
                 "idle")

    def __init__(self):
        self.slots, self.want = {}, {}
        self.seen = set()  # keys the dgrads of the current step asked for
        self.idle = {}     # key -> consecutive prepared steps that did not ask for it
        self.table = self.buf = None
        self.n = self.blocks = 0
        self.fresh = False
        self.base = self.end = self.tbase = self.tend = 0


_WT = _TransposedWeights()
BATCHED_WT = os.environ.get("MVAE_NO_BATCHED_WT") is None
WT_IDLE_STEPS = 2  # a table entry unused for this many prepared steps is dropped


def _wt_blocks(co, rs, c):
    return ((c + 63) // 64) * ((co + 63) // 64) * rs


def refresh_weight_tables(flat_data: torch.Tensor):
    """Build / extend the batched dgrad re-layout table from what earlier steps asked for (host work + one upload);
    called by prep_flat_weights and, before a step graph is captured, by the trainer (no upload inside a capture)."""
    n = flat_data.numel()
    _WT.base, _WT.end = flat_data.data_ptr(), flat_data.data_ptr() + 4 * n
    if BATCHED_WT:
        _wt_rebuild(flat_data.device)


def _wt_rebuild(dev):
    if (_WT.tbase, _WT.tend) != (_WT.base, _WT.end):  # a new flat buffer: the table's weight addresses are gone
        _WT.slots, _WT.table, _WT.buf, _WT.n, _WT.idle = {}, None, None, 0, {}
        _WT.want = {k: v for k, v in _WT.want.items() if _WT.base <= k[0] < _WT.end}
        _WT.tbase, _WT.tend = _WT.base, _WT.end
    # entries no step has asked for in the last WT_IDLE_STEPS prepared steps (e.g. the other arithmetic's formats after
    # a precision switch) leave the table instead of being re-laid out every step
    stale = [k for k, c in _WT.idle.items() if c >= WT_IDLE_STEPS]
    for k in stale:
        _WT.want.pop(k, None)
        _WT.idle.pop(k, None)
    if stale or any(k not in _WT.slots for k in _WT.want):
        import numpy as np
        keys = [k for k in _WT.slots if k in _WT.want] + [k for k in _WT.want if k not in _WT.slots]
        info = dict(_WT.want)
        offs, o = {}, 0
        for k in keys:
            offs[k] = o
            o += (info[k][5] + 255) // 256 * 256
        buf = torch.empty(o, dtype=torch.uint8, device=dev)
        dt = np.dtype([("w", "<u8"), ("wt", "<u8"), ("cout", "<i4"), ("rs", "<i4"), ("cin", "<i4"), ("split", "<i4"),
                       ("block0", "<i4"), ("pad0", "<i4")])
        arr = np.zeros(len(keys), dtype=dt)
        b0 = 0
        for i, k in enumerate(keys):
            wp, co, rs, c, split, _ = info[k]
            arr[i] = (wp, buf.data_ptr() + offs[k], co, rs, c, split, b0, 0)
            b0 += _wt_blocks(co, rs, c)
        table = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
        _WT.slots, _WT.table, _WT.buf, _WT.n, _WT.blocks = offs, table, buf, len(keys), b0
        _WT.want = dict(info)


def _prep_transposed(dev, st):
    _WT.fresh = False
    if not BATCHED_WT:
        return
    if not torch.cuda.is_current_stream_capturing():
        if _WT.seen:  # the previous prepared step's requests: age the entries it did not use
            for k in _WT.slots:
                _WT.idle[k] = 0 if k in _WT.seen else _WT.idle.get(k, 0) + 1
            _WT.seen = set()
        _wt_rebuild(dev)
    if _WT.n and (_WT.tbase, _WT.tend) == (_WT.base, _WT.end):
        if ARENA.pinning is not None:  # a step graph being recorded bakes in the table and its buffer
            for t in (_WT.table, _WT.buf):
                if not any(p is t for p in ARENA.pinning):
                    ARENA.pinning.append(t)
        _lib.call("mvae_conv_weight_transpose_batched", _WT.table.data_ptr(), _WT.n, _WT.blocks, st)
        _WT.fresh = True


def _weight_t(w, co, kh, kw, c, split, nbytes, st) -> int:
    """Device pointer of w re-laid out [cin][taps][cout] in format `split` (mvae_conv_weight_transpose): the slot the
    step's batched prep wrote, or a per-conv launch into arena scratch (recorded for the next table)."""
    p = w.data_ptr()
    key = (p, co, kh, kw, c, int(split))
    _WT.seen.add(key)
    if _WT.fresh and key in _WT.slots:
        return _WT.buf.data_ptr() + _WT.slots[key]
    wt = ARENA.get("wt", nbytes, w.device)
    _lib.call("mvae_conv_weight_transpose", p, wt.data_ptr(), co, kh, kw, c, int(split), st)
    if BATCHED_WT and _WT.base <= p < _WT.end and w.is_contiguous(memory_format=CL):
        _WT.want[key] = (p, co, kh * kw, c, int(split), nbytes)
    return wt.data_ptr()


# MVAE_NO_FLAT_PREP_WANTED=1: convert the whole flat buffer every step; MVAE_FLAT_PREP_GAP: runs closer than this many
# elements are converted as one launch
FLAT_PREP_WANTED = os.environ.get("MVAE_NO_FLAT_PREP_WANTED") is None
FLAT_PREP_GAP = int(os.environ.get("MVAE_FLAT_PREP_GAP", str(1 << 20)))


def prep_flat_weights(flat_data: torch.Tensor):
    """Convert the flat parameter buffer into the forward weight format of the current math mode (see
    _FlatWeights); a no-op in modes without a converted weight format."""
    fmt = 2 if _dma_fmt() == 2 else (1 if _MATH[0] == 0 and WEIGHT_SPLIT and _dma_fmt() == 0 else 0)
    _FLATW.fresh = False
    n = flat_data.numel()
    _WT.base, _WT.end = flat_data.data_ptr(), flat_data.data_ptr() + 4 * n
    _prep_transposed(flat_data.device, _stream(flat_data))
    if fmt == 0 or n % 8 or not _al16(flat_data):
        return
    nbytes = n * (4 if fmt == 1 else 2)
    if _FLATW.buf is None or _FLATW.buf.numel() < nbytes or _FLATW.buf.device != flat_data.device:
        _FLATW.buf = torch.empty(nbytes, dtype=torch.uint8, device=flat_data.device)
    fn = "mvae_split_bf16" if fmt == 1 else "mvae_pack_bf16"
    if ARENA.pinning is not None and not any(p is _FLATW.buf for p in ARENA.pinning):
        ARENA.pinning.append(_FLATW.buf)  # (a step graph being recorded bakes it in)
    base = flat_data.data_ptr()
    same = _FLATW.base == base and _FLATW.end == base + 4 * n and _FLATW.fmt == fmt
    want = _FLATW.want if same and FLAT_PREP_WANTED else {}
    _FLATW.want = {}
    if want:
        runs = []
        for p, numel in sorted(want.items()):
            a = ((p - base) // 4) & ~7  # (whole 8-element groups: 16-B aligned source and packed destination)
            e = min(n, ((p - base) // 4 + numel + 7) & ~7)
            if runs and a - runs[-1][1] <= FLAT_PREP_GAP:
                runs[-1][1] = max(runs[-1][1], e)
            else:
                runs.append([a, e])
        eb = 4 if fmt == 1 else 2
        for a, e in runs:
            _lib.call(fn, base + 4 * a, _FLATW.buf.data_ptr() + eb * a, e - a, _stream(flat_data))
        _FLATW.covered = set(want)
    else:
        _lib.call(fn, base, _FLATW.buf.data_ptr(), n, _stream(flat_data))
        _FLATW.covered = None
    _FLATW.base, _FLATW.end, _FLATW.fmt, _FLATW.fresh = base, base + 4 * n, fmt, True


def release_weight_buffers():
    """Free the step's converted weight copies (_FLATW.buf: the flat buffer in split4 / packed bf16, 4 / 2 B per
    parameter; _WT: the dgrad re-layouts, about one more copy of the conv weights -- together ~7.4 GB for the 927 M
    parameters of c4 in the 3xBF16 mode) and forget the re-layout table. The next prepared step rebuilds them."""
    flat_weights_stale()
    _FLATW.buf, _FLATW.base, _FLATW.end = None, 0, 0
    _FLATW.want, _FLATW.covered = {}, None
    _WT.slots, _WT.want, _WT.seen, _WT.idle = {}, {}, set(), {}
    _WT.table = _WT.buf = None
    _WT.n = _WT.blocks = 0
    _WT.tbase = _WT.tend = 0


def flat_weights_stale():
    _FLATW.fresh = False
    _WT.fresh = False


def _flat_weight_ptr(w: torch.Tensor, fmt: int) -> Optional[int]:
    """Device pointer of w's prepared copy (fmt 1: split4_bf16, 2: packed bf16), or None."""
    p = w.data_ptr()
    if not (_FLATW.fresh and _FLATW.fmt == fmt and _FLATW.base <= p < _FLATW.end and
            w.is_contiguous(memory_format=CL)):
        return None
    _FLATW.want[p] = w.numel()
    if _FLATW.covered is not None and p not in _FLATW.covered:
        return None  # (not in this step's copy: converted by the caller, and from the next step on by the prep)
    off = p - _FLATW.base
    return _FLATW.buf.data_ptr() + (off if fmt == 1 else off // 2)


def pack_bf16(t: torch.Tensor, key: str) -> torch.Tensor:
    """DMA-staged operand copy of an fp32 tensor in arena scratch `key`: packed bf16 (round to nearest even, 2 B per
    element) in the bf16-mixed mode, planar 3xBF16 (hi plane then lo plane) in the 3xBF16 mode."""
    out = ARENA.get(key, _dma_bytes(t.numel()), t.device)
    fn = "mvae_split_planar" if _dma_fmt() == 3 else "mvae_pack_bf16"
    _lib.call(fn, t.data_ptr(), out.data_ptr(), t.numel(), _stream(t))
    return out


# current GEMM arithmetic (mirror of mvae_get_math_mode, kept by set_precision / math_scope): 0 = 3xBF16,
# 1 = bf16, 2 = exact fp32 (f32-input MFMA). The 3xBF16 pre-split operand layouts are value splits and are
# not used in the exact mode.
_MATH = [0]


def _splits_ok() -> bool:
    return _MATH[0] != 2


class math_scope:
    """Run the enclosed launches in GEMM math mode `mode` (a module whose convolutions must run in a fixed
    arithmetic whatever the trainer precision, e.g. the discriminator in exact fp32)."""

    def __init__(self, mode: Optional[int]):
        self.mode = mode

    def __enter__(self):
        self.prev = _MATH[0]
        if self.mode is not None and self.mode != self.prev:
            _lib.call("mvae_set_math_mode", int(self.mode))
            _MATH[0] = int(self.mode)
        return self

    def __exit__(self, *exc):
        if _MATH[0] != self.prev:
            _lib.call("mvae_set_math_mode", int(self.prev))
            _MATH[0] = self.prev
        return False


# Split-K for under-filled conv launches (mvae_conv2d_ws_nhwc: the small-spatial, wide-channel layers of the 28x28
# models leave most CUs idle for a partial round); MVAE_NO_CONV_SPLITK=1 keeps every fwd / dgrad launch unsplit.
CONV_SPLITK = os.environ.get("MVAE_NO_CONV_SPLITK") is None
_CONV_WS_CACHE = {}


def _conv_call(x, w, b, res, y, n, h, wd, c, co, kh, kw, stride, pad_t, pad_l, ho, wo, mode, st):
    """mvae_conv2d_nhwc, or its split-K form when the library's planner splits this geometry."""
    nbytes = 0
    if CONV_SPLITK:
        key = (n, c, co, kh, kw, ho, wo)
        nbytes = _CONV_WS_CACHE.get(key)
        if nbytes is None:
            nbytes = _CONV_WS_CACHE[key] = int(_lib.query("mvae_conv2d_split_workspace_bytes", n, c, co, kh, kw, ho, wo))
    if nbytes:
        ws = ARENA.get("convsplit", nbytes, y.device)
        _lib.call("mvae_conv2d_ws_nhwc", x, w, b, res, y.data_ptr(), n, h, wd, c, co, kh, kw, stride, pad_t, pad_l, ho,
                  wo, mode, ws.data_ptr(), ws.numel(), st)
    else:
        _lib.call("mvae_conv2d_nhwc", x, w, b, res, y.data_ptr(), n, h, wd, c, co, kh, kw, stride, pad_t, pad_l, ho, wo,
                  mode, st)


def conv2d_forward_raw(x, w, b, res, g: ConvGeom, x_split: bool = False, gn_part=None, x_bf16: bool = False,
                       keep_v=None, lazy=None):
    """gn_part (fp64 [n*ho*wo/32 * cout/4 * 2]): also emit the GroupNorm statistics of y from the GEMM
    epilogue (mvae_conv2d_gnstats_nhwc; only on the plain implicit-GEMM path -- the caller checks).
    x_bf16: x holds packed bf16 (BF16_ATTR; bf16-mixed mode)."""
    n, c, h, wd = x.shape
    co = w.shape[0]
    ho, wo = g.out_hw(h, wd)
    y = torch.empty((n, co, ho, wo), device=x.device, dtype=torch.float32, memory_format=CL)
    ref = 2.0 * n * ho * wo * co * c * g.kh * g.kw
    sub = _subpixel_upsample(g)
    alg = ref * 4 / 9 if sub else ref
    st = _stream(x)
    # (the vector gather keeps one validity bit per filter tap: kernels of more than 32 taps take the scalar path,
    # which reads unsplit weights)
    split = WEIGHT_SPLIT and _splits_ok() and c % 4 == 0 and _al16(x) and not g.pointwise and g.kh * g.kw <= 32
    if x_split and (g.pointwise or g.upsample or c % 4 or not _al16(x)):
        raise RuntimeError("conv2d: a pre-split input needs a non-pointwise, non-upsample conv with cin % 4 == 0")
    # (the Winograd form first: in the bf16-mixed mode it takes the small wide levels off the LDS-DMA path)
    wino = not x_bf16 and _wino_ok(g, n, h, wd, c, co) and _al16(w) and (b is None or _al16(b)) and \
        (res is None or _al16(res)) and (gn_part is None or _wino_blocks(h, wd)) and _al16(lazy.x if lazy is not None else x)
    wups = not x_bf16 and not x_split and lazy is None and res is None and gn_part is None and \
        _wino_ups_ok(g, n, h, wd, c, co) and _al16(x, w) and (b is None or _al16(b))
    if wups:
        with _timed("conv_fwd", _wino_alg(ref), (n, c, h, wd, co, g.kh, g.stride, g.upsample), ref):
            kc = ARENA.get("wups_k", 4 * co * 9 * c * 4, x.device)
            _lib.call("mvae_winograd_upsample_weights", w.data_ptr(), kc.data_ptr(), c, co, st)
            u = None
            for b0, b1 in _wino_chunks(n, h, wd, max(c, 4 * co)):
                m, u = _winograd(x[b0:b1], kc, b1 - b0, h, wd, c, 4 * co, False, False, st, keep_v, key=x, u=u,
                                 chunk=(b0, b1))
                _lib.call("mvae_winograd_output_transform_upsample", m.data_ptr(), _ptr(b), y[b0:b1].data_ptr(),
                          b1 - b0, h, wd, co, _wtile(), st)
        return y
    if not wino and _dma_ok(ref / 2) and c % 8 == 0 and not x_split and _al16(x) and not g.pointwise and \
            g.kh * g.kw <= 32 and (sub or not g.upsample):
        return _conv_fwd_bf16(x, w, b, res, g, y, n, c, h, wd, co, ho, wo, sub, alg, ref, gn_part, st, x_bf16)
    if x_bf16:
        raise RuntimeError("conv2d: a packed bf16 input needs the bf16-mixed LDS-DMA conv path")
    if lazy is not None and not wino:  # a deferred GroupNorm output whose conv cannot normalize on load: write it
        x, lazy = lazy.materialize(), None
    if wino:
        with _timed("conv_fwd", _wino_alg(ref), (n, c, h, wd, co, g.kh, g.stride, g.upsample), ref):
            src = lazy.x if lazy is not None else x
            u = None
            for b0, b1 in _wino_chunks(n, h, wd, max(c, co)):
                m, u = _winograd(src[b0:b1], w, b1 - b0, h, wd, c, co, x_split, False, st, keep_v, gn=lazy, key=x,
                                 u=u, chunk=(b0, b1))
                gp = gn_part[b0 * (h * wd // 32) * (co // 4) * 2:] if gn_part is not None else None
                _lib.call("mvae_winograd_output_transform", m.data_ptr(), _ptr(b),
                          _ptr(res[b0:b1] if res is not None else None), y[b0:b1].data_ptr(), _ptr(gp), b1 - b0, h,
                          wd, co, _wtile(), st)
        return y
    wg = w
    if sub:  # tap-summed per-class weights (prepared outside the timed GEMM launch)
        wg = ARENA.get("w4", 16 * co * c * 4, x.device)
        _lib.call("mvae_conv_weight_upsample_fwd", w.data_ptr(), wg.data_ptr(), co, c, int(split), st)
    elif split:
        wp = _flat_weight_ptr(w, 1)
        if wp is None:
            wg = ARENA.get("wsplit", w.numel() * 4, x.device)
            _lib.call("mvae_split_bf16", w.data_ptr(), wg.data_ptr(), w.numel(), st)
            wp = wg.data_ptr()
    wptr = wg.data_ptr() if not split or sub else wp
    with _timed("conv_fwd", alg, (n, c, h, wd, co, g.kh, g.stride, g.upsample), ref):
        if g.pointwise:
            # 1x1 conv = GEMM [pixels][cin] x [cout][cin]^T
            _lib.call("mvae_gemm_strided_batched", 0, 1, n * h * wd, co, c, 1.0, x.data_ptr(), c, 0,
                      w.data_ptr(), c, 0, 0.0, y.data_ptr(), co, 0, 1, _ptr(b), _ptr(res), co, 0, None, 0, st)
        elif sub:
            _lib.call("mvae_conv2d_upsample_nhwc", x.data_ptr(), wg.data_ptr(), _ptr(b), _ptr(res), y.data_ptr(), n,
                      h, wd, c, co, int(split), st)
        elif gn_part is None and _direct32(g, c, co, wd) and _al16(x, wg) and (res is None or _al16(res)):
            _lib.call("mvae_conv2d_direct32_nhwc", x.data_ptr(), wptr, _ptr(b), _ptr(res), y.data_ptr(), n, h, wd,
                      (MVAE_CONV_WSPLIT if split else 0) | (MVAE_CONV_XSPLIT if x_split else 0), st)
        else:
            mode = (1 if g.upsample else 0) | (MVAE_CONV_WSPLIT if split else 0) | (MVAE_CONV_XSPLIT if x_split else 0)
            if gn_part is not None:
                _lib.call("mvae_conv2d_gnstats_nhwc", x.data_ptr(), wptr, _ptr(b), _ptr(res), y.data_ptr(),
                          n, h, wd, c, co, g.kh, g.kw, g.stride, g.pad_t, g.pad_l, ho, wo, mode, gn_part.data_ptr(), st)
            else:
                _conv_call(x.data_ptr(), wptr, _ptr(b), _ptr(res), y, n, h, wd, c, co, g.kh, g.kw, g.stride,
                           g.pad_t, g.pad_l, ho, wo, mode, st)
    return y


def _conv_fwd_bf16(x, w, b, res, g, y, n, c, h, wd, co, ho, wo, sub, alg, ref, gn_part, st, x_bf16=False):
    """bf16-mixed forward on packed bf16 x and weights (MVAE_CONV_BF16)."""
    fmt, flag = _dma_fmt(), _dma_flag()
    xb = x if x_bf16 else pack_bf16(x, "xbf")
    if sub:
        wg = ARENA.get("w4", _dma_bytes(16 * co * c), x.device)
        _lib.call("mvae_conv_weight_upsample_fwd", w.data_ptr(), wg.data_ptr(), co, c, fmt, st)
    else:
        wp = _flat_weight_ptr(w, 2) if fmt == 2 else None
        wg = pack_bf16(w, "wsplit") if wp is None else None
    wptr = wg.data_ptr() if wg is not None else wp
    with _timed("conv_fwd", alg, (n, c, h, wd, co, g.kh, g.stride, g.upsample), ref):
        if sub:
            _lib.call("mvae_conv2d_upsample_nhwc", xb.data_ptr(), wptr, _ptr(b), _ptr(res), y.data_ptr(), n,
                      h, wd, c, co, fmt, st)
        elif gn_part is not None:
            _lib.call("mvae_conv2d_gnstats_nhwc", xb.data_ptr(), wptr, _ptr(b), _ptr(res), y.data_ptr(),
                      n, h, wd, c, co, g.kh, g.kw, g.stride, g.pad_t, g.pad_l, ho, wo, flag, gn_part.data_ptr(), st)
        else:
            _conv_call(xb.data_ptr(), wptr, _ptr(b), _ptr(res), y, n, h, wd, c, co, g.kh, g.kw, g.stride,
                       g.pad_t, g.pad_l, ho, wo, flag, st)
    return y


def pack_dy(dy: torch.Tensor, g: ConvGeom, cin: int, bias_out=None, beta: float = 1.0):
    """dy as packed bf16 for the backward GEMMs of the bf16-mixed mode, or None when that path does not apply.
    bias_out: also accumulate the conv bias gradient (beta * bias_out + column sums of the fp32 dy) from the same pass
    (mvae_pack_bf16_colsum). Returns (packed dy or None, whether the bias gradient was produced)."""
    if not _bf16_dma() or g.pointwise or dy.dim() != 4 or dy.shape[1] % 8 or g.kh * g.kw > 32 or not _al16(dy) or \
            not dy.is_contiguous(memory_format=CL) or not _dma_ok(float(dy.numel()) * cin * g.kh * g.kw) or \
            _wino_ok(g, dy.shape[0], dy.shape[2], dy.shape[3], cin, dy.shape[1]) or \
            _wino_ups_ok(g, dy.shape[0], dy.shape[2] // 2, dy.shape[3] // 2, cin, dy.shape[1]):  # (Winograd: fp32 dy)
        return None, False
    if bias_out is None:
        return pack_bf16(dy, "dybf"), False
    n, co, ho, wo = dy.shape
    rows = n * ho * wo
    out = ARENA.get("dybf", _dma_bytes(dy.numel()), dy.device)
    ws = ARENA.get("bias", _lib.query("mvae_bias_grad_workspace_bytes", rows, co), dy.device)
    fn = "mvae_split_planar_colsum" if _dma_fmt() == 3 else "mvae_pack_bf16_colsum"
    _lib.call(fn, dy.data_ptr(), out.data_ptr(), rows, co, bias_out.data_ptr(), float(beta), ws.data_ptr(), ws.numel(),
              _stream(dy))
    return out, True


def split_dy(dy: torch.Tensor) -> Optional[torch.Tensor]:
    """dy in the 3xBF16 operand layout (split4_bf16 groups), or None when the conv cannot use it."""
    if not DY_SPLIT or not _splits_ok() or dy.dim() != 4 or dy.shape[1] % 4 or dy.numel() < DY_SPLIT_MIN or not _al16(dy) or \
            not dy.is_contiguous(memory_format=CL):
        return None
    ds = torch.empty_like(dy, memory_format=CL)
    _lib.call("mvae_split_bf16", dy.data_ptr(), ds.data_ptr(), dy.numel(), _stream(dy))
    return ds


def conv2d_dgrad_raw(dy, w, x_shape, g: ConvGeom, gn_link=None, dys=None, dyb=None, dkeep=None, out=None,
                     beta: float = 0.0, u_pre=None):
    """gn_link (GnBwdLink): the conv's input was silu?(GroupNorm(x)) -- also emit that GroupNorm's backward
    partials from the GEMM epilogue (mvae_conv2d_dgrad_gnbwd_nhwc) into gn_link.part when the launch allows it.
    dys: dy pre-split by split_dy (same values; used as the gathered GEMM operand when given).
    dyb: dy as packed bf16 (pack_dy; bf16-mixed mode).
    dkeep (a list): on the Winograd path also keep the weight gradient's transformed dy per image chunk (_winograd).
    out / beta (1x1 convs only): dx = beta * out + dy W into out (DxSum).
    u_pre ((U', event)): the Winograd filter transform computed during the forward on a side stream (_upre_launch)."""
    n, c, h, wd = x_shape
    co = w.shape[0]
    _, _, ho, wo = dy.shape
    if out is not None and not g.pointwise:
        raise RuntimeError("conv2d_dgrad_raw: an accumulating output is for 1x1 convs")
    dx = out if out is not None else torch.empty((n, c, h, wd), device=dy.device, dtype=torch.float32,
                                                 memory_format=CL)
    st = _stream(dy)
    flops = 2.0 * n * ho * wo * co * c * g.kh * g.kw  # reference count
    shp = (n, c, h, wd, co, g.kh, g.stride, g.upsample)
    if dyb is None and dys is None and _wino_ups_ok(g, n, h, wd, c, co) and _al16(dy, w) and \
            dy.is_contiguous(memory_format=CL):
        # the Upsample conv's input gradient on the Winograd form: sum over the classes of the class sub-images of dy
        # convolved with the flipped, transposed class kernels -- one GEMM over K = 4 cout
        mt = _wtile()
        pos = (mt + 2) ** 2
        with _timed("conv_dgrad", _wino_alg(flops), shp, flops):
            kc = ARENA.get("wups_k", 4 * co * 9 * c * 4, dy.device)
            _lib.call("mvae_winograd_upsample_weights", w.data_ptr(), kc.data_ptr(), c, co, st)
            u = ARENA.get("wino_u", _wel() * pos * c * 4 * co, dy.device)
            _lib.call("mvae_winograd_weight_transform", kc.data_ptr(), u.data_ptr(), c, 4 * co, 1, mt, st)
            for b0, b1 in _wino_chunks(n, h, wd, max(c, 4 * co)):
                nb, t = b1 - b0, _wino_tiles(b1 - b0, h, wd)
                v = ARENA.get("wino_v", _wel() * pos * t * 4 * co, dy.device)
                if dkeep is not None:
                    d = torch.empty(_wel() * pos * t * 4 * co, dtype=torch.uint8, device=dy.device)
                    dkeep.append((d, mt, dy.data_ptr(), dy._version, (b0, b1)))
                else:
                    d = ARENA.get("wino_d", _wel() * pos * t * 4 * co, dy.device)
                _lib.call("mvae_winograd_dy_transforms_upsample", dy[b0:b1].data_ptr(), v.data_ptr(), d.data_ptr(), nb,
                          h, wd, co, mt, st)
                m = ARENA.get("wino_m", 4 * pos * t * c, dy.device)
                _lib.call("mvae_winograd_gemm", v.data_ptr(), u.data_ptr(), m.data_ptr(), t, 4 * co, c, mt, st)
                _lib.call("mvae_winograd_output_transform", m.data_ptr(), None, None, dx[b0:b1].data_ptr(), None, nb, h,
                          wd, c, mt, st)
        return dx
    if dyb is not None and (gn_link is None or not gn_link.usable(dx)):
        return _conv_dgrad_bf16(dyb, w, dx, g, n, c, h, wd, co, ho, wo, flops, shp, st)
    if dys is not None and (g.pointwise or co % 4):
        dys = None
    dya = dy if dys is None else dys
    if _wino_ok(g, n, h, wd, co, c) and _al16(dya, w) and dy.is_contiguous(memory_format=CL):
        # the input gradient is the 3x3 / pad-1 conv of dy with the flipped, transposed filters
        link = gn_link if gn_link is not None and gn_link.usable(dx) and _wino_blocks(h, wd) else None
        part = torch.empty(n * h * wd // 32 * c * 2, device=dy.device, dtype=torch.float64) if link else None
        with _timed("conv_dgrad", _wino_alg(flops), shp, flops):
            u = None
            if u_pre is not None:  # (made during the forward on the side stream: joined here)
                torch.cuda.current_stream(dy.device).wait_event(u_pre[1])
                u = u_pre[0]
            for b0, b1 in _wino_chunks(n, h, wd, max(c, co)):
                nb = b1 - b0
                m, u = _winograd(dya[b0:b1], w, nb, h, wd, co, c, dys is not None, True, st, u=u, key=dya,
                                 chunk=(b0, b1), dkeep=dkeep)
                if link is None:
                    _lib.call("mvae_winograd_output_transform", m.data_ptr(), None, None, dx[b0:b1].data_ptr(), None, nb,
                              h, wd, c, _wtile(), st)
                else:  # with the GroupNorm backward partials (mvae_conv2d_dgrad_gnbwd_nhwc's epilogue sums)
                    L = link
                    _lib.call("mvae_winograd_output_gnbwd", m.data_ptr(), dx[b0:b1].data_ptr(), L.x[b0:b1].data_ptr(),
                              L.mean[b0 * L.groups:].data_ptr(), L.rstd[b0 * L.groups:].data_ptr(),
                              L.gamma.data_ptr(), L.beta.data_ptr(), L.groups, L.silu,
                              part[b0 * (h * wd // 32) * c * 2:].data_ptr(), nb, h, wd, c, _wtile(), st)
            if link is not None:
                link.part, link.dx = part, dx
        return dx
    if gn_link is not None and gn_link.usable(dx) and not g.pointwise and not g.upsample and g.stride == 1 and \
            co % 4 == 0 and _al16(dy, dx):
        split = WEIGHT_SPLIT and _splits_ok()
        wtp = _weight_t(w, co, g.kh, g.kw, c, int(split), c * g.kh * g.kw * co * 4, st)
        part = torch.empty(n * h * wd // 32 * c * 2, device=dy.device, dtype=torch.float64)
        L = gn_link
        flags = int(split) | (2 if dys is not None else 0)
        with _timed("conv_dgrad", flops, shp):
            _lib.call("mvae_conv2d_dgrad_gnbwd_nhwc", dya.data_ptr(), wtp, dx.data_ptr(), n, ho, wo, co, c,
                      g.kh, g.kw, g.pad_t, g.pad_l, h, wd, flags, L.x.data_ptr(), L.mean.data_ptr(),
                      L.rstd.data_ptr(), L.gamma.data_ptr(), L.beta.data_ptr(), L.groups, L.silu, part.data_ptr(), st)
        L.part, L.dx = part, dx
        return dx
    if g.pointwise:
        # dx[m][c] = sum_n dy[m][n] W[n][c]  (W stored [K=cout][N=cin])
        with _timed("conv_dgrad", flops, shp):
            _lib.call("mvae_gemm_strided_batched", 0, 0, n * h * wd, c, co, 1.0, dy.data_ptr(), co, 0, w.data_ptr(), c,
                      0, float(beta), dx.data_ptr(), c, 0, 1, None, None, 0, 0, None, 0, st)
        return dx
    # the dgrad GEMM's K runs over cout: transposed weights [cin][taps][cout], pre-split when cout % 4 == 0
    split = WEIGHT_SPLIT and _splits_ok() and co % 4 == 0 and _al16(dy) and g.kh * g.kw <= 32
    wflag = MVAE_CONV_WSPLIT if split else 0
    xflag = MVAE_CONV_XSPLIT if dys is not None else 0
    if g.upsample:
        wt = ARENA.get("wt", c * 16 * co * 4, dy.device)
        _lib.call("mvae_conv_weight_upsample_dgrad", w.data_ptr(), wt.data_ptr(), co, c, int(split), st)
        # dX = stride-2, pad-1 4x4 conv of dY with the tap-summed kernel (16 taps per low-res pixel)
        with _timed("conv_dgrad", flops * 4 / 9, shp, flops):
            _lib.call("mvae_conv2d_nhwc", dya.data_ptr(), wt.data_ptr(), None, None, dx.data_ptr(), n, ho, wo, co, c,
                      4, 4, 2, 1, 1, h, wd, wflag | xflag, st)
        return dx
    if _direct32(g, c, co, wd) and _al16(w, dya):
        # 32 -> 32 channels (c3's 28x28 level): the direct stencil kernel with the flipped, transposed taps
        with _timed("conv_dgrad", flops, shp):
            _lib.call("mvae_conv2d_direct32_nhwc", dya.data_ptr(), w.data_ptr(), None, None, dx.data_ptr(), n, h, wd,
                      MVAE_CONV_DGRAD_DIRECT | xflag, st)
        return dx
    wtp = _weight_t(w, co, g.kh, g.kw, c, int(split), c * g.kh * g.kw * co * 4, st)
    if g.stride == 2 and h % 2 == 0 and wd % 2 == 0 and g.kh <= 4 and g.kw <= 4 and STRIDE2_CLASSES:
        # Downsample's input gradient by dx parity class: only the useful taps (no stride holes)
        wc = ARENA.get("wcls", c * g.kh * g.kw * co * 4, dy.device)
        flags = int(split) | (2 if dys is not None else 0)
        with _timed("conv_dgrad", flops, shp):
            _lib.call("mvae_conv2d_dgrad_stride2_nhwc", dya.data_ptr(), wtp, dx.data_ptr(), n, h, wd, c, co,
                      g.kh, g.kw, g.pad_t, g.pad_l, ho, wo, flags, wc.data_ptr(), wc.numel(), st)
        return dx
    with _timed("conv_dgrad", flops, shp):
        _conv_call(dya.data_ptr(), wtp, None, None, dx, n, ho, wo, co, c, g.kh, g.kw, g.stride, g.pad_t,
                   g.pad_l, h, wd, 2 | wflag | xflag, st)
    return dx


def _conv_dgrad_bf16(dyb, w, dx, g, n, c, h, wd, co, ho, wo, flops, shp, st):
    """bf16-mixed input gradient on packed bf16 dy and weights (MVAE_CONV_BF16)."""
    dev = dx.device
    fmt, flag = _dma_fmt(), _dma_flag()
    if g.upsample:
        wt = ARENA.get("wt", _dma_bytes(c * 16 * co), dev)
        _lib.call("mvae_conv_weight_upsample_dgrad", w.data_ptr(), wt.data_ptr(), co, c, fmt, st)
        with _timed("conv_dgrad", flops * 4 / 9, shp, flops):
            # dX = stride-2, pad-1 4x4 (forward-gather) conv of dY with the tap-summed kernel
            _lib.call("mvae_conv2d_nhwc", dyb.data_ptr(), wt.data_ptr(), None, None, dx.data_ptr(), n, ho, wo, co, c,
                      4, 4, 2, 1, 1, h, wd, flag, st)
        return dx
    wtp = _weight_t(w, co, g.kh, g.kw, c, fmt, _dma_bytes(c * g.kh * g.kw * co), st)
    if g.stride == 2 and h % 2 == 0 and wd % 2 == 0 and g.kh <= 4 and g.kw <= 4 and STRIDE2_CLASSES:
        wc = ARENA.get("wcls", c * g.kh * g.kw * co * 4, dev)
        with _timed("conv_dgrad", flops, shp):
            _lib.call("mvae_conv2d_dgrad_stride2_nhwc", dyb.data_ptr(), wtp, dx.data_ptr(), n, h, wd, c, co,
                      g.kh, g.kw, g.pad_t, g.pad_l, ho, wo, 8 if fmt == 3 else 4, wc.data_ptr(), wc.numel(), st)
        return dx
    with _timed("conv_dgrad", flops, shp):
        _conv_call(dyb.data_ptr(), wtp, None, None, dx, n, ho, wo, co, c, g.kh, g.kw, g.stride, g.pad_t,
                   g.pad_l, h, wd, 2 | flag, st)
    return dx


def conv2d_wgrad_raw(dy, x, dw, beta: float, g: ConvGeom, db=None, x_split: bool = False, dys=None, dyb=None,
                     x_bf16: bool = False, wino_v=None, wino_d=None, lazy=None):
    """dw (+ db when given and the conv is not pointwise) accumulate with `beta`. Returns True when
    the bias gradient was produced by the fused wgrad kernel. dys: dy pre-split by split_dy; dyb: dy as packed bf16
    (pack_dy, bf16-mixed mode). lazy (LazyGn): x is a deferred GroupNorm output -- the Winograd weight gradient takes
    the forward's kept V (or re-derives it from the GroupNorm input); any other weight gradient gets x written first."""
    n, c, h, wd = x.shape
    co = dy.shape[1]
    _, _, ho, wo = dy.shape
    if lazy is not None and (dyb is not None or not _wino_wgrad_ok(g, lazy.x, dy, dw, dys)):
        x, lazy = lazy.materialize(), None
    ref = 2.0 * n * ho * wo * co * c * g.kh * g.kw
    alg = ref * 4 / 9 if _subpixel_upsample(g) else ref
    if dyb is None and (_wino_wgrad_ok(g, x if lazy is None else lazy.x, dy, dw, dys) or _wino_ups_wgrad_ok(g, x, dy, dw)):
        alg = _wino_alg(ref)
    if dyb is not None and not x_split and not g.upsample and c % 8 == 0 and co % 8 == 0 and _al16(x):
        # bf16-mixed weight gradient on packed bf16 dy and x (LDS-DMA main loop); the bias gradient is summed from the
        # fp32 dy by the caller
        xb = x if x_bf16 else pack_bf16(x, "xbf")
        st = _stream(dy)
        nbytes = _lib.query("mvae_conv2d_wgrad_workspace_bytes", n, c, co, g.kh, g.kw, ho, wo)
        ws = ARENA.get("ws", nbytes, dy.device)
        with _timed("conv_wgrad", alg, (n, c, h, wd, co, g.kh, g.stride, g.upsample), ref):
            _lib.call("mvae_conv2d_wgrad_nhwc", dyb.data_ptr(), xb.data_ptr(), dw.data_ptr(), None, float(beta), n, h,
                      wd, c, co, g.kh, g.kw, g.stride, g.pad_t, g.pad_l, ho, wo, _dma_flag(), ws.data_ptr(),
                      ws.numel(), st)
        return False
    if x_bf16:
        raise RuntimeError("conv2d wgrad: a packed bf16 input needs the bf16-mixed LDS-DMA path (packed dy, cout % 8)")
    with _timed("conv_wgrad", alg, (n, c, h, wd, co, g.kh, g.stride, g.upsample), ref):
        return _conv_wgrad_launch(dy, x, dw, beta, g, n, c, h, wd, co, ho, wo, db, x_split, dys, wino_v, wino_d, lazy)


def _conv_wgrad_launch(dy, x, dw, beta, g, n, c, h, wd, co, ho, wo, db=None, x_split=False, dys=None, wino_v=None,
                       wino_d=None, lazy=None):
    st = _stream(dy)
    # a deferred GroupNorm output has no values to read: its weight gradient is the Winograd one, on the kept (or
    # re-derived) V, ahead of the kernels below that read x -- the direct cout-32 kernel would otherwise take a 32-channel
    # conv and read n*h*w*c floats from the placeholder's one-element allocation
    deferred = isinstance(x, DeferredGnOutput)
    if deferred and (lazy is None or not _wino_wgrad_ok(g, lazy.x, dy, dw, dys)):
        # (conv2d_wgrad_raw materializes such an x for every other path: reaching here would read the placeholder)
        raise RuntimeError("conv2d wgrad: a deferred GroupNorm output reached a weight-gradient kernel that reads x")
    if x_split and (g.pointwise or g.upsample):
        raise RuntimeError("conv2d wgrad: a pre-split input needs a non-pointwise, non-upsample conv")
    if g.pointwise and db is None:
        m = n * h * wd
        nbytes = _lib.query("mvae_gemm_workspace_bytes", co, c, m, 1)
        ws = ARENA.get("ws", nbytes, dy.device)
        # dW[n][c] = sum_m dy[m][n] x[m][c]: A = dy stored [K=m][M=cout], B = x stored [K=m][N=cin]
        _lib.call("mvae_gemm_strided_batched", 1, 0, co, c, m, 1.0, dy.data_ptr(), co, 0, x.data_ptr(), c, 0,
                  float(beta), dw.data_ptr(), c, 0, 1, None, None, 0, 0, ws.data_ptr(), ws.numel(), st)
        return False
    if (not deferred and SMALL_COUT_WGRAD and co <= 4 and c % 4 == 0 and not g.upsample and g.kh == 3 and g.kw == 3 and g.stride == 1
            and (g.pad_t, g.pad_l, g.pad_b, g.pad_r) == (1, 1, 1, 1) and _al16(x)):
        # Decoder.conv_out (cout 3): x read once, scattered into its 9 taps (no 9x im2col stream)
        nbytes = _lib.query("mvae_conv2d_wgrad_small_cout_workspace_bytes", n, c)
        ws = ARENA.get("ws", nbytes, dy.device)
        _lib.call("mvae_conv2d_wgrad_small_cout_nhwc", dy.data_ptr(), x.data_ptr(), dw.data_ptr(), _ptr(db),
                  float(beta), n, h, wd, c, co, int(x_split), ws.data_ptr(), ws.numel(), st)
        return db is not None
    if (not deferred and DIRECT_WGRAD and dys is None and c in (32, 64) and co in DIRECT_WGRAD_COUT and _MATH[0] != 2 and
            not g.upsample and g.kh == 3 and g.kw == 3 and g.stride == 1 and (g.pad_t, g.pad_l, g.pad_b, g.pad_r) == (1, 1, 1, 1) and
            _al16(x, dy)):
        # cout 32 (c3's 28x28 / 14x14 levels): per-tap MFMA products over LDS-resident row bands; 28x28x32 at bs 512
        # 128 -> 75 us, 28x28 64->32 185 -> 118 us (tools/wgrad_bench.py); cout 64 ties the GEMM and keeps it
        nbytes = _lib.query("mvae_conv2d_wgrad_direct_workspace_bytes", n, h, wd, c, co)
        ws = ARENA.get("ws", nbytes, dy.device)
        _lib.call("mvae_conv2d_wgrad_direct_nhwc", dy.data_ptr(), x.data_ptr(), dw.data_ptr(), _ptr(db), float(beta),
                  n, h, wd, c, co, int(x_split), ws.data_ptr(), ws.numel(), st)
        return db is not None
    if not deferred and not x_split and _wino_ups_wgrad_ok(g, x, dy, dw):
        # the Upsample conv's weight gradient on the Winograd form: the class kernels' gradients G^T [sum_t D'_pq (.) V] G
        # (D' of the class sub-images of dy, kept by the input gradient's pass; V the forward's), folded onto the taps
        mt = _wtile()
        pos = (mt + 2) ** 2
        dev = dy.device
        kept = {e[4]: e[0] for e in wino_v or () if e[1] == mt and e[2] == x.data_ptr() and e[3] == x._version}
        kept_d = {e[4]: e[0] for e in wino_d or () if e[1] == mt and e[2] == dy.data_ptr() and e[3] == dy._version}
        dkc = ARENA.get("wups_dk", 4 * co * 9 * c * 4, dev)
        for i, (b0, b1) in enumerate(_wino_chunks(n, h, wd, max(c, 4 * co))):
            nb, t = b1 - b0, _wino_tiles(b1 - b0, h, wd)
            v, dt = kept.get((b0, b1)), kept_d.get((b0, b1))
            if dt is None:
                dt = ARENA.get("wino_d", _wel() * pos * t * 4 * co, dev)
                _lib.call("mvae_winograd_dy_transforms_upsample", dy[b0:b1].data_ptr(), None, dt.data_ptr(), nb, h, wd,
                          co, mt, st)
            if v is None:
                v = ARENA.get("wino_v", _wel() * pos * t * c, dev)
                _lib.call("mvae_winograd_input_transform", x[b0:b1].data_ptr(), v.data_ptr(), nb, h, wd, c, 0, mt, st)
            m = ARENA.get("wino_mw", 4 * pos * 4 * co * c, dev)
            ws = ARENA.get("ws", _lib.query("mvae_gemm_workspace_bytes", 4 * co, c, t, pos), dev)
            _lib.call("mvae_winograd_wgrad_gemm", dt.data_ptr(), v.data_ptr(), m.data_ptr(), t, 4 * co, c, mt,
                      ws.data_ptr(), ws.numel(), st)
            _lib.call("mvae_winograd_wgrad_output", m.data_ptr(), dkc.data_ptr(), 0.0 if i == 0 else 1.0, 4 * co, c, mt,
                      st)
        _lib.call("mvae_winograd_upsample_fold", dkc.data_ptr(), dw.data_ptr(), float(beta), c, co, st)
        return False
    if not deferred and _subpixel_upsample(g):
        nbytes = _lib.query("mvae_conv2d_wgrad_upsample_workspace_bytes", n, h, wd, c, co)
        ws = ARENA.get("ws", nbytes, dy.device)
        _lib.call("mvae_conv2d_wgrad_upsample_nhwc", dy.data_ptr(), x.data_ptr(), dw.data_ptr(), _ptr(db),
                  float(beta), n, h, wd, c, co, ws.data_ptr(), ws.numel(), st)
        return db is not None
    if _wino_wgrad_ok(g, x if lazy is None else lazy.x, dy, dw, dys):
        # Winograd F(3x3, 2x2): dW = G^T [sum_tiles (A D A^T) (.) (B^T X B)] G (csrc/winograd.hip); the bias gradient is
        # left to the caller
        mt = _wtile()
        pos = (mt + 2) ** 2
        dev = dy.device
        dya = dys if dys is not None else dy
        # the forward's V of this x, per image chunk, when it was kept (same tile size, x unchanged since)
        kept = {}
        for e in wino_v or ():
            if e[1] == mt and e[2] == x.data_ptr() and e[3] == x._version:
                kept[e[4]] = e[0]
        kept_d = {}  # the input gradient's pass over dy kept D' too (mvae_winograd_dy_transforms)
        for e in wino_d or ():
            if e[1] == mt and e[2] == dya.data_ptr() and e[3] == dya._version:
                kept_d[e[4]] = e[0]
        for i, (b0, b1) in enumerate(_wino_chunks(n, h, wd, max(c, co))):
            nb, t = b1 - b0, _wino_tiles(b1 - b0, h, wd)
            v = kept.get((b0, b1))
            dt = kept_d.get((b0, b1))
            m = ARENA.get("wino_mw", 4 * pos * co * c, dev)
            ws = ARENA.get("ws", _lib.query("mvae_gemm_workspace_bytes", co, c, t, pos), dev)
            if dt is None:
                dt = ARENA.get("wino_d", _wel() * pos * t * co, dev)
                _lib.call("mvae_winograd_dy_transform", dya[b0:b1].data_ptr(), dt.data_ptr(), nb, h, wd, co,
                          int(dys is not None), mt, st)
            if v is None and lazy is not None:  # (the kept V is gone -- a second backward: re-derived, normalized on load)
                v = ARENA.get("wino_v", _wel() * pos * t * c, dev)
                _lib.call("mvae_winograd_input_transform_gn", lazy.x[b0:b1].data_ptr(), lazy.scale[b0 * c:].data_ptr(),
                          lazy.shift[b0 * c:].data_ptr(), lazy.silu, v.data_ptr(), nb, h, wd, c, mt, st)
            elif v is None:
                v = ARENA.get("wino_v", _wel() * pos * t * c, dev)
                _lib.call("mvae_winograd_input_transform", x[b0:b1].data_ptr(), v.data_ptr(), nb, h, wd, c,
                          int(x_split), mt, st)
            _lib.call("mvae_winograd_wgrad_gemm", dt.data_ptr(), v.data_ptr(), m.data_ptr(), t, co, c, mt,
                      ws.data_ptr(), ws.numel(), st)
            # (image chunks accumulate: the first with the caller's beta, the rest onto it)
            _lib.call("mvae_winograd_wgrad_output", m.data_ptr(), dw.data_ptr(), float(beta) if i == 0 else 1.0, co, c,
                      mt, st)
        return False
    nbytes = _lib.query("mvae_conv2d_wgrad_workspace_bytes", n, c, co, g.kh, g.kw, ho, wo)
    ws = ARENA.get("ws", nbytes, dy.device)
    mode = (1 if g.upsample else 0) | (MVAE_CONV_XSPLIT if x_split else 0)
    dya = dy
    if dys is not None and co % 4 == 0:  # (a pre-split dy carries no in-kernel bias sum: the caller sums it)
        mode |= MVAE_CONV_DYSPLIT
        dya = dys
        db = None
    _lib.call("mvae_conv2d_wgrad_nhwc", dya.data_ptr(), x.data_ptr(), dw.data_ptr(), _ptr(db), float(beta), n, h, wd,
              c, co, g.kh, g.kw, g.stride, g.pad_t, g.pad_l, ho, wo, mode, ws.data_ptr(), ws.numel(), st)
    return db is not None


def bias_grad_raw(dy2d_ptr, rows, n, out, beta, device, stream):
    nbytes = _lib.query("mvae_bias_grad_workspace_bytes", rows, n)
    ws = ARENA.get("bias", nbytes, device)
    _lib.call("mvae_bias_grad", dy2d_ptr, rows, n, n, out.data_ptr(), float(beta), ws.data_ptr(), ws.numel(), stream)


class DxSum:
    """The input gradient of several 1x1 convs that read the same tensor (AttnBlock's q, k and v of norm(x),
    encoder_decoder.py:83-107): each conv's input-gradient GEMM accumulates into one buffer (beta = 1 after the first)
    and only the last of them returns it, so autograd never sums the three activation-sized gradients (two adds of
    [B, C, 16, 16] per attention block). Re-armed after the last, so a retained graph's next backward works alike; a conv
    whose input gradient is not requested never touches it. MVAE_NO_DX_SUM=1: autograd sums them."""
    __slots__ = ("n", "left", "buf")

    def __init__(self, n: int):
        self.n = self.left = n
        self.buf = None


DX_SUM = os.environ.get("MVAE_NO_DX_SUM") is None


class GradSink:
    """Side channel for the two gradient branches of a block input x (ResnetBlock: norm1(x) and the
    residual / nin_shortcut(x), encoder_decoder.py:141-170; AttnBlock: norm(x) and the residual, :83-107).
    The residual-side op's backward (the producer: Conv2dFn's residual passthrough or the nin_shortcut
    dgrad) parks its gradient here instead of returning it, and the GroupNorm backward of norm1 (the
    consumer) sums it into dx inside gn_dx -- no separate autograd add over the activation. If the
    consumer runs first (engine order), it marks the sink closed and the producer returns its gradient
    normally, so the result is correct in either order."""
    __slots__ = ("g", "closed")

    def __init__(self):
        self.g = None
        self.closed = False

    def park(self, g) -> bool:
        # one producer per sink and backward pass: a gradient still parked here is left over from a pass
        # that never reached the consumer (a partial torch.autograd.grad) and is replaced
        if self.closed:
            return False
        self.g = g
        return True

    def take(self):
        g, self.g = self.g, None
        self.closed = g is None
        return g


# bf16-mixed mode: a conv output that a GroupNorm normalizes carries a DyPack request. The GroupNorm backward then writes
# its dx -- this conv's output gradient -- also as packed bf16 with the conv bias gradient summed in the same pass
# (mvae_group_norm_bwd_pack_nhwc), and the conv backward takes both from it instead of a pack_bf16_colsum pass over dy.
DYPACK_ATTR = "_mvae_dypack"
DYPACK = os.environ.get("MVAE_NO_DYPACK") is None
# fp32-class (3xBF16) mode: the same request with the output gradient written as split4_bf16 groups
# (mvae_group_norm_bwd_split_nhwc) -- the pre-split dY operand of both backward GEMMs (input gradient: the gathered A
# operand, MVAE_CONV_XSPLIT; weight gradient: dY^T, MVAE_CONV_DYSPLIT), so neither splits dy in its K loop, and the
# conv bias gradient summed in the same pass. MVAE_NO_DYSPLIT=1: the conv backward splits dy in registers as before.
DYSPLIT = os.environ.get("MVAE_NO_DYSPLIT") is None
# ... and, for a Winograd conv that reads dy in fp32, the bias gradient alone (mvae_group_norm_bwd_colsum_nhwc).
# MVAE_NO_DYBIAS=1: a separate column-sum pass over dy.
DYBIAS = os.environ.get("MVAE_NO_DYBIAS") is None
# The Winograd convs of the 3xBF16 and bf16 arithmetics take dy in fp32 too (their dy transform splits / rounds it in
# registers) and get only the bias gradient from the GroupNorm backward: one 4-B write per element fewer wherever that
# GroupNorm also writes dx (the next block's norm1). MVAE_WINOGRAD_DY_SPLIT=1: the split copy as before.
WINOGRAD_DY_FP32 = os.environ.get("MVAE_WINOGRAD_DY_SPLIT") is None
# only for convs of at least this many MACs (the c4 levels): measured same box, interleaved (profiles/r05_dysplit_ab.txt),
# c4 +0.9 % (dgrad 442 -> 459, wgrad 414 -> 426 TF/s against +4.3 ms of GroupNorm backward for the extra 4 B per
# element), while c2 (-0.6 %) and c3 (-3.6 %) lose: their GEMMs gain less than the wider GroupNorm pass costs
DYSPLIT_MIN_MACS = 1e11


class DyPack:
    __slots__ = ("bias_ref", "packed", "dx_ref", "dx_version", "dx_shape", "bias_done", "db", "split", "nodx",
                 "copy_ok")

    def __init__(self, bias_ref, split: bool = False):
        self.bias_ref = bias_ref
        # False: packed bf16 (bf16-mixed); True: split4_bf16 (3xBF16); "bias": the bias gradient only (a conv that reads
        # dy in fp32 -- the exact-fp32 Winograd convs, the Upsample conv's Winograd form)
        self.split = split
        self.packed = self.dx_ref = self.dx_version = self.dx_shape = self.db = None
        self.bias_done = False
        self.nodx = False  # the GroupNorm wrote only the copy (its dx has this conv as its only consumer)
        self.copy_ok = False  # (set by conv2d: every backward path of this conv reads the copy, never the fp32 dy)

    def take(self, dy):
        """(packed dy, bias gradient done, returned bias gradient) when the GroupNorm backward produced them from
        exactly this gradient tensor (same storage, untouched since), else None; consumed once. The GroupNorm's dx is
        tracked by a weak reference, not its address: once autograd has summed another branch into a new tensor and
        freed dx, that address can come back from the allocator for an unrelated dy (a layout copy of the sum) --
        a stale address match the weak reference rules out."""
        packed, ref, ver, shp, nodx = self.packed, self.dx_ref, self.dx_version, self.dx_shape, self.nodx
        out = (packed, self.bias_done, self.db)
        self.packed = self.dx_ref = self.dx_version = self.dx_shape = self.db = None
        self.bias_done = self.nodx = False
        dx = ref() if ref is not None else None
        if packed is None or dx is None or dy.data_ptr() != dx.data_ptr() or dy._version != ver or \
                tuple(dy.shape) != shp or not dy.is_contiguous(memory_format=CL):
            if nodx:
                raise RuntimeError("conv2d backward: the GroupNorm wrote only the copy of its dx for this conv (its only "
                                   "consumer), but the conv's output gradient is another tensor")
            return None
        return out


# Input and weight gradients of one conv on two streams: the weight-gradient GEMM runs on a per-device side stream
# while the input-gradient GEMM runs on the current one, so the partial last wave of either fills with the other's
# tiles. Only for convs up to MVAE_BWD_OVERLAP_MAX_GF GFLOP (default 200): c3 +1.7 %, c2 +0.6 % img/s; the c4 convs
# (1.2 TFLOP each) already fill the chip and lose 3 % to the contention; c1 / c5 neutral (profiles/r04_bwd_overlap_ab.txt).
# MVAE_BWD_OVERLAP=0: one stream. Streams and events are made outside graph capture and reused.
BWD_OVERLAP = os.environ.get("MVAE_BWD_OVERLAP", "1") != "0"
BWD_OVERLAP_MAX_FLOPS = float(os.environ.get("MVAE_BWD_OVERLAP_MAX_GF", "200")) * 1e9
_SIDE = {}


def _bwd_side(t: torch.Tensor):
    # (off while bench.py's instrumented step records per-launch HIP events: concurrent kernels would overlap the
    # brackets and overstate each launch's duration)
    if not BWD_OVERLAP or PROFILE is not None or not t.is_cuda:
        return None
    side = _SIDE.get(t.device)
    if side is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        side = _SIDE[t.device] = (torch.cuda.Stream(t.device), torch.cuda.Event(), torch.cuda.Event())
        _SIDE_STREAMS.add(side[0].cuda_stream)
    return side


# The Winograd input gradient's filter transform U' (the flipped, transposed filters in the transform domain) depends on
# the weights alone: it is computed during the forward, on a side stream concurrent with the forward's compute-bound
# position GEMMs, instead of on the backward's critical path (c4: 31 launches, 4.1 ms per step). The buffers live from
# the forward to the backward (c4: ~10 GB). Off under graph capture and the bench's instrumented step. Measured neutral
# (c4 769.1 vs 768.0, c5 976.9 vs 977.0 img/s, same box, interleaved, profiles/r06_ab_winograd_upre.txt: the side-stream
# transform slows the concurrent GEMMs by about what it hides), so opt-in: MVAE_WINOGRAD_UPRE=1.
WINOGRAD_UPRE = os.environ.get("MVAE_WINOGRAD_UPRE") is not None
_UPRE = {}


def _upre_launch(w: torch.Tensor, g: ConvGeom, x_shape):
    """(U' buffer, event) for the conv's Winograd input gradient, launched now on a side stream, or None."""
    n, c, h, wd = x_shape
    co = w.shape[0]
    if not WINOGRAD_UPRE or PROFILE is not None or not w.is_cuda or torch.cuda.is_current_stream_capturing() or \
            g.upsample or not _wino_ok(g, n, h, wd, co, c) or not _al16(w):
        return None
    side = _UPRE.get(w.device)
    if side is None:
        side = _UPRE[w.device] = torch.cuda.Stream(w.device)
    mt = _wtile()
    u = torch.empty(_wel() * (mt + 2) ** 2 * c * co, dtype=torch.uint8, device=w.device)
    side.wait_stream(torch.cuda.current_stream(w.device))  # (w as written by the weight prep / optimizer)
    _lib.call("mvae_winograd_weight_transform", w.data_ptr(), u.data_ptr(), c, co, 1, mt, side.cuda_stream)
    ev = side.record_event()
    u.record_stream(side)
    w.record_stream(side)
    return u, ev


# experiment knob: also overlap the two backward passes of the Winograd convs (their memory-bound transforms against the
# other pass's GEMM), whatever their size
BWD_OVERLAP_WINO = os.environ.get("MVAE_BWD_OVERLAP_WINO") is not None


def _overlap_ok(x, dy, g) -> bool:
    n, c, h, w = x.shape
    _, co, ho, wo = dy.shape
    if BWD_OVERLAP_WINO and _wino_ok(g, n, h, w, c, co):
        return True
    # (image-side convs -- cout 3 / latent channels -- run memory-bound special kernels: c4 lost 0.35 % overlapping them)
    return not g.pointwise and min(c, co) >= 32 and 2.0 * n * ho * wo * co * c * g.kh * g.kw <= BWD_OVERLAP_MAX_FLOPS


class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, geom: ConvGeom, res_sink=None, x_sink=None, gn_part=None,
                gn_link=None, dypack=None, grad_on: bool = True, dx_sum=None):
        """grad_on: grad mode at the call (inside forward it is always off): no kept Winograd transform for a conv
        that will have no backward (eval / validation under torch.no_grad)."""
        _check(x, "conv input")
        xs = bool(getattr(x, XSPLIT_ATTR, False))
        xb16 = bool(getattr(x, BF16_ATTR, False))
        lazy = getattr(x, GN_LAZY_ATTR, None)
        if (xs or xb16) and not x.is_contiguous(memory_format=CL):
            raise RuntimeError("conv2d: a pre-split / packed input must not be re-laid out")
        w = _krsc(weight)
        res = nhwc(residual) if residual is not None else None
        want_w = bool(weight.requires_grad and grad_on)
        if lazy is not None and not _lazy_wino(lazy, x, w, bias, res, geom, gn_part, want_w):
            x, lazy = lazy.materialize(), None  # (the conv cannot normalize on load: the GroupNorm output is written)
        if lazy is None:
            x = nhwc(x)
        keep = [] if (WINOGRAD_KEEP_V or lazy is not None) and want_w else None
        y = conv2d_forward_raw(x, w, bias, res, geom, xs, gn_part, x_bf16=xb16, keep_v=keep, lazy=lazy)
        ctx.u_pre = _upre_launch(w, geom, tuple(x.shape)) if (grad_on and ctx.needs_input_grad[0]) else None
        ctx.wino_v = keep if keep else None
        ctx.lazy = lazy  # (the weight gradient re-derives V from it if the kept one is gone: a second backward)
        ctx.math = _MATH[0]  # the backward GEMMs run in the forward's arithmetic
        ctx.geom = geom
        ctx.x_split = xs
        ctx.x_bf16 = xb16
        ctx.has_bias = bias is not None
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, w)
        ctx.weight_ref = weight
        ctx.bias_ref = bias
        ctx.res_sink, ctx.x_sink = res_sink, x_sink
        ctx.gn_link = gn_link
        ctx.dx_sum = dx_sum
        ctx.dypack = dypack
        return y

    @staticmethod
    def backward(ctx, dy):
        with math_scope(ctx.math):
            return Conv2dFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x, w = ctx.saved_tensors
        g = ctx.geom
        dy = nhwc(dy)
        dx = dw_ret = db_ret = dres = None
        link = ctx.gn_link
        if link is not None:
            link.part = link.dx = None  # partials of an earlier pass are never reused
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        bias_done = False
        dyb = None
        got = ctx.dypack.take(dy) if ctx.dypack is not None else None
        dys = None
        if got is not None and ctx.dypack.split == "bias":  # the bias gradient (column sums of dx) by the GroupNorm
            _, bias_done, db_ret = got
            if not want_b:
                db_ret = None
            elif bias_done:
                bt = _main_grad(ctx.bias_ref)
                if bt is not None:
                    bt.add_(db_ret)
                    db_ret = None
        elif got is not None and ctx.dypack.split:  # dy pre-split (and the bias gradient) by the GroupNorm backward
            dys, bias_done, db_ret = got
            if not want_b:
                db_ret = None
            elif bias_done:
                bt = _main_grad(ctx.bias_ref)
                if bt is not None:  # into the flat slot now that dy is known to be the GroupNorm's dx
                    bt.add_(db_ret)
                    db_ret = None
        elif got is not None:  # packed dy (and the bias gradient) from the GroupNorm backward that produced dy
            dyb, bias_done, db_ret = got
            if not want_b:
                db_ret = None
            elif bias_done:
                bt = _main_grad(ctx.bias_ref)
                if bt is not None:  # into the flat slot now that dy is known to be the GroupNorm's dx
                    bt.add_(db_ret)
                    db_ret = None
        elif ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            # bf16-mixed: pack dy once for both GEMMs; the bias gradient comes out of the same pass
            bt = _main_grad(ctx.bias_ref) if want_b else None
            if want_b and bt is None:
                db_ret = torch.empty(dy.shape[1], device=dy.device, dtype=torch.float32)
            dyb, bias_done = pack_dy(dy, g, w.shape[1], bt if bt is not None else db_ret, 1.0 if bt is not None else 0.0)
            if not bias_done:
                db_ret = None
        if dys is None and not g.pointwise and not _subpixel_upsample(g) and dyb is None:
            dys = split_dy(dy)
        dkeep = None  # (set below when the input gradient's pass over dy also writes the weight gradient's D')

        def wgrad():
            nonlocal dw_ret, bias_done
            tgt = _main_grad(ctx.weight_ref)
            btgt = _main_grad(ctx.bias_ref) if want_b and not bias_done else None
            want_b_w = want_b and not bias_done
            xs, xb16 = ctx.x_split, ctx.x_bf16
            lz = ctx.lazy
            if tgt is not None and (not want_b_w or btgt is not None):
                fused = conv2d_wgrad_raw(dy, x, tgt, 1.0, g, btgt, x_split=xs, dys=dys, dyb=dyb, x_bf16=xb16,
                                         wino_v=ctx.wino_v, wino_d=dkeep, lazy=lz)
                bias_done = bias_done or fused
            elif tgt is not None:
                conv2d_wgrad_raw(dy, x, tgt, 1.0, g, x_split=xs, dys=dys, dyb=dyb, x_bf16=xb16, wino_v=ctx.wino_v,
                                 wino_d=dkeep, lazy=lz)
            else:
                dw_ret = torch.empty_like(w, memory_format=CL)
                conv2d_wgrad_raw(dy, x, dw_ret, 0.0, g, x_split=xs, dys=dys, dyb=dyb, x_bf16=xb16,
                                 wino_v=ctx.wino_v, wino_d=dkeep, lazy=lz)

        side = _bwd_side(dy) if ctx.needs_input_grad[0] and ctx.needs_input_grad[1] and \
            _main_grad(ctx.weight_ref) is not None and _overlap_ok(x, dy, g) else None
        if side is not None:
            # the weight gradient on the side stream, concurrent with the input gradient (the arena keys its scratch
            # buffers by stream, so the two never share one); joined before returning
            stream, ev_fork, ev_join = side
            main = torch.cuda.current_stream(dy.device)
            ev_fork.record(main)
            stream.wait_event(ev_fork)
            with torch.cuda.stream(stream):
                wgrad()
            ev_join.record(stream)
        # both gradients on the Winograd form, one after the other: the input gradient's pass over dy also writes the
        # weight gradient's transformed dy (mvae_winograd_dy_transforms), instead of a second pass
        n_, c_, h_, w_ = x.shape
        dkeep = [] if (WINOGRAD_DY2 and side is None and dyb is None and ctx.needs_input_grad[0] and
                       ctx.needs_input_grad[1] and WINOGRAD_WGRAD and not g.pointwise and
                       (_wino_ok(g, n_, h_, w_, c_, w.shape[0]) or _wino_ups_ok(g, n_, h_, w_, c_, w.shape[0]))) else None
        acc = ctx.dx_sum
        if ctx.needs_input_grad[0] and acc is not None:
            # one of several 1x1 convs reading the same input: accumulate into the shared input gradient (every one of
            # them must take this branch, or the sum would never be returned)
            if not _al16(dy):
                dy = dy.clone(memory_format=CL)
            first = acc.buf is None
            if first:
                acc.buf = torch.empty(tuple(x.shape), device=dy.device, dtype=torch.float32, memory_format=CL)
            conv2d_dgrad_raw(dy, w, x.shape, g, out=acc.buf, beta=0.0 if first else 1.0)
            acc.left -= 1
            dx = None
            if acc.left == 0:  # (the last of them returns the sum; re-armed for a retained graph's next backward)
                dx, acc.buf, acc.left = acc.buf, None, acc.n
        elif ctx.needs_input_grad[0]:
            dx = conv2d_dgrad_raw(dy, w, x.shape, g, link if ctx.x_sink is None else None, dys=dys, dyb=dyb,
                                  dkeep=dkeep, u_pre=ctx.u_pre)
            if ctx.x_sink is not None and ctx.x_sink.park(dx):
                dx = None
        if side is not None:
            main.wait_event(ev_join)
        elif ctx.needs_input_grad[1]:
            wgrad()
        ctx.wino_v = dkeep = ctx.u_pre = None  # (released after the join: a later main-stream allocation is ordered after its last use)
        if ctx.has_bias and ctx.needs_input_grad[2] and not bias_done:
            tgt = _main_grad(ctx.bias_ref)
            n, co, ho, wo = dy.shape
            if tgt is not None:
                bias_grad_raw(dy.data_ptr(), n * ho * wo, co, tgt, 1.0, dy.device, _stream(dy))
            else:
                db_ret = torch.empty(co, device=dy.device, dtype=torch.float32)
                bias_grad_raw(dy.data_ptr(), n * ho * wo, co, db_ret, 0.0, dy.device, _stream(dy))
        if ctx.has_res and ctx.needs_input_grad[3]:
            dres = dy
            if ctx.res_sink is not None and ctx.res_sink.park(dy):
                dres = None
        if ctx.needs_input_grad[1] and dw_ret is None:
            _grad_done(ctx.weight_ref)
        if want_b and db_ret is None:
            _grad_done(ctx.bias_ref)
        return dx, dw_ret, db_ret, dres, None, None, None, None, None, None, None, None


# The GroupNorm statistics of a conv output emitted by its GEMM epilogue travel with the output tensor
# (with its version counter: an in-place change before the GroupNorm invalidates them).
GN_PART_ATTR = "_mvae_gn_part"
GN_FUSED_STATS = os.environ.get("MVAE_NO_GN_FUSED") is None and os.environ.get("MVAE_NO_VEC_EPI") is None


def _conv_macs(x, weight, geom: ConvGeom) -> float:
    n, c, h, w = x.shape
    ho, wo = geom.out_hw(h, w)
    return float(n) * ho * wo * weight.shape[0] * c * geom.kh * geom.kw


def conv2d(x, weight, bias, geom: ConvGeom, residual=None, res_sink=None, x_sink=None, gn_stats: bool = False,
           gn_bias: bool = False, dx_sum=None):
    """gn_stats=True: the output feeds a Normalize (encoder_decoder.py:28-33) -- emit its statistics from the
    conv's epilogue so the GroupNorm skips its statistics pass (plain implicit-GEMM convs only)."""
    part = None
    if gn_stats and GN_FUSED_STATS and not geom.pointwise and not _subpixel_upsample(geom) and x.shape[1] % 4 == 0:
        n, _, h, w = x.shape
        ho, wo = geom.out_hw(h, w)
        co = weight.shape[0]
        if (ho * wo) % 32 == 0 and co % 4 == 0 and _al16(x, weight) and (bias is None or _al16(bias)) and (
                residual is None or _al16(residual)):
            part = torch.empty(n * ho * wo // 32 * (co // 4) * 2, device=x.device, dtype=torch.float64)
    link = getattr(x, GN_BWD_ATTR, None)
    if link is not None and not link.matches(x):
        link = None
    dyp = None
    # (a Winograd conv of the bf16-mixed mode reads dy in fp32 or 3xBF16-split form, not packed: the GroupNorm backward
    # writes it split, as in the 3xBF16 mode)
    wino_any = x.dim() == 4 and _wino_ok(geom, x.shape[0], x.shape[2], x.shape[3], x.shape[1], weight.shape[0])
    wino_bf16 = _MATH[0] == 1 and wino_any
    # (a Winograd conv splits / rounds dy in its own memory-bound transform: the GroupNorm backward then writes no
    # second copy of dx, only the bias gradient)
    wino_fp32_dy = WINOGRAD_DY_FP32 and wino_any and not _subpixel_upsample(geom)
    if gn_stats and DYPACK and _dma_fmt() == 2 and not wino_bf16 and not geom.pointwise and weight.shape[0] % 8 == 0 and \
            geom.kh * geom.kw <= 32 and torch.is_grad_enabled():
        dyp = DyPack(bias)
        # (the LDS-DMA input / weight gradients read the packed copy; GroupNorm-partials epilogues and odd channel
        # counts fall back to kernels that read the fp32 dy)
        dyp.copy_ok = not GN_BWD_FUSED and x.shape[1] % 8 == 0 and not geom.upsample
    elif gn_stats and DYSPLIT and ((_dma_fmt() == 0 and _MATH[0] == 0) or wino_bf16) and not wino_fp32_dy and \
            not geom.pointwise and \
            not _subpixel_upsample(geom) and weight.shape[0] % 4 == 0 and geom.kh * geom.kw <= 32 and \
            torch.is_grad_enabled() and _conv_macs(x, weight, geom) >= DYSPLIT_MIN_MACS:
        dyp = DyPack(bias, split=True)
        dyp.copy_ok = not GN_BWD_FUSED  # (the 3xBF16 GEMMs and Winograd transforms read the split copy)
    elif (gn_stats or gn_bias) and DYBIAS and bias is not None and bias.requires_grad and torch.is_grad_enabled() and \
            x.dim() == 4 and weight.shape[0] % 4 == 0 and (
                (_MATH[0] == 2 and not _subpixel_upsample(geom) and wino_any) or wino_fp32_dy or
                _wino_ups_ok(geom, x.shape[0], x.shape[2], x.shape[3], x.shape[1], weight.shape[0])):
        # a Winograd conv reading dy in fp32 whose output feeds a GroupNorm: the bias gradient comes out of that
        # GroupNorm's backward (column sums of its dx) instead of a separate pass over dy
        dyp = DyPack(bias, split="bias")
    if dx_sum is not None and not (DX_SUM and geom.pointwise and torch.is_grad_enabled() and x_sink is None):
        dx_sum = None
    y = Conv2dFn.apply(x, weight, bias, residual, geom, res_sink, x_sink, part, link, dyp, torch.is_grad_enabled(),
                       dx_sum)
    if part is not None:
        setattr(y, GN_PART_ATTR, (part, y._version))
    if dyp is not None:
        setattr(y, DYPACK_ATTR, (dyp, y._version))
    return y


# ------------------------------------------------------------------------------------------
# GroupNorm (+SiLU, +dropout)
# ------------------------------------------------------------------------------------------
# A GroupNorm output that feeds exactly one convolution carries a GnBwdLink: the conv's input-gradient GEMM
# emits the GroupNorm backward partials from its epilogue (mvae_conv2d_dgrad_gnbwd_nhwc) and the GroupNorm
# backward then skips its reduction pass over x and dy (mvae_group_norm_bwd_part_nhwc).
GN_BWD_ATTR = "_mvae_gn_bwd_link"
# Opt-in (MVAE_GN_BWD_FUSED=1): since the streaming GroupNorm kernels use non-temporal loads the separate reduction
# pass is cheaper than the epilogue work it saves -- c4 same-box A/B: dgrad 397 -> 433 TF/s, step +0.9 % unfused.
GN_BWD_FUSED = os.environ.get("MVAE_GN_BWD_FUSED") is not None and os.environ.get("MVAE_NO_VEC_EPI") is None


class GnBwdLink:
    __slots__ = ("x", "gamma", "beta", "mean", "rstd", "groups", "silu", "y_ref", "y_version", "part", "dx")

    def __init__(self, groups: int, silu: bool):
        self.groups, self.silu = groups, int(silu)
        self.x = self.gamma = self.beta = self.mean = self.rstd = None
        self.y_ref = self.y_version = self.part = self.dx = None

    def bind_output(self, y):
        self.y_ref, self.y_version = y.data_ptr(), y._version

    def matches(self, x) -> bool:  # the conv input is still the GroupNorm's untouched output
        return self.x is not None and x.data_ptr() == self.y_ref and x._version == self.y_version

    def usable(self, dx) -> bool:
        n, c, h, w = dx.shape
        return (self.x is not None and tuple(self.x.shape) == (n, c, h, w) and (h * w) % 32 == 0 and
                c % self.groups == 0 and (c // self.groups) % 4 == 0 and _al16(self.x))

    def take(self, dy):
        """The emitted partials, if they were computed from exactly this gradient tensor."""
        part, dx = self.part, self.dx
        self.part = self.dx = None
        if part is None or dx is None or dy.data_ptr() != dx.data_ptr() or dy.shape != dx.shape or \
                not dy.is_contiguous(memory_format=CL):
            return None
        return part


class GroupNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, groups: int, eps: float, silu: bool, drop_p: float, seed: int,
                y_split: bool = False, grad_sink=None, part=None, link=None, dypack=None, lazy=None,
                conv_dy_only: bool = False):
        _check(x, "group_norm input")
        x = nhwc(x)
        n, c, h, w = x.shape
        mean = torch.empty(n * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        nbytes = _lib.query("mvae_group_norm_workspace_bytes", n, h * w, c)
        ws = ARENA.get("gn", nbytes, x.device)
        if lazy is not None:  # statistics only; the consuming conv's input transform applies them (LazyGn)
            lazy.x = x
            lazy.scale = torch.empty(n * c, device=x.device, dtype=torch.float32)
            lazy.shift = torch.empty_like(lazy.scale)
            with _timed("gn_fwd", 0.0 if part is not None else 4.0 * x.numel(), (n, c, h * w)):
                _lib.call("mvae_group_norm_stats_nhwc", x.data_ptr(), _ptr(part), gamma.data_ptr(), beta.data_ptr(),
                          mean.data_ptr(), rstd.data_ptr(), lazy.scale.data_ptr(), lazy.shift.data_ptr(), n, h * w, c,
                          groups, float(eps), ws.data_ptr(), ws.numel(), _stream(x))
            # (group_norm hands it on as a DeferredGnOutput: never read, any read raises)
            y = torch.full((1,), float("nan"), device=x.device).expand(n, c, h, w)
        else:
            y = torch.empty_like(x, memory_format=CL)
            with _timed("gn_fwd", 8.0 * x.numel(), (n, c, h * w)):  # algorithmic HBM bytes: read x, write y
                if part is not None:  # statistics from the producing conv's epilogue: no pass over x for them
                    _lib.call("mvae_group_norm_fwd_part_nhwc", x.data_ptr(), part.data_ptr(), gamma.data_ptr(),
                              beta.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), n, h * w, c, groups,
                              float(eps), int(silu), float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, int(y_split),
                              ws.data_ptr(), ws.numel(), _stream(x))
                else:
                    _lib.call("mvae_group_norm_fwd_nhwc", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                              y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), n, h * w, c, groups, float(eps),
                              int(silu), float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF, int(y_split), ws.data_ptr(),
                              ws.numel(), _stream(x))
        ctx.save_for_backward(x, gamma, beta, mean, rstd)
        ctx.cfg = (groups, int(silu), float(drop_p), int(seed) & 0xFFFFFFFFFFFFFFFF)
        ctx.gamma_ref, ctx.beta_ref = gamma, beta
        ctx.grad_sink = grad_sink
        ctx.link = link
        ctx.dypack = dypack
        ctx.conv_dy_only = conv_dy_only
        if link is not None:
            link.x, link.gamma, link.beta, link.mean, link.rstd = x, gamma, beta, mean, rstd
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mean, rstd = ctx.saved_tensors
        groups, silu, drop_p, seed = ctx.cfg
        dy = nhwc(dy)
        n, c, h, w = x.shape
        dx = torch.empty_like(x, memory_format=CL)
        dg_ret = db_ret = None
        dg = _main_grad(ctx.gamma_ref) if ctx.needs_input_grad[1] else None
        db = _main_grad(ctx.beta_ref) if ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[1] and dg is None:
            dg = dg_ret = torch.zeros(c, device=x.device, dtype=torch.float32)
        if ctx.needs_input_grad[2] and db is None:
            db = db_ret = torch.zeros(c, device=x.device, dtype=torch.float32)
        nbytes = _lib.query("mvae_group_norm_workspace_bytes", n, h * w, c)
        ws = ARENA.get("gn", nbytes, x.device)
        add = ctx.grad_sink.take() if ctx.grad_sink is not None else None
        if add is not None:
            add = nhwc(add)
            if add.shape != x.shape or add.dtype != torch.float32:
                raise RuntimeError("group_norm backward: parked branch gradient has the wrong shape")
        gpart = ctx.link.take(dy) if ctx.link is not None and drop_p == 0.0 else None
        # algorithmic HBM bytes: read x, dy (and the residual branch's gradient when it is summed here); write dx
        req = ctx.dypack if ctx.dypack is not None and _al16(dy, dx) and (add is None or _al16(add)) else None
        if req is not None and gpart is not None and req.split is False:
            req = None  # (the backward from the conv's partials writes split4 dy or the bias column sums only)
        bias_only = req is not None and req.split == "bias"
        if bias_only and not (req.bias_ref is not None and req.bias_ref.requires_grad):
            req = None
        packed = tgt = cs = None
        if bias_only and req is not None:
            tgt = req.db = torch.empty(c, device=x.device, dtype=torch.float32)
            csb = _lib.query("mvae_group_norm_colsum_workspace_bytes", n, h * w, c)
            cs = ARENA.get("gncs", csb, x.device)
            packed = True  # (DyPack.take's "produced" mark: no second copy of dx)
        elif req is not None:
            # also dx as packed bf16 / split4 and the producing conv's bias gradient (DyPack)
            # packed bf16: 2 B per element; split4_bf16: 4 B per element, dx's layout (an fp32-sized buffer)
            packed = (torch.empty_like(x, memory_format=CL) if req.split else
                      torch.empty(x.numel() * 2, device=x.device, dtype=torch.uint8))
            bref = req.bias_ref
            if bref is not None and bref.requires_grad:
                # a private buffer, never the flat gradient slot: the conv adds it there only if DyPack.take()
                # accepts dy (a rejected dy -- another branch summed in by autograd -- gets its bias gradient from
                # the real dy instead, and nothing partial is left in the slot)
                tgt = req.db = torch.empty(c, device=x.device, dtype=torch.float32)
            csb = _lib.query("mvae_group_norm_colsum_workspace_bytes", n, h * w, c)
            cs = ARENA.get("gncs", csb, x.device) if tgt is not None else None
        # x is the output of the conv that requested the copy and has no other consumer: that conv reads the copy alone,
        # so the fp32 dx is left unwritten (its buffer is still autograd's gradient object)
        nodx = bool(ctx.conv_dy_only and DX_COPY_ONLY and req is not None and not bias_only and req.copy_ok)
        dxp = None if nodx else dx.data_ptr()
        if nodx and DX_POISON:
            dx.fill_(float("nan"))  # (test aid: any kernel that still reads the unwritten dx turns the step NaN)
        with _timed("gn_bwd", (12.0 + (4.0 if add is not None else 0.0)) * x.numel(), (n, c, h * w)):
            if gpart is not None and req is not None:  # reduction half from the conv + the conv's split dy / bias
                _lib.call("mvae_group_norm_bwd_part_split_nhwc", x.data_ptr(), dy.data_ptr(), gpart.data_ptr(),
                          gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dxp,
                          _ptr(add), _ptr(dg), _ptr(db), n, h * w, c, groups, silu, ws.data_ptr(), ws.numel(),
                          None if bias_only else packed.data_ptr(), _ptr(tgt), 0.0, _ptr(cs),
                          cs.numel() if cs is not None else 0, _stream(x))
            elif gpart is not None:  # reduction half emitted by the consuming conv's input-gradient GEMM
                _lib.call("mvae_group_norm_bwd_part_nhwc", x.data_ptr(), dy.data_ptr(), gpart.data_ptr(),
                          gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                          _ptr(add), _ptr(dg), _ptr(db), n, h * w, c, groups, silu, ws.data_ptr(), ws.numel(),
                          _stream(x))
            elif bias_only and req is not None:
                _lib.call("mvae_group_norm_bwd_colsum_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(),
                          beta.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), _ptr(add), _ptr(dg),
                          _ptr(db), n, h * w, c, groups, silu, drop_p, seed, ws.data_ptr(), ws.numel(), tgt.data_ptr(),
                          0.0, cs.data_ptr(), cs.numel(), _stream(x))
            elif req is not None:
                _lib.call("mvae_group_norm_bwd_split_nhwc" if req.split else "mvae_group_norm_bwd_pack_nhwc",
                          x.data_ptr(), dy.data_ptr(), gamma.data_ptr(),
                          beta.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dxp, _ptr(add), _ptr(dg),
                          _ptr(db), n, h * w, c, groups, silu, drop_p, seed, ws.data_ptr(), ws.numel(),
                          packed.data_ptr(), _ptr(tgt), 0.0, _ptr(cs), cs.numel() if cs is not None else 0,
                          _stream(x))
            else:
                _lib.call("mvae_group_norm_bwd_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                          mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), _ptr(add), _ptr(dg), _ptr(db), n, h * w,
                          c, groups, silu, drop_p, seed, ws.data_ptr(), ws.numel(), _stream(x))
        if req is not None:
            req.packed, req.dx_ref, req.dx_version, req.dx_shape = packed, weakref.ref(dx), dx._version, \
                tuple(dx.shape)
            req.bias_done = tgt is not None
            req.nodx = nodx
        if ctx.needs_input_grad[1] and dg_ret is None:
            _grad_done(ctx.gamma_ref)
        if ctx.needs_input_grad[2] and db_ret is None:
            _grad_done(ctx.beta_ref)
        return dx, dg_ret, db_ret, None, None, None, None, None, None, None, None, None, None, None, None


# Activations handed to a convolution in the pre-split 3xBF16 operand layout carry this attribute
# (the bytes are bf16 hi/lo pairs, not fp32 values): only Conv2dFn consumes them.
XSPLIT_ATTR = "_mvae_xsplit"
ACT_SPLIT = os.environ.get("MVAE_NO_ACT_SPLIT") is None
# bf16-mixed mode: a GroupNorm output whose consuming conv runs on packed bf16 operands (MVAE_CONV_BF16) is written
# packed (2 B per element in the first half of the fp32 tensor's bytes); only Conv2dFn consumes it, forward and
# weight gradient reading the same bytes
BF16_ATTR = "_mvae_bf16"


# A GroupNorm whose input is a conv output with no other consumer (ResnetBlock norm2 of conv1's output, conv_dy_only):
# when that conv takes its output gradient as the split / packed copy the backward writes, the fp32 dx is not written.
# MVAE_NO_DX_COPY_ONLY=1: always written.
DX_COPY_ONLY = os.environ.get("MVAE_NO_DX_COPY_ONLY") is None
DX_POISON = os.environ.get("MVAE_DX_POISON") == "1"  # tests: fill the unwritten dx with NaN


def group_norm(x, gamma, beta, groups, eps=1e-6, silu=False, drop_p=0.0, seed=0, for_conv=False, grad_sink=None,
               conv_dy_only: bool = False):
    """for_conv (True, or the consuming conv's output channel count): the caller feeds the result straight into
    ops.conv2d (3x3/stride-1, C % 4 == 0) -- the output is then written pre-split for the GEMM (GroupNorm -> conv is
    the ResnetBlock / norm_out pattern, encoder_decoder.py:141-163, :318-328); in the bf16-mixed mode, with a known
    output channel count that is a multiple of 8, packed bf16 for the LDS-DMA GEMM."""
    packed = bool(for_conv and not isinstance(for_conv, bool) and int(for_conv) % 8 == 0 and _bf16_dma() and
                  x.shape[1] % 8 == 0 and _al16(x) and _dma_ok(9.0 * x.numel() * int(for_conv)) and
                  not (x.dim() == 4 and _wino_ok(G3, x.shape[0], x.shape[2], x.shape[3], x.shape[1], int(for_conv))))
    split = _dma_fmt() if packed else int(bool(for_conv and ACT_SPLIT and _splits_ok() and not _bf16_dma() and
                                                x.shape[1] % 4 == 0))
    part = getattr(x, GN_PART_ATTR, None)
    if part is not None:
        delattr(x, GN_PART_ATTR)  # consumed once; frees the statistics with the next allocation cycle
        h, w = x.shape[2], x.shape[3]
        ok = part[1] == x._version and (h * w) % 32 == 0 and (x.shape[1] // groups) % 4 == 0 and \
            x.shape[1] % groups == 0 and x.is_contiguous(memory_format=CL)
        part = part[0] if ok else None
    link = GnBwdLink(groups, silu) if (for_conv and GN_BWD_FUSED and drop_p == 0.0 and x.requires_grad) else None
    dyp = getattr(x, DYPACK_ATTR, None)
    if dyp is not None:
        delattr(x, DYPACK_ATTR)  # one GroupNorm per conv output
        dyp = dyp[0] if dyp[1] == x._version and x.is_contiguous(memory_format=CL) and _al16(x) else None
    lazy = None
    if (WINOGRAD_GN and for_conv and not isinstance(for_conv, bool) and drop_p == 0.0 and not packed and
            x.dim() == 4 and _al16(x) and WINOGRAD_WGRAD):
        n, c, h, w = x.shape
        if _wino_ok(G3, n, h, w, c, int(for_conv)):  # (the consuming conv is 3x3 / stride 1 / pad 1: for_conv callers)
            lazy, split = LazyGn(x, silu), 0
            # the conv's Winograd input-gradient output transform also emits this GroupNorm's backward partials
            # (mvae_winograd_output_gnbwd: one extra read of x there) where the backward would otherwise make a partial
            # pass over x and dy (its streaming chain: the large levels, whose producing conv takes dy pre-split)
            if (link is None and WINOGRAD_GN_LINK and x.requires_grad and dyp is not None and dyp.split is not False and
                    _wino_blocks(h, w) and c % groups == 0 and (c // groups) % 4 == 0 and
                    _lib.query("mvae_group_norm_bwd_streaming", n, h * w, c, groups, 1)):
                link = GnBwdLink(groups, silu)
    y = GroupNormFn.apply(x, gamma, beta, groups, eps, silu, drop_p, seed, split, grad_sink, part, link, dyp, lazy,
                          conv_dy_only)
    if lazy is not None:
        y = y.as_subclass(DeferredGnOutput)  # (same autograd node; any read of its values raises)
        setattr(y, GN_LAZY_ATTR, lazy)
    elif split >= 2:
        setattr(y, BF16_ATTR, True)
    elif split:
        setattr(y, XSPLIT_ATTR, True)
    if link is not None:
        link.bind_output(y)
        setattr(y, GN_BWD_ATTR, link)
    return y


# ------------------------------------------------------------------------------------------
# attention core: softmax(q k^T * C^-1/2) v over the h*w tokens of each image
# ------------------------------------------------------------------------------------------
def _gemm(ta, tb, m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, st, residual=None):
    with _timed("attn_gemm", 2.0 * m * n * k * batch, (m, n, k, batch)):
        _lib.call("mvae_gemm_strided_batched", ta, tb, m, n, k, float(alpha), A.data_ptr(), lda, sA, B.data_ptr(), ldb,
                  sB, float(beta), C.data_ptr(), ldc, sC, batch, None, _ptr(residual), ldc, sC, None, 0, st)


ATTN_SMALL_MAXN = 64
ATTN_FUSED = os.environ.get("MVAE_NO_ATTN_FUSED") is None


# the fused kernel runs one workgroup per image, so its K loops are latency-bound once C is large: measured
# (tools/attn_bench.py, profiles/r04_attn_bench.txt) faster than the unfused path at 7x7x128 / 7x7x512 (c3 / c2:
# fwd 1.7x / 1.1x) and slower at 8x8x2048 (c4 / c5: fwd 162 vs 137 us, bwd 380 vs 279 us) -- used up to this C
ATTN_FUSED_MAXC = 512


def _attn_small_ok(q, n: int, c: int) -> bool:
    """the fused kernel's shape / alignment contract (and not switched off)"""
    return ATTN_FUSED and n <= ATTN_SMALL_MAXN and c % 64 == 0 and _al16(q)


def _attn_use_fused(q, n: int, c: int) -> bool:
    return _attn_small_ok(q, n, c) and c <= ATTN_FUSED_MAXC


# query-block fused attention (csrc/attn_tile.hip) for 64 <= n <= 256 tokens, n % 64 == 0, C % 128 == 0: c4 / c5's
# 16x16 level (n = 256, C = 1024) and, past ATTN_FUSED_MAXC, the 8x8 mid blocks (n = 64, C = 2048). Forward one launch
# (scores, softmax and P V in one workgroup per 64 queries; P saved for the backward); backward one launch for dP, dS and
# dQ plus the two batched GEMMs dV = P^T dO and dK = dS^T Q. Opt-in (MVAE_ATTN_TILE=1): measured at c4's 16x16x1024
# (tools/attn_bench.py, profiles/r05_attn_bench.txt) it is slower than the unfused path -- fwd 513 vs 366 us, bwd 847 vs
# 704 us: one 141 KB workgroup per CU walks 96 short K-tiles (12-24 MFMAs per wave each) behind one tile of prefetch, so
# every K-tile waits on a global load; the batched GEMMs' 256x256 tiles do not
ATTN_TILE = os.environ.get("MVAE_ATTN_TILE") is not None


def _attn_use_tile(q, n: int, c: int) -> bool:
    return ATTN_TILE and 64 <= n <= 256 and n % 64 == 0 and c % 128 == 0 and _al16(q) and q.shape[0] <= 65535


class AttnCoreFn(torch.autograd.Function):
    """softmax(q k^T * C^-1/2, dim=2) v over the h*w tokens of each image (encoder_decoder.py:90-103). n <= 64 (the
    7x7 / 8x8 mid blocks): the fused single-tile kernels, one launch per direction with the scores in LDS and only the
    row log-sum-exp saved (csrc/attn.hip); larger n (c4 / c5's 16x16 level): two batched GEMMs around a row softmax."""

    @staticmethod
    def forward(ctx, q, k, v):
        q, k, v = nhwc(q), nhwc(k), nhwc(v)
        b, c, h, w = q.shape
        n = h * w
        st = _stream(q)
        scale = float(c) ** -0.5
        ctx.scale = scale
        ctx.math = _MATH[0]
        if _attn_use_fused(q, n, c):
            o = torch.empty_like(q, memory_format=CL)
            lse = torch.empty((b, ATTN_SMALL_MAXN), device=q.device, dtype=torch.float32)
            fl = 4.0 * n * n * c * b  # S = Q K^T and O = P V
            with _timed("attn_gemm", fl, (n, c, n, b)):
                _lib.call("mvae_attention_small_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                          lse.data_ptr(), b, n, c, scale, st)
            ctx.save_for_backward(q, k, v, lse)
            ctx.fused = True
            return o
        ctx.fused = False
        s = torch.empty((b, n, n), device=q.device, dtype=torch.float32)
        ctx.tile = _attn_use_tile(q, n, c)
        if ctx.tile:  # S, softmax and P V in one launch; P (s) saved for the backward
            o = torch.empty_like(q, memory_format=CL)
            with _timed("attn_gemm", 4.0 * n * n * c * b, (n, c, n, b)):
                _lib.call("mvae_attention_tile_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                          s.data_ptr(), b, n, c, scale, st)
            ctx.save_for_backward(q, k, v, s)
            return o
        _gemm(0, 1, n, n, c, scale, q, c, n * c, k, c, n * c, 0.0, s, n, n * n, b, st)
        _lib.call("mvae_softmax_rows", s.data_ptr(), s.data_ptr(), b * n, n, st)
        o = torch.empty_like(q, memory_format=CL)
        _gemm(0, 0, n, c, n, 1.0, s, n, n * n, v, c, n * c, 0.0, o, c, n * c, b, st)
        ctx.save_for_backward(q, k, v, s)
        return o

    @staticmethod
    def backward(ctx, do):
        with math_scope(ctx.math):
            return AttnCoreFn._backward(ctx, do)

    @staticmethod
    def _backward(ctx, do):
        q, k, v, p = ctx.saved_tensors
        do = nhwc(do)
        b, c, h, w = q.shape
        n = h * w
        st = _stream(q)
        if ctx.fused:  # p = the row log-sum-exp; the kernel recomputes the scores
            if not (do.is_contiguous(memory_format=CL) and _al16(do)):
                do = do.contiguous(memory_format=CL)
            dq = torch.empty_like(q, memory_format=CL)
            dk = torch.empty_like(k, memory_format=CL)
            dv = torch.empty_like(v, memory_format=CL)
            # algorithm: S and dP (recomputed S, dO V^T) + dV, dQ, dK; reference: dP, dV, dQ, dK
            with _timed("attn_gemm", 10.0 * n * n * c * b, (n, c, n, b), 8.0 * n * n * c * b):
                _lib.call("mvae_attention_small_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), do.data_ptr(),
                          p.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), b, n, c, ctx.scale, st)
            return dq, dk, dv
        if ctx.tile:
            if not (do.is_contiguous(memory_format=CL) and _al16(do)):
                do = do.contiguous(memory_format=CL)
            dq = torch.empty_like(q, memory_format=CL)
            ds = torch.empty((b, n, n), device=q.device, dtype=torch.float32)
            with _timed("attn_gemm", 4.0 * n * n * c * b, (n, c, n, b)):  # dP = dO V^T, dQ = dS K
                _lib.call("mvae_attention_tile_bwd", k.data_ptr(), v.data_ptr(), do.data_ptr(), p.data_ptr(),
                          dq.data_ptr(), ds.data_ptr(), b, n, c, ctx.scale, st)
            dv = torch.empty_like(v, memory_format=CL)
            _gemm(1, 0, n, c, n, 1.0, p, n, n * n, do, c, n * c, 0.0, dv, c, n * c, b, st)  # dV = P^T dO
            dk = torch.empty_like(k, memory_format=CL)
            _gemm(1, 0, n, c, n, 1.0, ds, n, n * n, q, c, n * c, 0.0, dk, c, n * c, b, st)  # dK = dS^T Q (scale in dS)
            return dq, dk, dv
        dp = torch.empty((b, n, n), device=q.device, dtype=torch.float32)
        _gemm(0, 1, n, n, c, 1.0, do, c, n * c, v, c, n * c, 0.0, dp, n, n * n, b, st)   # dP = dO V^T
        dv = torch.empty_like(v, memory_format=CL)
        _gemm(1, 0, n, c, n, 1.0, p, n, n * n, do, c, n * c, 0.0, dv, c, n * c, b, st)   # dV = P^T dO
        _lib.call("mvae_softmax_rows_bwd", p.data_ptr(), dp.data_ptr(), dp.data_ptr(), b * n, n, st)  # dS
        dq = torch.empty_like(q, memory_format=CL)
        _gemm(0, 0, n, c, n, ctx.scale, dp, n, n * n, k, c, n * c, 0.0, dq, c, n * c, b, st)  # dQ = dS K
        dk = torch.empty_like(k, memory_format=CL)
        _gemm(1, 0, n, c, n, ctx.scale, dp, n, n * n, q, c, n * c, 0.0, dk, c, n * c, b, st)  # dK = dS^T Q
        return dq, dk, dv


def attention_core(q, k, v):
    return AttnCoreFn.apply(q, k, v)


# ------------------------------------------------------------------------------------------
# reparameterization, KL, reconstruction
# ------------------------------------------------------------------------------------------
def _pixel_ld(t: torch.Tensor) -> Optional[int]:
    """Row stride between consecutive pixels for a logical-NCHW tensor whose channels are
    contiguous; None if the tensor is not laid out that way."""
    n, c, h, w = t.shape
    if t.stride(1) != 1 and c > 1:
        return None
    ld = t.stride(3) if w > 1 else (t.stride(2) if h > 1 else (t.stride(0) if n > 1 else c))
    if w > 1 and t.stride(3) != ld:
        return None
    if h > 1 and t.stride(2) != w * ld:
        return None
    if n > 1 and t.stride(0) != h * w * ld:
        return None
    return ld


def _pix(t):
    ld = _pixel_ld(t)
    if ld is None:
        t = nhwc(t)
        ld = t.shape[1]
    return t, ld


class ReparamFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mean, logvar, eps):
        _check(mean, "mean")
        mean, ldm = _pix(mean)
        logvar, ldl = _pix(logvar)
        eps = nhwc(eps)
        n, zc, h, w = mean.shape
        z = torch.empty((n, zc, h, w), device=mean.device, dtype=torch.float32, memory_format=CL)
        if ldm != ldl:
            mean, logvar = nhwc(mean.contiguous()), nhwc(logvar.contiguous())
            ldm = ldl = zc
        with _timed("loss_fwd", 16.0 * z.numel(), ("reparam", n * h * w, zc)):  # read mu, logvar, eps; write z
            _lib.call("mvae_reparam_fwd", mean.data_ptr(), logvar.data_ptr(), ldm, eps.data_ptr(), z.data_ptr(),
                      n * h * w, zc, _stream(mean))
        ctx.save_for_backward(logvar, eps)
        ctx.ld = ldl
        return z

    @staticmethod
    def backward(ctx, dz):
        logvar, eps = ctx.saved_tensors
        dz = nhwc(dz)
        n, zc, h, w = dz.shape
        dlv = None
        if ctx.needs_input_grad[1]:
            dlv = torch.empty((n, zc, h, w), device=dz.device, dtype=torch.float32, memory_format=CL)
            with _timed("loss_bwd", 16.0 * dz.numel(), ("reparam", n * h * w, zc)):  # read dz, eps, logvar; write dlv
                _lib.call("mvae_reparam_bwd", dz.data_ptr(), eps.data_ptr(), logvar.data_ptr(), ctx.ld, dlv.data_ptr(),
                          n * h * w, zc, _stream(dz))
        return (dz if ctx.needs_input_grad[0] else None), dlv, None


def reparameterize(mean, logvar, eps):
    return ReparamFn.apply(mean, logvar, eps)


class LatentPrepFn(torch.autograd.Function):
    """The disentangled model's latent side in one launch per direction (mvae_latent_prep_fwd / _bwd): encode's NaN
    scrub + forward's clamps of mu / logvar (disentangled_conditional_vae.py:388-398), the reparameterization
    (base_vae.py:83-87) and the posterior's clamped std. h = the encoder output [n, 2 zc, hh, ww] (mean channels
    first, torch.chunk); the backward writes h's gradient directly (no chunk / accumulation launches)."""

    @staticmethod
    def forward(ctx, h, eps, zc: int):
        _check(h, "encoder output")
        if h.dim() != 4 or h.shape[1] != 2 * zc:
            raise RuntimeError(f"latent_prep: expected an encoder output [n, {2 * zc}, h, w], got {tuple(h.shape)}")
        h, ld = _pix(h)
        eps = nhwc(eps)
        n, _, hh, ww = h.shape
        outs = [torch.empty((n, zc, hh, ww), device=h.device, dtype=torch.float32, memory_format=CL) for _ in range(4)]
        mu, lv, sd, z = outs
        _lib.call("mvae_latent_prep_fwd", h.data_ptr(), h.data_ptr() + 4 * zc, ld, eps.data_ptr(), mu.data_ptr(),
                  lv.data_ptr(), sd.data_ptr(), z.data_ptr(), n * hh * ww, zc, _stream(h))
        ctx.save_for_backward(h, eps)
        ctx.ld, ctx.zc = ld, zc
        return mu, lv, sd, z

    @staticmethod
    def backward(ctx, gmu, glv, gsd, gz):
        h, eps = ctx.saved_tensors
        zc, ld = ctx.zc, ctx.ld
        n, c2, hh, ww = h.shape
        dh = torch.empty((n, c2, hh, ww), device=h.device, dtype=torch.float32, memory_format=CL)  # fully written
        gs = [None if g is None else nhwc(g.float()) for g in (gmu, glv, gsd, gz)]
        _lib.call("mvae_latent_prep_bwd", h.data_ptr(), h.data_ptr() + 4 * zc, ld, eps.data_ptr(),
                  *[_ptr(g) for g in gs], dh.data_ptr(), dh.data_ptr() + 4 * zc, c2, n * hh * ww, zc, _stream(h))
        return dh, None, None


def latent_prep(h, zc: int, eps):
    """(mu, logvar, std, z) of the disentangled forward from the encoder output h (see LatentPrepFn)."""
    return LatentPrepFn.apply(h, eps, int(zc))


class LossCombineFn(torch.autograd.Function):
    """DisentangledVAELoss's combination of its scalar terms (disentangled_conditional_vae.py:528-570) in one launch
    per direction: each term replaced by 0 when non-finite, the weighted sum in order, the total replaced by
    `nonfinite_total` when non-finite (mvae_loss_combine4_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, weights, nonfinite_total, *terms):
        nt = len(terms)
        dev = terms[0].device
        outs = [torch.empty((), device=dev, dtype=torch.float32) for _ in range(nt + 1)]  # total, terms
        flags = torch.empty(nt + 1, device=dev, dtype=torch.float32)
        tp = [t.detach().float().contiguous() for t in terms]
        ptrs = [t.data_ptr() for t in tp] + [None] * (4 - nt)
        optr = [o.data_ptr() for o in outs] + [None] * (4 - nt)
        w = list(map(float, weights)) + [0.0] * (4 - nt)
        _lib.call("mvae_loss_combine4_fwd", *ptrs, *w, nt, float(nonfinite_total), *optr, flags.data_ptr(),
                  _stream(terms[0]))
        ctx.w, ctx.nt = w, nt
        ctx.save_for_backward(flags)  # freed with the graph; a retained graph can run its backward again
        return tuple(outs)

    @staticmethod
    def backward(ctx, gtot, *gterms):
        nt = ctx.nt
        (flags,) = ctx.saved_tensors
        dev = flags.device
        gt = None if gtot is None else gtot.float().contiguous()
        gs = [None if g is None else g.float().contiguous() for g in gterms] + [None] * (4 - nt)
        out = torch.empty(nt, device=dev, dtype=torch.float32)
        _lib.call("mvae_loss_combine4_bwd", flags.data_ptr(), *ctx.w, nt, _ptr(gt), *[_ptr(g) for g in gs],
                  out.data_ptr(), _stream(out))
        return (None, None, *[out[i] for i in range(nt)])


def loss_combine(terms, weights, nonfinite_total: float = 1e6):
    """(total, *finite_or_zero(terms)) of DisentangledVAELoss (see LossCombineFn); up to 4 0-d device terms."""
    if not 1 <= len(terms) <= 4 or len(weights) != len(terms):
        raise ValueError("loss_combine: 1-4 terms with one weight each")
    return LossCombineFn.apply(tuple(weights), float(nonfinite_total), *terms)


class KLFn(torch.autograd.Function):
    """kind 0: mean over elements of KL(N(mu, e^{lv/2}) || N(0,1));
    kind 3: -0.5*sum(1+lv-mu^2-e^lv) / denom (DisentangledVAELoss)."""

    @staticmethod
    def forward(ctx, mean, logvar, kind: int, denom: float):
        mean, ldm = _pix(mean)
        logvar, ldl = _pix(logvar)
        if ldm != ldl:
            mean, logvar = nhwc(mean.contiguous()), nhwc(logvar.contiguous())
            ldm = ldl = mean.shape[1]
        n, zc, h, w = mean.shape
        out = torch.empty((), device=mean.device, dtype=torch.float32)
        ws = ARENA.get("red", _lib.query("mvae_reduce_workspace_bytes"), mean.device)
        scale = (1.0 / denom) if kind == 0 else (-0.5 / denom)
        with _timed("loss_fwd", 8.0 * n * h * w * zc, ("kl", n * h * w, zc)):  # read mu, logvar
            _lib.call("mvae_loss_reduce", kind, mean.data_ptr(), logvar.data_ptr(), ldm, n * h * w, zc, scale,
                      out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(mean))
        ctx.save_for_backward(mean, logvar)
        ctx.ld, ctx.denom = ldm, denom
        return out

    @staticmethod
    def backward(ctx, g):
        mean, logvar = ctx.saved_tensors
        g = g.contiguous().float()
        n, zc, h, w = mean.shape
        dmu = torch.empty((n, zc, h, w), device=mean.device, dtype=torch.float32, memory_format=CL)
        dlv = torch.empty_like(dmu, memory_format=CL)
        with _timed("loss_bwd", 16.0 * dmu.numel(), ("kl", n * h * w, zc)):  # read mu, logvar; write dmu, dlogvar
            _lib.call("mvae_kl_bwd", mean.data_ptr(), logvar.data_ptr(), ctx.ld, g.data_ptr(), 1.0 / ctx.denom,
                      dmu.data_ptr(), dlv.data_ptr(), n * h * w, zc, _stream(mean))
        return dmu, dlv, None, None


def kl_standard_normal_mean(mean, logvar):
    return KLFn.apply(mean, logvar, 0, float(mean.numel()))


def kl_closed_form_sum(mean, logvar, denom):
    return KLFn.apply(mean, logvar, 3, float(denom))


class ReconFn(torch.autograd.Function):
    """mean((a-b)^2) (kind 1) or mean|a-b| (kind 2); gradient w.r.t. a only."""

    @staticmethod
    def forward(ctx, a, b, kind: int):
        _check(a, "reconstruction")
        a = nhwc(a)
        b = nhwc(b.to(device=a.device, dtype=torch.float32))
        out = torch.empty((), device=a.device, dtype=torch.float32)
        ws = ARENA.get("red", _lib.query("mvae_reduce_workspace_bytes"), a.device)
        n = a.numel()
        with _timed("loss_fwd", 8.0 * n, ("recon", n)):  # read reconstruction, target
            _lib.call("mvae_loss_reduce", kind, a.data_ptr(), b.data_ptr(), 1, n, 1, 1.0 / n, out.data_ptr(),
                      ws.data_ptr(), ws.numel(), _stream(a))
        ctx.save_for_backward(a, b)
        ctx.kind = kind
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous().float()
        da = torch.empty_like(a, memory_format=CL) if a.dim() == 4 else torch.empty_like(a)
        with _timed("loss_bwd", 12.0 * a.numel(), ("recon", a.numel())):  # read reconstruction, target; write da
            _lib.call("mvae_recon_bwd", ctx.kind, a.data_ptr(), b.data_ptr(), g.data_ptr(), 1.0 / a.numel(),
                      da.data_ptr(), a.numel(), _stream(a))
        return da, None, None


class _FiniteGateFn(torch.autograd.Function):
    """v = fn(*inputs); the input gradients are handed back only if v was finite (device-side flag, no host
    sync). This is the reference's `if isnan(v) or isinf(v): v = tensor(0.)` (disentangled_conditional_vae.py:
    528-550): a non-finite term is cut out of the graph, so its backward can never inject 0*inf = NaN into the
    shared encoder gradients. fn runs once, under autograd on detached inputs; its small sub-graph (the [B, 8]
    latent statistics of the separation / contrastive terms) is kept for the backward instead of recomputed."""

    @staticmethod
    def forward(ctx, fn, *inputs):
        need = ctx.needs_input_grad[1:]
        with torch.enable_grad():
            req = [t.detach().requires_grad_(bool(n)) if torch.is_tensor(t) else t for t, n in zip(inputs, need)]
            v = fn(*req)
        ctx.v, ctx.req = v, req
        ok = torch.isfinite(v.detach())
        ctx.ok = ok.all() if ok.dim() else ok  # (a 0-d term needs no reduction launch)
        return v.detach()

    @staticmethod
    def backward(ctx, g):
        req, v = ctx.req, ctx.v
        ctx.v = ctx.req = None
        want = [r for r in req if torch.is_tensor(r) and r.requires_grad]
        got = list(torch.autograd.grad(v, want, g, allow_unused=True)) if want and v.requires_grad else \
            [None] * len(want)
        out = []
        for r in req:
            gr = got.pop(0) if torch.is_tensor(r) and r.requires_grad else None
            if gr is not None:
                gr = torch.where(ctx.ok, gr, 0.0)  # (scalar other: no fill launch)
            out.append(gr)
        return (None, *out)


def finite_gated(fn, *inputs):
    """fn(*inputs) as a loss term whose gradient is dropped when its value is NaN/Inf."""
    return _FiniteGateFn.apply(fn, *inputs)


def mse_mean(a, b):
    return ReconFn.apply(a, b, 1)


def l1_mean(a, b):
    return ReconFn.apply(a, b, 2)


# ------------------------------------------------------------------------------------------
# GEMM arithmetic (trainer precision)
# ------------------------------------------------------------------------------------------
_PRECISION = {"32": 0, "32-true": 0, "fp32": 0, 32: 0, "bf16": 1, "bf16-mixed": 1, "bf16-true": 1,
              "32-exact": 2, "fp32-exact": 2}


def set_precision(precision) -> int:
    """Map the reference trainer's `precision` flag onto the GEMM arithmetic of every following
    conv/bmm launch: "32" -> 3xBF16 fp32 emulation, "bf16-mixed" -> bf16 operands with fp32
    accumulation (what autocast runs these ops in), "32-exact" -> exact fp32 on the f32-input MFMA
    (parity mode, 1/5 of the 3xBF16 rate). Returns the previous mode."""
    if precision not in _PRECISION:
        raise ValueError(f"precision {precision!r} is not supported on the MI355X path "
                         f"(supported: {sorted(map(str, _PRECISION))})")
    prev = _lib.query("mvae_get_math_mode")
    _lib.call("mvae_set_math_mode", _PRECISION[precision])
    _MATH[0] = _PRECISION[precision]
    return prev


_SALT = {}


def dropout_salt(device) -> torch.Tensor:
    """The process-wide dropout salt of `device` (one int64 in device memory, allocated once and never freed) and
    make it the library's salt (mvae_set_dropout_salt): it is mixed into every following GroupNorm dropout seed, so
    a replayed graph of a training step that advances it draws fresh masks."""
    device = torch.device(device)
    t = _SALT.get(device)
    if t is None:
        t = _SALT[device] = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=device)
    _lib.call("mvae_set_dropout_salt", t.data_ptr())
    return t


def restore_math_mode(mode: int):
    _lib.call("mvae_set_math_mode", int(mode))
    _MATH[0] = int(mode)


# ------------------------------------------------------------------------------------------
# perceptual loss pieces (LPIPS, vae_losses.py:67-94)
# ------------------------------------------------------------------------------------------
def _like_cl(t):
    return torch.empty_like(t, memory_format=CL) if t.dim() == 4 else torch.empty_like(t)


class ReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _check(x, "relu input")
        x = nhwc(x)
        y = _like_cl(x)
        _lib.call("mvae_relu_fwd", x.data_ptr(), y.data_ptr(), x.numel(), _stream(x))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = nhwc(dy.float())
        dx = _like_cl(y)
        _lib.call("mvae_relu_bwd", y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel(), _stream(y))
        return dx


def relu(x):
    return ReluFn.apply(x)


class MaxPoolFn(torch.autograd.Function):
    """nn.MaxPool2d(kernel_size=k, stride=s), no padding (torchvision alexnet 3/2, vgg16 2/2)."""

    @staticmethod
    def forward(ctx, x, k: int, s: int):
        _check(x, "maxpool input")
        x = nhwc(x)
        n, c, h, w = x.shape
        ho, wo = (h - k) // s + 1, (w - k) // s + 1
        y = torch.empty((n, c, ho, wo), device=x.device, dtype=torch.float32, memory_format=CL)
        arg = torch.empty((n, ho, wo, c), device=x.device, dtype=torch.uint8)
        _lib.call("mvae_maxpool_fwd", x.data_ptr(), y.data_ptr(), arg.data_ptr(), n, h, w, c, k, s, _stream(x))
        ctx.save_for_backward(arg)
        ctx.shape, ctx.k, ctx.s = (n, c, h, w), k, s
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        n, c, h, w = ctx.shape
        dy = nhwc(dy.float())
        dx = torch.empty((n, c, h, w), device=dy.device, dtype=torch.float32, memory_format=CL)
        _lib.call("mvae_maxpool_bwd", dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), n, h, w, c, ctx.k, ctx.s,
                  _stream(dy))
        return dx, None, None


def max_pool(x, k: int, s: int):
    return MaxPoolFn.apply(x, k, s)


def max_pool3s2(x):
    return MaxPoolFn.apply(x, 3, 2)


class LpipsScaleFn(torch.autograd.Function):
    """y = (a*x + b - shift[c]) * inv_scale[c]  (`x*2-1` then lpips' ScalingLayer)."""

    @staticmethod
    def forward(ctx, x, shift, inv_scale, a: float, b: float):
        _check(x, "lpips input")
        x = nhwc(x.float())
        y = _like_cl(x)
        _lib.call("mvae_lpips_scale", x.data_ptr(), y.data_ptr(), x.numel(), x.shape[1], float(a), float(b),
                  shift.data_ptr(), inv_scale.data_ptr(), _stream(x))
        ctx.save_for_backward(inv_scale)
        ctx.a = float(a)
        return y

    @staticmethod
    def backward(ctx, dy):
        (inv_scale,) = ctx.saved_tensors
        dy = nhwc(dy.float())
        dx = _like_cl(dy)
        _lib.call("mvae_lpips_scale_bwd", dy.data_ptr(), dx.data_ptr(), dy.numel(), dy.shape[1], ctx.a,
                  inv_scale.data_ptr(), _stream(dy))
        return dx, None, None, None, None


def lpips_scale(x, shift, inv_scale, a=2.0, b=-1.0):
    return LpipsScaleFn.apply(x, shift, inv_scale, a, b)


class LpipsDistFn(torch.autograd.Function):
    """Per-image LPIPS layer distance: mean over pixels of sum_c w_c (f0/|f0| - f1/|f1|)^2."""

    @staticmethod
    def forward(ctx, f0, f1, w):
        _check(f0, "lpips features")
        f0, f1 = nhwc(f0), nhwc(f1)
        n, c, h, wd = f0.shape
        w = w.detach().contiguous().float()
        score = torch.empty(n, device=f0.device, dtype=torch.float32)
        _lib.call("mvae_lpips_dist", f0.data_ptr(), f1.data_ptr(), w.data_ptr(), score.data_ptr(), n, h * wd, c, 0.0,
                  _stream(f0))
        ctx.save_for_backward(f0, f1, w)
        return score

    @staticmethod
    def backward(ctx, g):
        f0, f1, w = ctx.saved_tensors
        n, c, h, wd = f0.shape
        g = g.contiguous().float()
        need0, need1 = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        df0 = _like_cl(f0)
        df1 = _like_cl(f1) if need1 else None
        _lib.call("mvae_lpips_dist_bwd", f0.data_ptr(), f1.data_ptr(), w.data_ptr(), g.data_ptr(), df0.data_ptr(),
                  _ptr(df1), n, h * wd, c, _stream(f0))
        return (df0 if need0 else None), df1, None


def lpips_dist(f0, f1, w):
    return LpipsDistFn.apply(f0, f1, w)


# ------------------------------------------------------------------------------------------
# adversarial branch: BatchNorm2d(+LeakyReLU), LeakyReLU, hinge / mean terms (row (f)2)
# ------------------------------------------------------------------------------------------
class BatchNormFn(torch.autograd.Function):
    """nn.BatchNorm2d (+ the following in-place LeakyReLU when slope >= 0) over NHWC."""

    @staticmethod
    def forward(ctx, x, gamma, beta, run_mean, run_var, training: bool, momentum: float, eps: float, slope: float):
        _check(x, "batch_norm input")
        x = nhwc(x)
        n, c, h, w = x.shape
        rows = n * h * w
        y = torch.empty_like(x, memory_format=CL)
        mean = torch.empty(c, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        ws = ARENA.get("bn", _lib.query("mvae_batch_norm_workspace_bytes", rows, c), x.device)
        _lib.call("mvae_batch_norm_fwd_nhwc", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), _ptr(run_mean), _ptr(run_var), rows, c, float(eps),
                  float(momentum), int(training), float(slope), ws.data_ptr(), ws.numel(), _stream(x))
        ctx.save_for_backward(x, y, gamma, mean, rstd)
        ctx.training, ctx.slope = training, slope
        ctx.gamma_ref, ctx.beta_ref = gamma, beta
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, mean, rstd = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("BatchNorm backward is built for training-mode statistics only")
        dy = nhwc(dy)
        n, c, h, w = x.shape
        rows = n * h * w
        dx = torch.empty_like(x, memory_format=CL)
        dg = _main_grad(ctx.gamma_ref) if ctx.needs_input_grad[1] else None
        db = _main_grad(ctx.beta_ref) if ctx.needs_input_grad[2] else None
        dg_ret = db_ret = None
        if ctx.needs_input_grad[1] and dg is None:
            dg = dg_ret = torch.zeros(c, device=x.device, dtype=torch.float32)
        if ctx.needs_input_grad[2] and db is None:
            db = db_ret = torch.zeros(c, device=x.device, dtype=torch.float32)
        ws = ARENA.get("bn", _lib.query("mvae_batch_norm_workspace_bytes", rows, c), x.device)
        _lib.call("mvae_batch_norm_bwd_nhwc", x.data_ptr(), y.data_ptr(), dy.data_ptr(), gamma.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), _ptr(dg), _ptr(db), rows, c, float(ctx.slope),
                  ws.data_ptr(), ws.numel(), _stream(x))
        if ctx.needs_input_grad[1] and dg_ret is None:
            _grad_done(ctx.gamma_ref)
        if ctx.needs_input_grad[2] and db_ret is None:
            _grad_done(ctx.beta_ref)
        return dx, dg_ret, db_ret, None, None, None, None, None, None, None


def batch_norm(x, gamma, beta, run_mean, run_var, training, momentum=0.1, eps=1e-5, slope=-1.0):
    return BatchNormFn.apply(x, gamma, beta, run_mean, run_var, training, momentum, eps, slope)


class LeakyReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slope: float):
        _check(x, "leaky_relu input")
        x = nhwc(x)
        y = _like_cl(x)
        _lib.call("mvae_leaky_relu_fwd", x.data_ptr(), y.data_ptr(), float(slope), x.numel(), _stream(x))
        ctx.save_for_backward(y)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = nhwc(dy.float())
        dx = _like_cl(y)
        _lib.call("mvae_leaky_relu_bwd", y.data_ptr(), dy.data_ptr(), dx.data_ptr(), float(ctx.slope), y.numel(),
                  _stream(y))
        return dx, None


def leaky_relu(x, slope=0.2):
    return LeakyReluFn.apply(x, slope)


class AdvTermFn(torch.autograd.Function):
    """scale * sum(term(a)): kind 4 relu(1-a), 5 relu(1+a), 6 a (hinge / generator terms)."""

    @staticmethod
    def forward(ctx, a, kind: int, scale: float):
        _check(a, "logits")
        a = a.contiguous() if a.dim() != 4 else nhwc(a)
        out = torch.empty((), device=a.device, dtype=torch.float32)
        ws = ARENA.get("red", _lib.query("mvae_reduce_workspace_bytes"), a.device)
        _lib.call("mvae_loss_reduce", kind, a.data_ptr(), a.data_ptr(), 1, a.numel(), 1, float(scale), out.data_ptr(),
                  ws.data_ptr(), ws.numel(), _stream(a))
        ctx.save_for_backward(a)
        ctx.kind, ctx.scale = kind, scale
        return out

    @staticmethod
    def backward(ctx, g):
        (a,) = ctx.saved_tensors
        g = g.contiguous().float()
        da = _like_cl(a)
        _lib.call("mvae_adv_bwd", ctx.kind, a.data_ptr(), g.data_ptr(), float(ctx.scale), da.data_ptr(), a.numel(),
                  _stream(a))
        return da, None, None


def hinge_real(logits):  # mean(relu(1 - logits))
    return AdvTermFn.apply(logits, 4, 1.0 / logits.numel())


def hinge_fake(logits):  # mean(relu(1 + logits))
    return AdvTermFn.apply(logits, 5, 1.0 / logits.numel())


def neg_mean(logits):  # -mean(logits)
    return AdvTermFn.apply(logits, 6, -1.0 / logits.numel())


# ------------------------------------------------------------------------------------------
# disentangled modality routing (disentangled_conditional_vae.py:124-193, 241-303): one launch per batch,
# each sample runs only its own modality's projector / head (csrc/routing.hip)
# ------------------------------------------------------------------------------------------
ROUTING_MAX_MODALITIES = 8


def _ptr_table(ts):
    arr = (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])
    return arr


def routing_fits(h: int, w: int, c: int, nm: int) -> bool:
    """The routing kernels keep a whole image (zero-bordered, 5 planes in the backward) in LDS."""
    return c == 3 and 1 <= nm <= ROUTING_MAX_MODALITIES and (4 * (h + 2) * (w + 2) * c + h * w * c) * 4 <= 160 * 1024


def _grad_targets(params):
    """Flat gradient slots of the parameters, or fresh zero tensors (returned to autograd)."""
    tg, ret = [], []
    for p in params:
        if p is None:
            tg.append(None)
            ret.append(None)
            continue
        g = _main_grad(p)
        if g is None:
            if p.dim() == 4:
                o, i, kh, kw = p.shape
                g = torch.zeros((o, kh, kw, i), device=p.device, dtype=torch.float32).permute(0, 3, 1, 2)
            else:
                g = torch.zeros_like(p, dtype=torch.float32)
            ret.append(g)
        else:
            ret.append(None)
        tg.append(g)
    return tg, ret


class ModalityHeadsFn(torch.autograd.Function):
    """Per-sample modality head conv3x3 -> ReLU -> conv3x3 (+ 1x1 output projector, zero-padded to out_c) for
    the whole batch in one launch. params: per modality (w1, b1, w2, b2, pw, pb), pw/pb None for colour
    modalities (no projector)."""

    @staticmethod
    def forward(ctx, rec, idx, out_c: int, nm: int, *params):
        _check(rec, "decoder output")
        rec = nhwc(rec)
        n, c, h, w = rec.shape
        idx = idx.to(device=rec.device, dtype=torch.long).contiguous()
        ws = [None if p is None else (_krsc(p) if p.dim() == 4 else p.contiguous()) for p in params]
        tab = _ptr_table(ws)
        out = torch.empty((n, out_c, h, w), device=rec.device, dtype=torch.float32, memory_format=CL)
        _lib.call("mvae_modality_heads_fwd", rec.data_ptr(), idx.data_ptr(), n, h, w, c, nm, tab, out_c,
                  out.data_ptr(), _stream(rec))
        ctx.save_for_backward(rec, idx, *[t for t in ws if t is not None])
        ctx.present = [t is not None for t in ws]
        ctx.out_c, ctx.nm = out_c, nm
        ctx.param_refs = params
        return out

    @staticmethod
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        rec, idx, rest = saved[0], saved[1], list(saved[2:])
        ws = [rest.pop(0) if pr else None for pr in ctx.present]
        n, c, h, w = rec.shape
        dout = nhwc(dout.float())
        drec = torch.empty_like(rec, memory_format=CL)
        tg, ret = _grad_targets(ctx.param_refs)
        gtab = _ptr_table(tg)
        tab = _ptr_table(ws)
        nbytes = _lib.query("mvae_modality_heads_workspace_bytes", n, c)
        wsp = ARENA.get("heads", nbytes, rec.device)
        _lib.call("mvae_modality_heads_bwd", rec.data_ptr(), idx.data_ptr(), n, h, w, c, ctx.nm, tab, ctx.out_c,
                  dout.data_ptr(), drec.data_ptr(), gtab, wsp.data_ptr(), wsp.numel(), _stream(rec))
        _grad_done(*[p for p, r in zip(ctx.param_refs, ret) if p is not None and r is None])
        return (drec, None, None, None, *ret)


def modality_heads(rec, idx, out_c: int, nm: int, params):
    return ModalityHeadsFn.apply(rec, idx, out_c, nm, *params)


class RouteInFn(torch.autograd.Function):
    """routed[b] = nan_to_zero(projector_m(nan_to_zero(x[b, :1]))) for modalities with an input projector,
    else nan_to_zero(x[b, :C]) (zero channels beyond x's). params: per modality (w, b) or (None, None)."""

    @staticmethod
    def forward(ctx, x, idx, c: int, nm: int, *params):
        _check(x, "input")
        x = nhwc(x)
        n, cx, h, w = x.shape
        idx = idx.to(device=x.device, dtype=torch.long).contiguous()
        ws = [None if p is None else p.contiguous() for p in params]
        routed = torch.empty((n, c, h, w), device=x.device, dtype=torch.float32, memory_format=CL)
        _lib.call("mvae_modality_route_in_fwd", x.data_ptr(), cx, idx.data_ptr(), n, h * w, c, nm, _ptr_table(ws),
                  routed.data_ptr(), _stream(x))
        ctx.save_for_backward(x, idx, *[t for t in ws if t is not None])
        ctx.present = [t is not None for t in ws]
        ctx.c, ctx.nm = c, nm
        ctx.param_refs = params
        return routed

    @staticmethod
    def backward(ctx, drouted):
        saved = ctx.saved_tensors
        x, idx, rest = saved[0], saved[1], list(saved[2:])
        ws = [rest.pop(0) if pr else None for pr in ctx.present]
        n, cx, h, w = x.shape
        drouted = nhwc(drouted.float())
        tg, ret = _grad_targets(ctx.param_refs)
        nbytes = _lib.query("mvae_modality_route_in_workspace_bytes", n, ctx.c)
        wsp = ARENA.get("route_in", nbytes, x.device)
        _lib.call("mvae_modality_route_in_bwd", x.data_ptr(), cx, idx.data_ptr(), n, h * w, ctx.c, ctx.nm,
                  _ptr_table(ws), drouted.data_ptr(), _ptr_table(tg), wsp.data_ptr(), wsp.numel(), _stream(x))
        _grad_done(*[p for p, r in zip(ctx.param_refs, ret) if p is not None and r is None])
        return (None, None, None, None, *ret)


def modality_route_in(x, idx, c: int, nm: int, params):
    return RouteInFn.apply(x, idx, c, nm, *params)


# ------------------------------------------------------------------------------------------
# ConditionalVAE concat conditioning (conditional_vae.py:65-69, 107-136): Linear + ReLU + bilinear + cat in two
# launches (csrc/condition.hip); bit-exact with the reference for a one-hot condition
# ------------------------------------------------------------------------------------------
class ConditionConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cond, weight, bias):
        _check(x, "input")
        x = nhwc(x)
        n, c, h, w = x.shape
        cond = cond.to(device=x.device, dtype=torch.float32).contiguous()
        k = cond.shape[1]
        if weight.shape != (c * 64, k) or bias.shape != (c * 64,):
            raise ValueError(f"condition_proj must be Linear({k} -> {c * 64}), got {tuple(weight.shape)}")
        m = torch.empty((n, c * 64), device=x.device, dtype=torch.float32)
        xc = torch.empty((n, 2 * c, h, w), device=x.device, dtype=torch.float32, memory_format=CL)
        _lib.call("mvae_condition_concat_fwd", x.data_ptr(), cond.data_ptr(), weight.contiguous().data_ptr(),
                  bias.data_ptr(), m.data_ptr(), xc.data_ptr(), n, c, h, w, k, _stream(x))
        ctx.save_for_backward(cond, m)
        ctx.mark_non_differentiable(m)
        ctx.param_refs = (weight, bias)
        ctx.x_grad = x.requires_grad
        ctx.shape = (n, c, h, w, k)
        return xc, m

    @staticmethod
    def backward(ctx, dxc, dm_unused):
        cond, m = ctx.saved_tensors
        n, c, h, w, k = ctx.shape
        dxc = nhwc(dxc.float())
        tg, ret = _grad_targets(ctx.param_refs)
        dpre = ARENA.get("cond", n * c * 64 * 4, dxc.device)
        _lib.call("mvae_condition_concat_bwd", dxc.data_ptr(), cond.data_ptr(), m.data_ptr(), _ptr(tg[0]),
                  _ptr(tg[1]), dpre.data_ptr(), n, c, h, w, k, _stream(dxc))
        _grad_done(*[p for p, r in zip(ctx.param_refs, ret) if r is None])
        dx = dxc[:, :c] if ctx.x_grad else None
        return (dx, None, *ret)


COND_MAX_HW = 256  # csrc/condition.hip COND_MAX_HW: the bilinear backward's LDS row buffer


def condition_concat_fits(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dim() == 4 and max(x.shape[2], x.shape[3]) <= COND_MAX_HW


def condition_concat(x, cond, weight, bias):
    """(x_cond [B, 2C, H, W] channels_last, relu(condition_proj) [B, C*64]); H, W <= COND_MAX_HW."""
    return ConditionConcatFn.apply(x, cond, weight, bias)


# ------------------------------------------------------------------------------------------
# DisentangledConditionalVAE's batch-coupled latent losses (disentangled_conditional_vae.py:195-206 partition,
# :305-349 separation, :351-386 contrastive) fused: two launches forward, two backward (csrc/latent.hip)
# ------------------------------------------------------------------------------------------
LATENT_MAX_B, LATENT_MAX_D = 1024, 16
LATENT_FUSED = os.environ.get("MVAE_NO_LATENT_FUSED") is None


def latent_aux_fits(z: torch.Tensor, d: int) -> bool:
    return LATENT_FUSED and z.is_cuda and z.dim() == 4 and z.shape[0] <= LATENT_MAX_B and 0 < d <= LATENT_MAX_D and \
        z.shape[0] * d <= LATENT_MAX_B * LATENT_MAX_D // 2 and \
        (z.is_contiguous(memory_format=CL) or z.is_contiguous())


class LatentAuxFn(torch.autograd.Function):
    """(separation, contrastive) of the modality partition z.view(B, -1)[:, off:off + d]; a non-finite value drops
    that term's gradient on the device (the reference's NaN -> 0 replacement, :540-550)."""

    @staticmethod
    def forward(ctx, z, idx, off: int, d: int, temperature: float):
        _check(z, "latent")
        n, c, h, w = z.shape
        cl = int(z.is_contiguous(memory_format=CL) and not z.is_contiguous())
        idx = idx.to(device=z.device, dtype=torch.long).contiguous()
        out = torch.empty(3, device=z.device, dtype=torch.float32)
        nbytes = _lib.query("mvae_latent_aux_workspace_bytes", n, d)
        ws = torch.empty(nbytes // 4, device=z.device, dtype=torch.float32)
        _lib.call("mvae_latent_aux_fwd", z.data_ptr(), idx.data_ptr(), n, c, h * w, cl, off, d, float(temperature),
                  out.data_ptr(), ws.data_ptr(), nbytes, _stream(z))
        ctx.save_for_backward(z, idx, out, ws)
        ctx.geo = (n, c, h * w, cl, off, d, float(temperature))
        sep, con = out[0], out[1]
        return sep, con

    @staticmethod
    def backward(ctx, gsep, gcon):
        z, idx, out, ws = ctx.saved_tensors
        n, c, hw, cl, off, d, t = ctx.geo
        gsep = (gsep if gsep is not None else torch.zeros((), device=z.device)).float().contiguous()
        gcon = (gcon if gcon is not None else torch.zeros((), device=z.device)).float().contiguous()
        dz = torch.zeros_like(z)  # same memory format as z; the kernels write the partition's elements only
        _lib.call("mvae_latent_aux_bwd", z.data_ptr(), idx.data_ptr(), n, c, hw, cl, off, d, t, out.data_ptr(),
                  gsep.data_ptr(), gcon.data_ptr(), dz.data_ptr(), ws.data_ptr(), ws.numel() * 4, _stream(z))
        return dz, None, None, None, None


def latent_aux_losses(z, idx, off: int, d: int, temperature: float = 0.1):
    return LatentAuxFn.apply(z, idx, off, d, temperature)
