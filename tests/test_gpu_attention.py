"""Fused single-tile attention core (csrc/attn.hip, ops.AttnCoreFn for n <= 64 tokens): AttnBlock's
softmax(q k^T * C^-1/2, dim=2) v and its backward (src/models/encoder_decoder.py:83-107) in one launch per direction,
at the mid-block geometries of the configs -- c3 (49 tokens, C = 128), c2 / c1 (49, 512), c4 / c5 (64, 2048) -- and edge
cases (1 token, ragged 17 tokens, C = 64). Checked against float64 torch in each GEMM arithmetic: 3xBF16 ("32"), exact
fp32 ("32-exact") and bf16 ("bf16-mixed"; the float64 reference then rounds q, k, v to bf16 and the tolerance covers
the bf16 rounding of P / dS inside the products), and against the unfused path (two batched GEMMs around a row
softmax) in the same arithmetic."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(8, 128, 7, 7), (4, 512, 7, 7), (2, 2048, 8, 8), (3, 64, 1, 1), (3, 64, 1, 17), (5, 64, 8, 8)]
TOL = {"32": (2e-5, 1e-4), "32-exact": (5e-6, 5e-6), "bf16-mixed": (1e-2, 2e-2)}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _rel(a, b):
    """relative L2 error; the denominator is floored at 1e-3 per element RMS (one token: softmax over a single key is
    constant, so the reference dq = dk = 0 exactly and only the absolute error means anything)"""
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-3 * b.numel() ** 0.5))


def _ref(q, k, v, go):
    b, c, h, w = q.shape
    n = h * w
    qr, kr, vr = (t.double().requires_grad_() for t in (q, k, v))
    s = torch.bmm(qr.reshape(b, c, n).permute(0, 2, 1), kr.reshape(b, c, n)) * c ** -0.5
    o = torch.bmm(vr.reshape(b, c, n), torch.softmax(s, 2).permute(0, 2, 1)).reshape(b, c, h, w)
    o.backward(go.double())
    return o, qr.grad, kr.grad, vr.grad


def _run(dev, q, k, v, go, prec, fused):
    from medvae_disentangled_multimodal_amd import ops
    qd, kd, vd = (t.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_() for t in (q, k, v))
    prev, saved, maxc = ops.set_precision(prec), ops.ATTN_FUSED, ops.ATTN_FUSED_MAXC
    ops.ATTN_FUSED = fused
    ops.ATTN_FUSED_MAXC = 1 << 30  # the kernel at every C it supports (the dispatch uses it up to C = 512)
    try:
        o = ops.attention_core(qd, kd, vd)
        o.backward(go.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
        ops.ATTN_FUSED, ops.ATTN_FUSED_MAXC = saved, maxc
    return o, qd.grad, kd.grad, vd.grad


@pytest.mark.parametrize("prec", sorted(TOL))
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_fused_attention_matches_float64(dev, shape, prec):
    from medvae_disentangled_multimodal_amd import ops
    b, c, h, w = shape
    assert ops._attn_small_ok(torch.empty(16, device=dev), h * w, c)
    g = torch.Generator().manual_seed(c + h * w)
    q, k, v = (torch.randn(shape, generator=g) for _ in range(3))
    go = torch.randn(shape, generator=g)
    qi, ki, vi = (t.bfloat16().float() for t in (q, k, v)) if prec == "bf16-mixed" else (q, k, v)
    ref = _ref(qi, ki, vi, go)
    got = _run(dev, q, k, v, go, prec, True)
    tf, tb = TOL[prec]
    assert _rel(got[0], ref[0]) < tf, ("out", _rel(got[0], ref[0]))
    for name, a, r in zip(("dq", "dk", "dv"), got[1:], ref[1:]):
        assert _rel(a, r) < tb, (name, _rel(a, r))


@pytest.mark.parametrize("prec", ["32", "bf16-mixed"])
def test_fused_attention_matches_unfused_path(dev, prec):
    """same arithmetic, the two implementations: only the fp32 accumulation / softmax evaluation order differs."""
    shape = (4, 512, 7, 7)
    g = torch.Generator().manual_seed(11)
    q, k, v, go = (torch.randn(shape, generator=g) for _ in range(4))
    fused = _run(dev, q, k, v, go, prec, True)
    unfused = _run(dev, q, k, v, go, prec, False)
    tol = 2e-5 if prec == "32" else 5e-3
    for a, r in zip(fused, unfused):
        assert _rel(a, r) < tol


def test_fused_attention_launch_count(dev):
    """one launch forward, one backward (the unfused path: 3 + 5)."""
    from medvae_disentangled_multimodal_amd import ops
    shape = (2, 128, 7, 7)
    g = torch.Generator().manual_seed(3)
    q, k, v, go = (torch.randn(shape, generator=g) for _ in range(4))
    qd, kd, vd = (t.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_() for t in (q, k, v))
    assert ops._attn_use_fused(qd, 49, 128)
    ops.PROFILE = []
    try:
        o = ops.attention_core(qd, kd, vd)
        o.backward(go.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        rec = [r for r in ops.PROFILE if r[0] == "attn_gemm"]
    finally:
        ops.PROFILE = None
    assert len(rec) == 2


# query-block fused attention (csrc/attn_tile.hip): the 16x16 level of c4 / c5 (n = 256, C = 1024), the 8x8 mid blocks
# at C = 2048 (n = 64), and n = 128 / 192
TILE_SHAPES = [(2, 1024, 16, 16), (2, 2048, 8, 8), (3, 128, 8, 16), (2, 256, 12, 16)]


def _run_tile(dev, q, k, v, go, prec, tile):
    from medvae_disentangled_multimodal_amd import ops
    qd, kd, vd = (t.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_() for t in (q, k, v))
    prev, saved = ops.set_precision(prec), (ops.ATTN_FUSED, ops.ATTN_TILE)
    ops.ATTN_FUSED, ops.ATTN_TILE = False, tile
    try:
        o = ops.attention_core(qd, kd, vd)
        o.backward(go.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
        ops.ATTN_FUSED, ops.ATTN_TILE = saved
    return o, qd.grad, kd.grad, vd.grad


@pytest.mark.parametrize("prec", sorted(TOL))
@pytest.mark.parametrize("shape", TILE_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_tile_attention_matches_float64(dev, shape, prec, monkeypatch):
    from medvae_disentangled_multimodal_amd import ops
    b, c, h, w = shape
    monkeypatch.setattr(ops, "ATTN_TILE", True)  # (opt-in path: eligibility with the switch on)
    assert ops._attn_use_tile(torch.empty((b, 16), device=dev), h * w, c)
    g = torch.Generator().manual_seed(c + h * w + 1)
    q, k, v = (torch.randn(shape, generator=g) for _ in range(3))
    go = torch.randn(shape, generator=g)
    qi, ki, vi = (t.bfloat16().float() for t in (q, k, v)) if prec == "bf16-mixed" else (q, k, v)
    ref = _ref(qi, ki, vi, go)
    got = _run_tile(dev, q, k, v, go, prec, True)
    tf, tb = TOL[prec]
    assert _rel(got[0], ref[0]) < tf, ("out", _rel(got[0], ref[0]))
    for name, a, r in zip(("dq", "dk", "dv"), got[1:], ref[1:]):
        assert _rel(a, r) < tb, (name, _rel(a, r))


@pytest.mark.parametrize("prec", ["32", "bf16-mixed"])
def test_tile_attention_matches_unfused_path(dev, prec):
    shape = (2, 1024, 16, 16)
    g = torch.Generator().manual_seed(12)
    q, k, v, go = (torch.randn(shape, generator=g) for _ in range(4))
    tile = _run_tile(dev, q, k, v, go, prec, True)
    unfused = _run_tile(dev, q, k, v, go, prec, False)
    tol = 2e-5 if prec == "32" else 5e-3
    for a, r in zip(tile, unfused):
        assert _rel(a, r) < tol


def test_tile_attention_launch_count(dev):
    """forward one launch; backward one launch + the dV / dK batched GEMMs (the unfused path: 2 GEMMs + softmax forward,
    4 GEMMs + softmax backward)."""
    from medvae_disentangled_multimodal_amd import ops
    shape = (2, 1024, 16, 16)
    g = torch.Generator().manual_seed(3)
    q, k, v, go = (torch.randn(shape, generator=g) for _ in range(4))
    ops.PROFILE = []
    try:
        _run_tile(dev, q, k, v, go, "32", True)
        rec = [r for r in ops.PROFILE if r[0] == "attn_gemm"]
    finally:
        ops.PROFILE = None
    assert len(rec) == 4


def _attn_block_grads(dev, dx_sum: bool, prec: str, n_tok: int, retain: bool, calls):
    from medvae_disentangled_multimodal_amd import _lib, encoder_decoder as ED, ops
    torch.manual_seed(3)
    blk = ED.AttnBlock(64).to(dev)
    g = torch.Generator().manual_seed(9)
    hw = int(n_tok ** 0.5)
    x0 = torch.randn(2, 64, hw, hw, generator=g)
    go = torch.randn(2, 64, hw, hw, generator=g)
    x = x0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    saved, real_call = ops.DX_SUM, _lib.call

    def counting(name, *args):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *args)
    ops.DX_SUM, _lib.call = dx_sum, counting
    prev = ops.set_precision(prec)
    try:
        y = blk(x)
        gy = go.to(dev).contiguous(memory_format=torch.channels_last)
        y.backward(gy, retain_graph=retain)
        if retain:
            y.backward(gy)  # (a retained graph's second backward: the sum re-armed)
        torch.cuda.synchronize()
    finally:
        ops.DX_SUM, _lib.call = saved, real_call
        ops.restore_math_mode(prev)
    return [t.detach().double().cpu() for t in (x.grad, *[p.grad for p in blk.parameters()])]


@pytest.mark.parametrize("prec", ["32", "bf16-mixed", "32-exact"])
@pytest.mark.parametrize("n_tok,retain", [(64, False), (256, False), (256, True)])
def test_attn_block_input_gradient_summed_in_the_dgrad_gemms(dev, prec, n_tok, retain):
    """AttnBlock's q / k / v 1x1 convs accumulate the gradient of their shared input in one buffer (ops.DxSum: the
    dgrad GEMMs with beta = 1 after the first) instead of autograd summing three activation-sized gradients: every
    gradient equals the autograd-summed path within fp32 summation order (1e-6), also for a retained graph's second
    backward, and no torch add runs over the activation."""
    c_on, c_off = {}, {}
    on = _attn_block_grads(dev, True, prec, n_tok, retain, c_on)
    off = _attn_block_grads(dev, False, prec, n_tok, retain, c_off)
    for a, b in zip(on, off):
        assert _rel(a, b) < 1e-6
    assert c_on.get("mvae_gemm_strided_batched", 0) == c_off.get("mvae_gemm_strided_batched", 0)
