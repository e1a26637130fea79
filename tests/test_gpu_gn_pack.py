"""GroupNorm backward that also emits the producing conv's bf16 output gradient and bias gradient
(mvae_group_norm_bwd_pack_nhwc, ops.DyPack): the bf16-mixed mode's replacement for a pack_bf16_colsum pass over dy
(the conv bias half of convolution_backward, encoder_decoder.py:141-163). Checked on both GroupNorm backward paths
(streaming chain at large per-sample sizes, register-resident at small ones): dx bitwise equal to the plain backward,
the packed output bitwise equal to mvae_pack_bf16(dx), the bias gradient equal to float64 column sums of dx; and a
bf16-mixed training step whose gradients match the step with the separate pack pass."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


# (nb, h, w, C, groups): 64x64x128 takes the streaming chain, 8x8x512 / 7x7x256 the resident kernel
SHAPES = [(4, 64, 64, 128, 32), (8, 8, 8, 512, 32), (6, 7, 7, 256, 32)]


@pytest.mark.parametrize("fmt", ["pack", "split"])
@pytest.mark.parametrize("add", [False, True])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_gn_bwd_pack_matches_plain_backward(dev, shape, add, fmt):
    """fmt pack: dx also as packed bf16 (bf16-mixed); split: as split4_bf16 groups (3xBF16, the pre-split dY operand)"""
    from medvae_disentangled_multimodal_amd._lib import call, query
    nb, h, w, c, g = shape
    gen = torch.Generator(device=dev).manual_seed(nb * c + h)
    x = torch.randn(nb, h, w, c, device=dev, generator=gen)
    dy = torch.randn(nb, h, w, c, device=dev, generator=gen)
    gamma = 1 + 0.1 * torch.randn(c, device=dev, generator=gen)
    beta = 0.1 * torch.randn(c, device=dev, generator=gen)
    dadd = torch.randn(nb, h, w, c, device=dev, generator=gen) if add else None
    mean = x.view(nb, h * w, g, c // g).mean((1, 3)).reshape(-1).contiguous()
    rstd = (x.view(nb, h * w, g, c // g).var((1, 3), unbiased=False) + 1e-6).rsqrt().reshape(-1).contiguous()
    ws = torch.empty(query("mvae_group_norm_workspace_bytes", nb, h * w, c), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    dx0 = torch.empty_like(x)
    dg0, db0 = torch.zeros(c, device=dev), torch.zeros(c, device=dev)
    call("mvae_group_norm_bwd_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
         rstd.data_ptr(), dx0.data_ptr(), ptr(dadd), dg0.data_ptr(), db0.data_ptr(), nb, h * w, c, g, 1, 0.0, 0,
         ws.data_ptr(), ws.numel(), st)
    dx1 = torch.empty_like(x)
    dg1, db1 = torch.zeros(c, device=dev), torch.zeros(c, device=dev)
    packed = torch.empty(x.numel() * (4 if fmt == "split" else 2), dtype=torch.uint8, device=dev)
    bias = torch.randn(c, device=dev, generator=gen)
    bias0 = bias.clone()
    cs = torch.empty(query("mvae_group_norm_colsum_workspace_bytes", nb, h * w, c), dtype=torch.uint8, device=dev)
    call("mvae_group_norm_bwd_split_nhwc" if fmt == "split" else "mvae_group_norm_bwd_pack_nhwc",
         x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), dx1.data_ptr(), ptr(dadd), dg1.data_ptr(), db1.data_ptr(), nb, h * w, c, g,
         1, 0.0, 0, ws.data_ptr(), ws.numel(), packed.data_ptr(), bias.data_ptr(), 1.0, cs.data_ptr(), cs.numel(), st)
    ref_packed = torch.empty_like(packed)
    call("mvae_split_bf16" if fmt == "split" else "mvae_pack_bf16", dx0.data_ptr(), ref_packed.data_ptr(), x.numel(), st)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0)
    assert torch.equal(dg1, dg0) and torch.equal(db1, db0)
    assert torch.equal(packed, ref_packed)
    ref_bias = bias0.double() + dx0.double().sum((0, 1, 2))
    err = float((bias.double() - ref_bias).abs().max() / ref_bias.abs().max())
    assert err < 1e-6, err



@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("add", [False, True])
def test_gn_bwd_colsum_matches_plain_backward(dev, shape, add):
    """mvae_group_norm_bwd_colsum_nhwc: the plain backward's dx / dgamma / dbeta bit for bit, plus the producing conv's
    bias gradient (column sums of dx accumulated onto the bias slot) without a second copy of dx"""
    from medvae_disentangled_multimodal_amd._lib import call, query
    nb, h, w, c, g = shape
    gen = torch.Generator(device=dev).manual_seed(nb * c + h + 7)
    x = torch.randn(nb, h, w, c, device=dev, generator=gen)
    dy = torch.randn(nb, h, w, c, device=dev, generator=gen)
    gamma = 1 + 0.1 * torch.randn(c, device=dev, generator=gen)
    beta = 0.1 * torch.randn(c, device=dev, generator=gen)
    dadd = torch.randn(nb, h, w, c, device=dev, generator=gen) if add else None
    mean = x.view(nb, h * w, g, c // g).mean((1, 3)).reshape(-1).contiguous()
    rstd = (x.view(nb, h * w, g, c // g).var((1, 3), unbiased=False) + 1e-6).rsqrt().reshape(-1).contiguous()
    ws = torch.empty(query("mvae_group_norm_workspace_bytes", nb, h * w, c), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    dx0 = torch.empty_like(x)
    dg0, db0 = torch.zeros(c, device=dev), torch.zeros(c, device=dev)
    call("mvae_group_norm_bwd_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
         rstd.data_ptr(), dx0.data_ptr(), ptr(dadd), dg0.data_ptr(), db0.data_ptr(), nb, h * w, c, g, 1, 0.0, 0,
         ws.data_ptr(), ws.numel(), st)
    dx1 = torch.empty_like(x)
    dg1, db1 = torch.zeros(c, device=dev), torch.zeros(c, device=dev)
    bias = torch.randn(c, device=dev, generator=gen)
    bias0 = bias.clone()
    cs = torch.empty(query("mvae_group_norm_colsum_workspace_bytes", nb, h * w, c), dtype=torch.uint8, device=dev)
    call("mvae_group_norm_bwd_colsum_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
         mean.data_ptr(), rstd.data_ptr(), dx1.data_ptr(), ptr(dadd), dg1.data_ptr(), db1.data_ptr(), nb, h * w, c, g,
         1, 0.0, 0, ws.data_ptr(), ws.numel(), bias.data_ptr(), 1.0, cs.data_ptr(), cs.numel(), st)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0)
    assert torch.equal(dg1, dg0) and torch.equal(db1, db0)
    ref_bias = bias0.double() + dx0.double().sum((0, 1, 2))
    err = float((bias.double() - ref_bias).abs().max() / ref_bias.abs().max())
    assert err < 1e-6, err
    with pytest.raises(RuntimeError, match="column-sum workspace"):
        call("mvae_group_norm_bwd_colsum_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
             mean.data_ptr(), rstd.data_ptr(), dx1.data_ptr(), None, None, None, nb, h * w, c, g, 1, 0.0, 0,
             ws.data_ptr(), ws.numel(), bias.data_ptr(), 1.0, None, 0, st)

def _model_grads(dev, dypack: bool, calls=None):
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import _lib, ops
    kw = dict(input_channels=3, latent_dim=8, hidden_channels=64, ch_mult=(1, 2), num_res_blocks=1,
              attn_resolutions=[], dropout=0.0, resolution=32)
    torch.manual_seed(0)
    model = M.BaseVAE(**kw).to(dev)
    mod = M.VAELightningModule(model, {"type": "adam", "lr": 1e-4}, {"type": "none"}, {"type": "vae"},
                               gradient_clip_val=None, precision="bf16-mixed")
    mod.configure_optimizers()
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(4, 3, 32, 32, generator=g) * 2 - 1).to(dev)
    eps = torch.randn(4, 8, 16, 16, generator=g).to(dev)
    saved, real_call = ops.DYPACK, _lib.call
    ops.DYPACK = dypack
    if calls is not None:
        def counting(name, *args):
            calls[name] = calls.get(name, 0) + 1
            return real_call(name, *args)
        _lib.call = counting
    try:
        prev = ops.set_precision("bf16-mixed")
        try:
            mod.optimizer.zero_grad()
            ops.prep_flat_weights(mod.flat.data)
            loss = mod.training_step((x, torch.zeros(4, 1, dtype=torch.long, device=dev)), 0, eps=eps)
            loss.backward()
            ops.flat_weights_stale()
        finally:
            ops.restore_math_mode(prev)
        torch.cuda.synchronize()
    finally:
        ops.DYPACK = saved
        _lib.call = real_call
    return mod.flat.grad.detach().double().cpu(), mod.flat


def test_bf16_step_with_gn_packed_dy_matches_pack_pass(dev):
    """the same bf16-mixed step with the conv output gradients packed by the GroupNorm backward and by the separate
    pack pass: identical packed operands, so only the bias gradients' summation order differs."""
    c_fused, c_pass = {}, {}
    g_fused, flat = _model_grads(dev, True, c_fused)
    g_pass, _ = _model_grads(dev, False, c_pass)
    assert c_fused.get("mvae_group_norm_bwd_pack_nhwc", 0) >= 4
    assert c_fused.get("mvae_pack_bf16_colsum", 0) + c_fused["mvae_group_norm_bwd_pack_nhwc"] == \
        c_pass.get("mvae_pack_bf16_colsum", 0)
    rel = float((g_fused - g_pass).norm() / g_pass.norm())
    assert rel < 1e-5, rel
    for p, off, name in zip(flat.params, flat.offsets, flat.names):
        a, b = g_fused[off:off + p.numel()], g_pass[off:off + p.numel()]
        assert float((a - b).abs().max()) <= 1e-5 * max(1.0, float(b.abs().max())), name


def _dypack_rejection_grads(dev, dypack: bool, calls):
    from medvae_disentangled_multimodal_amd import _lib, ops
    from medvae_disentangled_multimodal_amd.optim import FlatParameters
    torch.manual_seed(3)
    m = torch.nn.ModuleDict(dict(c1=torch.nn.Conv2d(16, 32, 3, padding=1), n=torch.nn.GroupNorm(8, 32),
                                 c2=torch.nn.Conv2d(32, 16, 3, padding=1))).to(dev)
    flat = FlatParameters(m, dev)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 16, 16, 16, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
    saved, real_call = ops.DYPACK, _lib.call

    def counting(name, *args):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *args)
    ops.DYPACK, _lib.call = dypack, counting
    prev = ops.set_precision("bf16-mixed")
    try:
        y = ops.conv2d(x, m["c1"].weight, m["c1"].bias, geom, gn_stats=True)
        h = ops.group_norm(y, m["n"].weight, m["n"].bias, 8, silu=True, for_conv=16)
        out = ops.conv2d(h, m["c2"].weight, m["c2"].bias, geom)
        # y has a second consumer with no GradSink: autograd sums its gradient into the GroupNorm's dx, so the conv
        # backward's dy is not the tensor the GroupNorm packed
        loss = out.square().mean() + (y * 0.25).sum()
        flat.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
        ops.DYPACK, _lib.call = saved, real_call
    return {n: p._mvae_main_grad.detach().double().cpu().clone() for n, p in m.named_parameters()}


def test_dypack_rejected_dy_leaves_no_partial_bias_grad(dev):
    """when DyPack.take() rejects dy (another branch summed in after the GroupNorm backward), the conv's bias
    gradient comes from the real dy alone -- the GroupNorm's column sums must not have been added to the flat slot."""
    c_on, c_off = {}, {}
    g_on = _dypack_rejection_grads(dev, True, c_on)
    g_off = _dypack_rejection_grads(dev, False, c_off)
    assert c_on.get("mvae_group_norm_bwd_pack_nhwc", 0) == 1  # the request was made ...
    assert c_on.get("mvae_pack_bf16_colsum", 0) == c_off.get("mvae_pack_bf16_colsum", 0)  # ... and rejected
    for name in g_off:
        rel = float((g_on[name] - g_off[name]).norm() / g_off[name].norm())
        assert rel < 1e-6, (name, rel)


def _model_grads_3x(dev, dysplit: bool, calls):
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import _lib, ops
    kw = dict(input_channels=3, latent_dim=8, hidden_channels=64, ch_mult=(1, 2), num_res_blocks=1,
              attn_resolutions=[], dropout=0.0, resolution=32)
    torch.manual_seed(0)
    model = M.BaseVAE(**kw).to(dev)
    mod = M.VAELightningModule(model, {"type": "adam", "lr": 1e-4}, {"type": "none"}, {"type": "vae"},
                               gradient_clip_val=None)
    mod.configure_optimizers()
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(4, 3, 32, 32, generator=g) * 2 - 1).to(dev)
    eps = torch.randn(4, 8, 16, 16, generator=g).to(dev)
    saved, real_call, mn = ops.DYSPLIT, _lib.call, ops.DYSPLIT_MIN_MACS

    def counting(name, *args):
        calls[name] = calls.get(name, 0) + 1
        return real_call(name, *args)
    ops.DYSPLIT, _lib.call, ops.DYSPLIT_MIN_MACS = dysplit, counting, 0.0  # (every conv of the small model)
    try:
        mod.optimizer.zero_grad()
        ops.prep_flat_weights(mod.flat.data)
        loss = mod.training_step((x, torch.zeros(4, 1, dtype=torch.long, device=dev)), 0, eps=eps)
        loss.backward()
        ops.flat_weights_stale()
        torch.cuda.synchronize()
    finally:
        ops.DYSPLIT, _lib.call, ops.DYSPLIT_MIN_MACS = saved, real_call, mn
    return mod.flat.grad.detach().double().cpu(), mod.flat


def test_3xbf16_step_with_gn_split_dy_matches_register_split(dev):
    """the fp32-class (3xBF16) step with each conv's output gradient pre-split by the GroupNorm backward that produces
    it (mvae_group_norm_bwd_split_nhwc -> MVAE_CONV_XSPLIT / MVAE_CONV_DYSPLIT GEMM operands) against the step whose
    GEMMs split dy in registers: identical operand bits, so only the bias gradients' summation order differs."""
    c_on, c_off = {}, {}
    g_on, flat = _model_grads_3x(dev, True, c_on)
    g_off, _ = _model_grads_3x(dev, False, c_off)
    assert c_on.get("mvae_group_norm_bwd_split_nhwc", 0) >= 3 and "mvae_group_norm_bwd_split_nhwc" not in c_off
    rel = float((g_on - g_off).norm() / g_off.norm())
    assert rel < 1e-5, rel
    for p, off, name in zip(flat.params, flat.offsets, flat.names):
        a, b = g_on[off:off + p.numel()], g_off[off:off + p.numel()]
        assert float((a - b).abs().max()) <= 1e-5 * max(1.0, float(b.abs().max())), name


def _fit_params(dev, wanted: bool, calls):
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import _lib, ops
    kw = dict(input_channels=3, latent_dim=8, hidden_channels=64, ch_mult=(1, 2), num_res_blocks=1,
              attn_resolutions=[16], dropout=0.0, resolution=32)
    torch.manual_seed(0)
    model = M.BaseVAE(**kw).to(dev)
    mod = M.VAELightningModule(model, {"type": "adamw", "lr": 1e-3}, {"type": "none"}, {"type": "vae"},
                               gradient_clip_val=1.0)
    mod.configure_optimizers()
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(4, 3, 32, 32, generator=g) * 2 - 1).to(dev)
    eps = torch.randn(4, 8, 16, 16, generator=g).to(dev)
    saved, real_call = ops.FLAT_PREP_WANTED, _lib.call

    def counting(name, *args):
        if name == "mvae_split_bf16":
            calls.append(args[2])
        return real_call(name, *args)
    ops.FLAT_PREP_WANTED, _lib.call = wanted, counting
    ops.release_weight_buffers()
    try:
        for _ in range(3):
            mod.fit_step((x, torch.zeros(4, 1, dtype=torch.long, device=dev)), 0, eps=eps)
        torch.cuda.synchronize()
    finally:
        ops.FLAT_PREP_WANTED, _lib.call = saved, real_call
        ops.release_weight_buffers()
    return mod.flat.data.detach().cpu(), mod.flat.data.numel()


def test_flat_weight_prep_converts_only_the_wanted_ranges(dev):
    """From the second step on, the 3xBF16 step's weight prep splits only the flat-buffer ranges the previous step's
    convs read in that format (_FlatWeights.want): the parameters after three AdamW steps are bitwise those of the
    whole-buffer prep, and the later preps move fewer elements."""
    c_on, c_off = [], []
    p_on, n = _fit_params(dev, True, c_on)
    p_off, _ = _fit_params(dev, False, c_off)
    assert torch.equal(p_on, p_off)
    assert c_off.count(n) == 3  # the whole buffer every step
    assert c_on.count(n) == 1 and sum(c for c in c_on if c != n) < 2 * n


@pytest.mark.parametrize("prec", ["32", "bf16-mixed"])
@pytest.mark.parametrize("wino", [False, True])
def test_groupnorm_leaves_dx_unwritten_for_its_only_consumer(dev, prec, wino, monkeypatch):
    """ResnetBlock's norm2 (conv1's output has no other consumer) writes only conv1's split / packed copy of its dx:
    with the unwritten dx poisoned to NaN, a training step of a model whose ResnetBlocks run every conv1 path (implicit
    GEMM, LDS-DMA bf16, Winograd) gives finite gradients equal to the step that writes dx (bitwise: the conv reads the
    same copy either way)."""
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ops
    if wino:
        for k, v in (("WINOGRAD_MIN_C", 1), ("WINOGRAD_MIN_C_WIDE", 1), ("WINOGRAD_MIN_MACS", 0.0),
                     ("WINOGRAD_MAX_W", 64), ("WINOGRAD_BF16_MAX_W", 64), ("WINOGRAD_DY_FP32", False)):
            monkeypatch.setattr(ops, k, v)  # (the split-copy form of the Winograd convs: MVAE_WINOGRAD_DY_SPLIT=1)
    else:
        monkeypatch.setattr(ops, "WINOGRAD", False)
    monkeypatch.setattr(ops, "DYSPLIT_MIN_MACS", 0.0)
    kw = dict(input_channels=3, latent_dim=8, hidden_channels=64, ch_mult=(1, 2), num_res_blocks=1,
              attn_resolutions=[], dropout=0.0, resolution=32)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(4, 3, 32, 32, generator=g) * 2 - 1).to(dev)
    eps = torch.randn(4, 8, 16, 16, generator=g).to(dev)
    from medvae_disentangled_multimodal_amd import _lib
    grads, skipped = [], []
    real_call = _lib.call

    def spy(name, *args):
        if name in ("mvae_group_norm_bwd_split_nhwc", "mvae_group_norm_bwd_pack_nhwc") and args[6] is None:
            skipped.append(name)
        if name == "mvae_group_norm_bwd_part_split_nhwc" and args[7] is None:
            skipped.append(name)
        return real_call(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    for copy_only in (True, False):
        monkeypatch.setattr(ops, "DX_COPY_ONLY", copy_only)
        monkeypatch.setattr(ops, "DX_POISON", copy_only)
        torch.manual_seed(0)
        model = M.BaseVAE(**kw).to(dev)
        mod = M.VAELightningModule(model, {"type": "adam", "lr": 1e-4}, {"type": "none"}, {"type": "vae"},
                                   gradient_clip_val=None, precision=prec)
        mod.configure_optimizers()
        prev = ops.set_precision(prec)
        try:
            mod.optimizer.zero_grad()
            ops.prep_flat_weights(mod.flat.data)
            loss = mod.training_step((x, torch.zeros(4, 1, dtype=torch.long, device=dev)), 0, eps=eps)
            loss.backward()
            ops.flat_weights_stale()
            torch.cuda.synchronize()
        finally:
            ops.restore_math_mode(prev)
        grads.append(mod.flat.grad.detach().double().cpu())
    assert len(skipped) >= 2  # (every ResnetBlock's norm2 left dx unwritten)
    assert torch.isfinite(grads[0]).all()
    rel = float((grads[0] - grads[1]).norm() / grads[1].norm())
    assert rel < 1e-6, rel
