"""Conv backward with the weight gradient on a side stream (ops.BWD_OVERLAP, MVAE_BWD_OVERLAP=1): the same kernels
as the one-stream backward, so input and flat-buffer weight / bias gradients must match it bit for bit -- eagerly and
replayed from a captured HIP graph -- over the ResnetBlock chain (GroupNorm -> 3x3 conv with fused statistics ->
GroupNorm -> 3x3 conv + residual), a Downsample and an Upsample conv (encoder_decoder.py:36-80, :123-146)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _params(dev, c, seed):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(seed)
    ps = {}
    for name, shape in (("w1", (c, c, 3, 3)), ("w2", (c, c, 3, 3)), ("wd", (c, c, 3, 3)), ("wu", (c, c, 3, 3))):
        ps[name] = (torch.randn(shape, generator=g) / (3.0 * c ** 0.5)).to(dev).contiguous(
            memory_format=torch.channels_last)
    for name in ("b1", "b2", "bd", "bu"):
        ps[name] = (torch.randn(c, generator=g) * 0.1).to(dev)
    for p in ps.values():
        p.requires_grad_()
        p._mvae_main_grad = torch.zeros_like(p)
    ps["gamma"] = torch.ones(c, device=dev)
    ps["beta"] = torch.zeros(c, device=dev)
    assert ops is not None
    return ps


def _chain(ps, x):
    from medvae_disentangled_multimodal_amd import ops
    c = x.shape[1]
    h = ops.group_norm(x, ps["gamma"], ps["beta"], 8, silu=True, for_conv=c)
    h = ops.conv2d(h, ps["w1"], ps["b1"], ops.ConvGeom(3, 3, 1, 1, 1, 1, 1), gn_stats=True)
    h = ops.group_norm(h, ps["gamma"], ps["beta"], 8, silu=True, for_conv=c)
    h = ops.conv2d(h, ps["w2"], ps["b2"], ops.ConvGeom(3, 3, 1, 1, 1, 1, 1), residual=x)
    d = ops.conv2d(h, ps["wd"], ps["bd"], ops.ConvGeom(3, 3, 2, 0, 0, 1, 1))          # Downsample (pad 0,1,0,1)
    u = ops.conv2d(d, ps["wu"], ps["bu"], ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, True))    # Upsample (nearest x2 + conv)
    return u


def _grads(ps, xd):
    return [xd.grad.clone()] + [ps[k]._mvae_main_grad.clone() for k in ("w1", "w2", "wd", "wu", "b1", "b2", "bd", "bu")]


def _eager(dev, prec, overlap, shape=(8, 64, 16, 16)):
    from medvae_disentangled_multimodal_amd import ops
    prev, saved = ops.set_precision(prec), ops.BWD_OVERLAP
    ops.BWD_OVERLAP = overlap
    try:
        ps = _params(dev, shape[1], 3)
        g = torch.Generator().manual_seed(11)
        xd = torch.randn(shape, generator=g).to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
        go = torch.randn(shape, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
        u = _chain(ps, xd)
        u.backward(go)
        torch.cuda.synchronize()
        return [u.detach().clone()] + _grads(ps, xd)
    finally:
        ops.restore_math_mode(prev)
        ops.BWD_OVERLAP = saved


@pytest.mark.parametrize("prec", ["32", "bf16-mixed"])
def test_overlap_matches_one_stream(dev, prec):
    from medvae_disentangled_multimodal_amd import ops
    one = _eager(dev, prec, False)
    two = _eager(dev, prec, True)
    assert dev in ops._SIDE  # the side stream was taken
    for i, (a, b) in enumerate(zip(one, two)):
        assert torch.equal(a, b), i


def test_overlap_under_graph_capture(dev):
    """fork / join inside a captured step: replay gives the eager one-stream gradients"""
    from medvae_disentangled_multimodal_amd import ops
    ref = _eager(dev, "32", False)
    prev, saved = ops.set_precision("32"), ops.BWD_OVERLAP
    ops.BWD_OVERLAP = True
    try:
        shape = (8, 64, 16, 16)
        ps = _params(dev, shape[1], 3)
        g = torch.Generator().manual_seed(11)
        xd = torch.randn(shape, generator=g).to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
        go = torch.randn(shape, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm-up outside capture (creates the side stream, sizes the scratch arena)
            _chain(ps, xd).backward(go)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            xd.grad = None
            for k in ("w1", "w2", "wd", "wu", "b1", "b2", "bd", "bu"):
                ps[k]._mvae_main_grad.zero_()
            u = _chain(ps, xd)
            u.backward(go)
        graph.replay()
        torch.cuda.synchronize()
        got = [u.detach().clone()] + _grads(ps, xd)
    finally:
        ops.restore_math_mode(prev)
        ops.BWD_OVERLAP = saved
    for i, (a, b) in enumerate(zip(ref, got)):
        assert torch.equal(a, b), i
