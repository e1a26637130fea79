"""The one-hot conditioning HIP kernels (csrc/condition.hip: ConditionalVAE.condition_proj + ReLU + bilinear map +
concat, src/models/conditional_vae.py:65-69, 107-136) on the MI355X. north_star: the one-hot modality-conditioning
index path is bit-exact. Forward: bitwise against the reference's own projection / condition map (golden fixtures)
and against the CPU restatement at the bench geometry (B=256, 64x64); the projection equals W[:, idx] + b bitwise.
Backward (weight / bias gradient of the projection through the interpolation): against float64 torch autograd,
1e-5 relative."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_io import golden_state, load_case
from oracle.torch_ref import condition_map_exact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _bits(t):
    return np.ascontiguousarray(np.asarray(t, np.float32)).view(np.int32)


def _run(dev, x, oh, w, b):
    from medvae_disentangled_multimodal_amd import ops
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    xc, m = ops.condition_concat(xd, oh.to(dev), w.to(dev), b.to(dev))
    torch.cuda.synchronize()
    return xc.cpu(), m.cpu()


@pytest.mark.parametrize("case", ["cvae_c4", "cvae_c4_full"])
def test_condition_concat_bitwise_vs_reference_fixture(dev, case):
    meta, d = load_case(case)
    P = golden_state(meta)
    w, b = P["condition_proj.0.weight"], P["condition_proj.0.bias"]
    x, oh = torch.from_numpy(d["in.x"]), torch.from_numpy(d["in.cond"])
    xc, m = _run(dev, x, oh, w, b)
    C = x.shape[1]
    assert np.array_equal(_bits(xc[:, :C]), _bits(x))                      # concat keeps x bit for bit
    assert np.array_equal(_bits(xc[:, C:]), _bits(d["out.cond_map"]))       # the reference's condition map
    assert np.array_equal(_bits(m), _bits(np.maximum(d["out.cond_proj"], 0)))
    idx = oh.argmax(1)
    assert np.array_equal(_bits(m), _bits(torch.relu(w.t()[idx] + b)))     # index path: column select + bias


def test_condition_concat_bitwise_at_bench_geometry(dev):
    """c4's batch (256 one-hot rows over all 12 modalities) at 64x64: kernel == CPU restatement bitwise."""
    g = torch.Generator().manual_seed(21)
    B, C, H = 256, 3, 64
    w = torch.randn(C * 64, 12, generator=g) * 0.2
    b = torch.randn(C * 64, generator=g) * 0.2
    idx = torch.arange(B) % 12
    oh = F.one_hot(idx, 12).float()
    x = torch.randint(0, 256, (B, C, H, H), generator=g).float() / 255 * 2 - 1
    xc, m = _run(dev, x, oh, w, b)
    pre, cmap = condition_map_exact(w.numpy(), b.numpy(), oh.numpy(), C, H, H)
    assert np.array_equal(_bits(xc[:, C:]), _bits(cmap))
    assert np.array_equal(_bits(m), _bits(np.maximum(pre, 0)))


@pytest.mark.parametrize("H", [64, 28])
def test_condition_concat_backward(dev, H):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(H)
    B, C = 5, 3
    w = torch.randn(C * 64, 12, generator=g) * 0.2
    b = torch.randn(C * 64, generator=g) * 0.2
    oh = F.one_hot(torch.tensor([0, 3, 11, 3, 7]), 12).float()
    x = torch.randn(B, C, H, H, generator=g)
    dxc = torch.randn(B, 2 * C, H, H, generator=g)
    wd = w.to(dev).requires_grad_()
    bd = b.to(dev).requires_grad_()
    xc, _ = ops.condition_concat(x.to(dev).contiguous(memory_format=torch.channels_last), oh.to(dev), wd, bd)
    xc.backward(dxc.to(dev).contiguous(memory_format=torch.channels_last))
    wr = w.double().requires_grad_()
    br = b.double().requires_grad_()
    cm = F.interpolate(F.relu(F.linear(oh.double(), wr, br)).view(B, C, 8, 8), size=(H, H), mode="bilinear",
                       align_corners=False)
    (cm * dxc[:, C:].double()).sum().backward()
    for a, r in ((wd.grad, wr.grad), (bd.grad, br.grad)):
        a = a.double().cpu()
        assert float((a - r).norm() / r.norm()) < 1e-5


def test_conditional_encode_above_kernel_size_limit(dev):
    """288 x 288 (> the kernel's 256 LDS rows): ConditionalVAE.encode takes the module path (Linear + ReLU + bilinear
    + cat) instead of failing with MVAE_EINVAL; its condition map matches the CPU module path."""
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ops
    assert not ops.condition_concat_fits(torch.empty(1, 3, 288, 288, device=dev))
    torch.manual_seed(0)
    m = M.ConditionalVAE(input_channels=3, latent_dim=4, hidden_channels=32, ch_mult=(1, 2), num_res_blocks=1,
                         attn_resolutions=[], dropout=0.0, resolution=288, condition_method="concat")
    oh = F.one_hot(torch.tensor([1, 7]), 12).float()
    ref = m.create_condition_map(oh, 288, 288)
    m = m.to(dev)
    x = torch.randn(2, 3, 288, 288, device=dev)
    mean, logvar = m.encode(x, oh.to(dev))
    assert mean.shape == (2, 4, 144, 144) and torch.isfinite(mean).all() and torch.isfinite(logvar).all()
    got = m.create_condition_map(oh.to(dev), 288, 288).cpu()
    assert float((got - ref).abs().max()) <= 1e-5 * float(ref.abs().max())
