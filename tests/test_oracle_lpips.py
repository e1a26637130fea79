"""CPU checks of the LPIPS oracle restatement (oracle/torch_ref.py:lpips_alex) and of the LPIPS
module's host logic (weight naming, refusal without weights). Parity against the real `lpips`
package is unpinned: the package and its pretrained weights are not available offline."""
import pytest
import torch

from oracle.torch_ref import lpips_alex


def _weights(seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = {"conv1": (64, 3, 11, 11), "conv2": (192, 64, 5, 5), "conv3": (384, 192, 3, 3),
              "conv4": (256, 384, 3, 3), "conv5": (256, 256, 3, 3)}
    W = {}
    for k, s in shapes.items():
        fan = s[1] * s[2] * s[3]
        W[f"{k}.weight"] = (torch.rand(s, generator=g, dtype=torch.float64) * 2 - 1) * (6.0 / fan) ** 0.5
        W[f"{k}.bias"] = (torch.rand(s[0], generator=g, dtype=torch.float64) * 2 - 1) * 0.1
    for i, c in enumerate((64, 192, 384, 256, 256)):
        W[f"lins.{i}"] = torch.rand(c, generator=g, dtype=torch.float64) / c
    return W


def test_lpips_oracle_metric_properties():
    W = _weights()
    g = torch.Generator().manual_seed(1)
    x = torch.rand(3, 3, 64, 64, generator=g, dtype=torch.float64)
    y = torch.rand(3, 3, 64, 64, generator=g, dtype=torch.float64)
    d_xy = lpips_alex(W, x, y)
    assert d_xy.shape == (3, 1, 1, 1)
    assert torch.all(d_xy > 0)
    assert torch.allclose(d_xy, lpips_alex(W, y, x), rtol=1e-12, atol=0)
    assert float(lpips_alex(W, x, x).abs().max()) == 0.0
    # nearer images score lower
    near = (x + 0.01 * (y - x))
    assert torch.all(lpips_alex(W, x, near) < d_xy)


def test_lpips_module_weight_names_and_refusal():
    pytest.importorskip("medvae_disentangled_multimodal_amd")
    from medvae_disentangled_multimodal_amd.lpips import LPIPS
    import os
    if not os.environ.get("MVAE_LPIPS_WEIGHTS"):
        with pytest.raises(RuntimeError):
            LPIPS()
    m = LPIPS(allow_synthetic=True, seed=3)
    assert m.pretrained is False
    assert all(not p.requires_grad for p in m.parameters())
    # round trip through the lpips package's own state-dict names
    sd = {}
    for k, idx in zip(range(5), (0, 3, 6, 8, 10)):
        conv = m.convs()[k]
        sd[f"net.slice{k + 1}.{idx}.weight"] = conv.weight.detach().clone() * 2
        sd[f"net.slice{k + 1}.{idx}.bias"] = conv.bias.detach().clone()
        sd[f"lin{k}.model.1.weight"] = m.lins[k].detach().clone().view(1, -1, 1, 1)
    m2 = LPIPS(weights=sd)
    assert m2.pretrained is True
    assert torch.equal(m2.conv3.weight, m.conv3.weight * 2)
    assert torch.equal(m2.lins[4], m.lins[4])


def test_ssim_oracle_properties():
    from oracle.torch_ref import ssim_torchmetrics
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 3, 32, 32, generator=g, dtype=torch.float64)
    assert float(ssim_torchmetrics(x, x)) == pytest.approx(1.0, abs=1e-12)
    y = x + 0.3 * torch.randn(x.shape, generator=g, dtype=torch.float64)
    s = float(ssim_torchmetrics(y, x))
    assert 0.0 < s < 1.0
    assert float(ssim_torchmetrics(x, y)) == pytest.approx(s, rel=1e-12)  # symmetric
