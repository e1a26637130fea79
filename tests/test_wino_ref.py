"""The float64 Winograd emulation the bf16 parity tests check against (tests/wino_ref.py) is itself pinned here: with no
operand rounding it must reproduce the direct convolution, its input gradient and its weight gradient (torch float64
autograd) to rounding, for both output tiles and ragged image sizes; and with bf16 rounding its error against float64
must sit at the measured levels the ops.py comment states (F2 ~4e-3, F4 ~3e-2 at 16x16x256)."""
import pytest
import torch
import torch.nn.functional as F

import wino_ref as W


@pytest.mark.parametrize("m", [2, 4])
@pytest.mark.parametrize("n,c,k,h,w", [(2, 8, 6, 8, 8), (2, 8, 4, 7, 7), (1, 4, 8, 14, 10)])
def test_emulation_is_the_convolution(m, n, c, k, h, w):
    g = torch.Generator().manual_seed(n + c + k + h + w + m)
    x = torch.randn(n, c, h, w, dtype=torch.float64, generator=g)
    wt = torch.randn(k, c, 3, 3, dtype=torch.float64, generator=g)
    b = torch.randn(k, dtype=torch.float64, generator=g)
    dy = torch.randn(n, k, h, w, dtype=torch.float64, generator=g)
    xr, wr = x.clone().requires_grad_(), wt.clone().requires_grad_()
    y = F.conv2d(xr, wr, b, padding=1)
    y.backward(dy)
    assert torch.allclose(W.conv(x, wt, m, W.ident) + b.view(1, -1, 1, 1), y, atol=1e-11)
    ns = torch.randint(0, n, (12,), generator=g)
    oh, ow = torch.randint(0, h, (12,), generator=g), torch.randint(0, w, (12,), generator=g)
    assert torch.allclose(W.rows(x, wt, b, ns, oh, ow, m, W.ident), y[ns, :, oh, ow], atol=1e-11)
    assert torch.allclose(W.conv(dy, W.dgrad_weights(wt), m, W.ident), xr.grad, atol=1e-11)
    assert torch.allclose(W.wgrad(x, dy, m, W.ident), wr.grad, atol=1e-11)
    cols = torch.tensor([k - 1, 0])
    assert torch.allclose(W.wgrad(x, dy, m, W.ident, cols=cols), wr.grad[cols], atol=1e-11)


def test_bf16_emulation_error_levels():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 256, 16, 16, dtype=torch.float64, generator=g)
    wt = torch.randn(64, 256, 3, 3, dtype=torch.float64, generator=g) / 48
    y = F.conv2d(x, wt, padding=1)

    def rel(a):
        return float((a - y).norm() / y.norm())
    e2, e4 = rel(W.conv(x, wt, 2, W.bf16)), rel(W.conv(x, wt, 4, W.bf16))
    direct = rel(F.conv2d(W.bf16(x), W.bf16(wt), padding=1))
    assert 1e-3 < direct < 4e-3 and 2.5e-3 < e2 < 6e-3 and 1.5e-2 < e4 < 4e-2


@pytest.mark.parametrize("m", [2, 4])
def test_upsample_emulation_is_the_upsampled_convolution(m):
    g = torch.Generator().manual_seed(3 + m)
    x = torch.randn(2, 6, 7, 5, dtype=torch.float64, generator=g)
    wt = torch.randn(4, 6, 3, 3, dtype=torch.float64, generator=g)
    dy = torch.randn(2, 4, 14, 10, dtype=torch.float64, generator=g)
    xr, wr = x.clone().requires_grad_(), wt.clone().requires_grad_()
    y = F.conv2d(F.interpolate(xr, scale_factor=2.0, mode="nearest"), wr, padding=1)
    y.backward(dy)
    assert torch.allclose(W.ups_conv(x, wt, m, W.ident), y, atol=1e-11)
    assert torch.allclose(W.ups_dgrad(dy, wt, m, W.ident), xr.grad, atol=1e-11)
    assert torch.allclose(W.ups_wgrad(x, dy, m, W.ident), wr.grad, atol=1e-11)
