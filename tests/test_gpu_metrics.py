"""On-device validation metrics vs the oracle restatement of src/utils/metrics.py (torchmetrics 1.7.4
SSIM/PSNR restated, not installed -- pinned only through that restatement) in float64 on the CPU.
Tolerance 1e-5 relative (fp32 reductions); the validation step produces every `val/*` key."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def test_reconstruction_and_kl_metrics(dev):
    from medvae_disentangled_multimodal_amd import metrics
    from oracle import torch_ref as R
    g = torch.Generator().manual_seed(0)
    x = torch.rand(3, 3, 28, 28, generator=g) * 2 - 1
    rec = x + 0.1 * torch.randn(x.shape, generator=g)
    cl = lambda t: t.to(dev).contiguous(memory_format=torch.channels_last)
    got = metrics.compute_reconstruction_metrics(cl(x), cl(rec))
    ref = R.reconstruction_metrics(x.double(), rec.double())
    for k in ref:
        assert got[k] == pytest.approx(ref[k], rel=1e-5), k
    mu = torch.randn(4, 16, 7, 7, generator=g)
    lv = torch.randn(4, 16, 7, 7, generator=g) * 0.5
    got = metrics.compute_kl_metrics(cl(mu), cl(lv))
    ref = R.kl_metrics(mu.double(), lv.double())
    for k in ref:
        assert got[k] == pytest.approx(ref[k], rel=1e-5), k
    # 2-D latents ([B, D], the docstring's shape)
    got = metrics.compute_kl_metrics(mu.flatten(1).to(dev), lv.flatten(1).to(dev))
    ref = R.kl_metrics(mu.flatten(1).double(), lv.flatten(1).double())
    for k in ref:
        assert got[k] == pytest.approx(ref[k], rel=1e-5), k


def test_validation_step_logs(dev):
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(0)
    model = M.BaseVAE(input_channels=3, latent_dim=4, hidden_channels=32, ch_mult=(1, 2), num_res_blocks=1,
                      attn_resolutions=[], resolution=16).to(dev)
    mod = M.VAELightningModule(model, {"type": "adam", "lr": 1e-3}, {"type": "none"}, {"type": "vae"})
    x = torch.rand(2, 3, 16, 16, device=dev) * 2 - 1
    logs = mod.evaluate((x, torch.zeros(2, 1, dtype=torch.long, device=dev)), "val")
    for k in ("mse", "mae", "psnr", "ssim", "kl_total", "kl_mean", "kl_std", "kl_per_dim_mean", "loss"):
        assert f"val/{k}" in logs and torch.isfinite(torch.as_tensor(logs[f"val/{k}"])).all(), k
    assert model.training


def test_kl_mse_mae_vs_reference_fixture(dev):
    """Device metrics against the reference's own compute_kl_metrics / compute_reconstruction_metrics (MSE, MAE)
    outputs (tests/golden/make_ref_fixtures.py); PSNR / SSIM stay pinned only to the torchmetrics restatement."""
    import os
    import numpy as np
    from medvae_disentangled_multimodal_amd import metrics
    ref = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_metrics.npz"),
                       allow_pickle=False))
    for tag in ("flat", "spatial"):
        mu = torch.from_numpy(ref[f"kl.{tag}.mean"]).to(dev)
        lv = torch.from_numpy(ref[f"kl.{tag}.logvar"]).to(dev)
        if mu.dim() == 4:
            mu, lv = mu.contiguous(memory_format=torch.channels_last), lv.contiguous(memory_format=torch.channels_last)
        got = metrics.compute_kl_metrics(mu, lv)
        for k in ("kl_total", "kl_mean", "kl_std", "kl_per_dim_mean"):
            assert float(got[k]) == pytest.approx(float(ref[f"kl.{tag}.{k}"]), rel=1e-5), (tag, k)
    cl = lambda t: torch.from_numpy(t).to(dev).contiguous(memory_format=torch.channels_last)
    got = metrics.compute_reconstruction_metrics(cl(ref["recon.x"]), cl(ref["recon.rec"]))
    assert float(got["mse"]) == pytest.approx(float(ref["recon.mse"]), rel=1e-5)
    assert float(got["mae"]) == pytest.approx(float(ref["recon.mae"]), rel=1e-5)
