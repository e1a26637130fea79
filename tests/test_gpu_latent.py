"""Fused batch-coupled latent losses of DisentangledConditionalVAE (csrc/latent.hip: partition_latent +
modality_separation_loss + contrastive_loss, src/models/disentangled_conditional_vae.py:195-206, 305-386) against the
model's own torch formulation (the restatement the golden dis_c3* fixtures pin) evaluated in float64 on the CPU:
values and the gradient w.r.t. z, 1e-4 relative (fp32 sums over B <= 512 rows and exp(10)-scaled similarities).
Cases: the c3 bench geometry (B=512, 5 modalities, NHWC z [512, 16, 7, 7]), out-of-range ids kept as their own
centroids, one modality only (separation 0), rows without positives, a NaN latent (the term's gradient is dropped)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

KW = dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4),
          num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _ref(model, z, idx):
    zr = z.detach().double().cpu().requires_grad_()
    ir = idx.cpu()
    sep = model.modality_separation_loss(zr, ir)
    con = model.contrastive_loss(zr, ir)
    return zr, sep, con


CASES = {
    "c3_b512": lambda g: torch.randint(0, 5, (512,), generator=g),
    "ids_out_of_range": lambda g: torch.tensor([0, 1, 2, 3, 4, 7, 1, 0, 17, 3, 2, 4, 4, 9, 1, 0]),
    "one_modality": lambda g: torch.full((12,), 3, dtype=torch.long),
    "singletons": lambda g: torch.tensor([0, 1, 2, 3, 4, 4, 5, 6]),  # rows 0-3, 6, 7 have no positives
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_latent_aux_matches_torch_formulation(dev, case):
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ops
    model = M.DisentangledConditionalVAE(**KW)
    g = torch.Generator().manual_seed(len(case))
    idx = CASES[case](g)
    B = idx.shape[0]
    z = torch.randn(B, 16, 7, 7, generator=g)
    zd = z.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    sep, con = ops.latent_aux_losses(zd, idx.to(dev), 8, 8)
    ws, wc = torch.randn(2, generator=g).tolist()
    (ws * sep + wc * con).backward()
    zr, rs, rc = _ref(model, z, idx)
    (ws * rs + wc * rc).backward()
    # 1e-4 relative, plus an fp32-rounding floor for terms that vanish (one modality: ps == tot, l = -log(1 + 1e-8))
    assert abs(float(sep) - float(rs)) <= 1e-4 * abs(float(rs)) + 2e-6, (float(sep), float(rs))
    assert abs(float(con) - float(rc)) <= 1e-4 * abs(float(rc)) + 2e-6, (float(con), float(rc))
    gd, gr = zd.grad.double().cpu(), zr.grad
    assert float((gd - gr).norm()) <= 1e-4 * float(gr.norm()) + 1e-6
    if case == "one_modality":
        assert float(sep) == 0.0
    # only the partition (flat NCHW elements 8..15 = channel 0, pixels 8..15) carries gradient
    mask = torch.zeros(16 * 49, dtype=torch.bool)
    mask[8:16] = True
    assert float(gd.reshape(B, -1)[:, ~mask].abs().max()) == 0.0


def test_latent_aux_nan_drops_gradient(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(3)
    idx = torch.tensor([0, 1, 0, 1, 2, 2])
    z = torch.randn(6, 16, 7, 7, generator=g)
    z.view(6, -1)[2, 9] = float("nan")
    zd = z.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    sep, con = ops.latent_aux_losses(zd, idx.to(dev), 8, 8)
    assert not torch.isfinite(sep) and not torch.isfinite(con)
    (sep + con).backward()
    assert float(zd.grad.abs().max()) == 0.0


def test_disentangled_forward_uses_fused_losses(dev):
    """The model's forward routes sep / con through the fused op at the c3 geometry, same values as the torch glue."""
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ops
    torch.manual_seed(0)
    model = M.DisentangledConditionalVAE(**KW).to(dev)
    g = torch.Generator().manual_seed(5)
    idx = torch.randint(0, 5, (64,), generator=g).to(dev)
    x = (torch.rand(64, 3, 28, 28, generator=g) * 2 - 1).to(dev)
    eps = torch.randn(64, 16, 7, 7, generator=g).to(dev)
    out = model(x, idx, eps=eps)
    zr = out["z"].detach().double().cpu()
    rs = model.modality_separation_loss(zr, idx.cpu())
    rc = model.contrastive_loss(zr, idx.cpu())
    assert abs(float(out["separation_loss"]) - float(rs)) <= 1e-4 * abs(float(rs))
    assert abs(float(out["contrastive_loss"]) - float(rc)) <= 1e-4 * abs(float(rc))
    assert ops.latent_aux_fits(out["z"], 8)
