"""Lightning checkpoint interchange on CPU (no kernels run): the written layout loads into the
reference-side objects (`model.`-prefixed state dict, torch.optim.AdamW state_dict format), and a
checkpoint round-trips model weights and Adam moments through the flat buffers."""
import os
import tempfile

import pytest
import torch

import medvae_disentangled_multimodal_amd as M
from medvae_disentangled_multimodal_amd import checkpoint

KW = dict(input_channels=3, latent_dim=4, hidden_channels=32, ch_mult=(1, 2), num_res_blocks=1,
          attn_resolutions=[], resolution=16)


def _module(seed):
    torch.manual_seed(seed)
    model = M.BaseVAE(**KW)
    mod = M.VAELightningModule(model, {"type": "adamw", "lr": 2e-4, "betas": [0.5, 0.999]}, {"type": "none"},
                               {"type": "vae"}, gradient_clip_val=1.0)
    mod.configure_optimizers()
    return mod


def test_checkpoint_roundtrip_and_torch_format():
    a = _module(0)
    g = torch.Generator().manual_seed(1)
    a.optimizer.exp_avg.copy_(torch.randn(a.optimizer.exp_avg.shape, generator=g))
    a.optimizer.exp_avg_sq.copy_(torch.rand(a.optimizer.exp_avg_sq.shape, generator=g))
    a.optimizer.steps.fill_(7)
    a.global_step_count = 7
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "last.ckpt")
        checkpoint.save_checkpoint(a, path, epoch=3)
        ck = torch.load(path, weights_only=True)
        # Lightning layout, reference names (quick_generate.py:37-42 recipe works)
        assert ck["epoch"] == 3 and ck["global_step"] == 7
        names = [k[6:] for k in ck["state_dict"]]
        assert names == list(a.model.state_dict().keys())
        w = ck["state_dict"]["model.encoder.conv_in.weight"]
        assert w.shape == (32, 3, 3, 3) and w.is_contiguous()
        # torch.optim.AdamW accepts the optimizer state as its own
        ref_model = M.BaseVAE(**KW)
        ref_opt = torch.optim.AdamW(ref_model.parameters(), lr=1.0)
        ref_opt.load_state_dict(ck["optimizer_states"][0])
        p0 = next(iter(ref_model.parameters()))
        assert float(ref_opt.state[p0]["step"]) == 7.0
        # round trip into a differently initialised module
        b = _module(5)
        checkpoint.load_checkpoint(b, path)
    assert torch.equal(b.flat.data, a.flat.data)
    from medvae_disentangled_multimodal_amd.optim import FlatParameters as F
    for pa, pb, off in zip(a.flat.params, b.flat.params, a.flat.offsets):  # padding between tensors is not state
        assert torch.equal(F._view(b.optimizer.exp_avg, off, pb), F._view(a.optimizer.exp_avg, off, pa))
        assert torch.equal(F._view(b.optimizer.exp_avg_sq, off, pb), F._view(a.optimizer.exp_avg_sq, off, pa))
    assert torch.equal(b.optimizer.steps, a.optimizer.steps)
    assert b.global_step_count == 7


def test_checkpoint_lpips_discriminator_roundtrip():
    """config-5 / adversarial objective: the criterion's state (LPIPS network, NLayerDiscriminator weights and
    BatchNorm buffers) is written as `criterion.*` and the discriminator's Adam as optimizer_states[1]; both
    round-trip."""
    def make(seed):
        torch.manual_seed(seed)
        model = M.BaseVAE(**KW)
        loss = {"type": "lpips_discriminator", "allow_synthetic_lpips": True, "lpips_net": "alex",
                "discriminator": {"input_nc": 3, "ndf": 8, "n_layers": 2}}
        mod = M.VAELightningModule(model, {"type": "adam", "lr": 2e-4}, {"type": "none"}, loss)
        mod.configure_optimizers()
        return mod

    a = make(0)
    with torch.no_grad():
        for n, b in a.criterion.discriminator.named_buffers():
            if b.is_floating_point():
                b.uniform_(0.5, 1.5)
    a.optimizer_d.exp_avg.normal_()
    a.optimizer_d.exp_avg_sq.uniform_()
    a.optimizer_d.steps.fill_(3)
    ck = checkpoint.lightning_checkpoint(a)
    keys = list(ck["state_dict"])
    assert any(k.startswith("criterion.discriminator.") and k.endswith("running_mean") for k in keys)
    assert any(k.startswith("criterion.perceptual_loss.") for k in keys)
    assert len(ck["optimizer_states"]) == 2
    ref_d = torch.optim.Adam(a.criterion.discriminator.parameters(), lr=1.0)
    ref_d.load_state_dict(ck["optimizer_states"][1])  # torch's own format
    b = make(9)
    checkpoint.load_checkpoint(b, ck)
    assert torch.equal(b.flat_d.data, a.flat_d.data)
    for (ka, va), (kb, vb) in zip(a.criterion.state_dict().items(), b.criterion.state_dict().items()):
        assert ka == kb and torch.equal(va, vb), ka
    assert torch.equal(b.optimizer_d.steps, a.optimizer_d.steps)
    from medvae_disentangled_multimodal_amd.optim import FlatParameters as F
    for pa, pb, off in zip(a.flat_d.params, b.flat_d.params, a.flat_d.offsets):
        assert torch.equal(F._view(b.optimizer_d.exp_avg, off, pb), F._view(a.optimizer_d.exp_avg, off, pa))


def _lpips_package_keys(net):
    """The key set `lpips.LPIPS(net=...).state_dict()` (lpips 0.1.4) writes: ScalingLayer buffers, the
    torchvision feature convs under their slice / `features` index, and each linear layer twice (lin<k> and
    its alias lins.<k> in the ModuleList)."""
    convs = ((1, 0), (2, 3), (3, 6), (4, 8), (5, 10)) if net == "alex" else (
        (1, 0), (1, 2), (2, 5), (2, 7), (3, 10), (3, 12), (3, 14), (4, 17), (4, 19), (4, 21), (5, 24), (5, 26), (5, 28))
    keys = ["scaling_layer.shift", "scaling_layer.scale"]
    keys += [f"net.slice{s}.{i}.{t}" for s, i in convs for t in ("weight", "bias")]
    keys += [f"lin{k}.model.1.weight" for k in range(5)] + [f"lins.{k}.model.1.weight" for k in range(5)]
    return keys


@pytest.mark.parametrize("net", ["alex", "vgg"])
def test_lpips_state_dict_uses_package_names(net):
    """`criterion.perceptual_loss.lpips.*` carries the lpips package's names, so a reference
    LPIPS / LPIPS+discriminator checkpoint loads strictly and written checkpoints match its key layout."""
    from medvae_disentangled_multimodal_amd.lpips import LPIPS
    m = LPIPS(net=net, allow_synthetic=True, seed=1)
    sd = m.state_dict()
    assert sorted(sd) == sorted(_lpips_package_keys(net))
    assert sd["lin0.model.1.weight"].shape == (1, 64, 1, 1)
    assert sd["scaling_layer.scale"].shape == (1, 3, 1, 1)
    # a "reference" state dict (package names, different values) loads strictly and lands in the right slots
    ref = {k: (v * 2 if k.startswith(("net.", "lin")) else v).clone() for k, v in sd.items()}
    ref["lins.0.model.1.weight"] = ref["lin0.model.1.weight"]
    m2 = LPIPS(net=net, allow_synthetic=True, seed=5)
    m2.load_state_dict(ref, strict=True)
    assert torch.equal(m2.convs()[2].weight, m.convs()[2].weight * 2)
    assert torch.equal(m2.lins[4], m.lins[4] * 2)
    assert torch.equal(m2.inv_scale, 1.0 / m.scale)
    with pytest.raises(RuntimeError):  # strict: a missing conv is still an error
        m2.load_state_dict({k: v for k, v in ref.items() if not k.startswith("net.slice1.")}, strict=True)


def test_checkpoint_loads_reference_named_criterion():
    """A reference LPIPSWithDiscriminator checkpoint: `criterion.perceptual_loss.lpips.<lpips names>` +
    `criterion.discriminator.*` load with strict=True."""
    torch.manual_seed(0)
    loss = {"type": "lpips_discriminator", "allow_synthetic_lpips": True, "lpips_net": "alex",
            "discriminator": {"input_nc": 3, "ndf": 8, "n_layers": 2}}
    a = M.VAELightningModule(M.BaseVAE(**KW), {"type": "adam", "lr": 2e-4}, {"type": "none"}, loss)
    ck = checkpoint.lightning_checkpoint(a)
    pk = [k[len("criterion.perceptual_loss.lpips."):] for k in ck["state_dict"]
          if k.startswith("criterion.perceptual_loss.lpips.")]
    assert sorted(pk) == sorted(_lpips_package_keys("alex"))
    for k in list(ck["state_dict"]):
        if k.startswith("criterion.perceptual_loss.lpips.net."):
            ck["state_dict"][k] = ck["state_dict"][k] + 1.0
    b = M.VAELightningModule(M.BaseVAE(**KW), {"type": "adam", "lr": 2e-4}, {"type": "none"}, loss)
    checkpoint.load_checkpoint(b, ck, strict=True, load_optimizer=False)
    assert torch.equal(b.criterion.perceptual_loss.lpips.conv1.weight, a.criterion.perceptual_loss.lpips.conv1.weight + 1)
