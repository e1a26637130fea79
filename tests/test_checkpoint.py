"""Lightning checkpoint interchange on CPU (no kernels run): the written layout loads into the
reference-side objects (`model.`-prefixed state dict, torch.optim.AdamW state_dict format), and a
checkpoint round-trips model weights and Adam moments through the flat buffers."""
import os
import tempfile

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
