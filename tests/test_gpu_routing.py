"""Batched modality routing kernels (csrc/routing.hip) against a float64 per-sample loop written like the
reference's (src/models/disentangled_conditional_vae.py:137-169 encode projectors, :255-301 decode heads):
outputs, input gradient and every per-modality parameter gradient. Index routing is selection: samples of
modality m touch only modality m's parameters (absent modalities get exactly zero gradient)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

KW = dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4),
          num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28)


def _model(dev):
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(3)
    m = M.DisentangledConditionalVAE(**KW).to(dev)
    with torch.no_grad():  # non-trivial biases
        for n, p in m.named_parameters():
            if n.startswith("modality_") and n.endswith("bias"):
                p.uniform_(-0.3, 0.3)
    return m


def _ref_heads(model, rec, idx, out_c):
    outs = []
    for b in range(rec.shape[0]):
        m = min(int(idx[b]), 4)
        head = model.modality_decoders[m]
        h = F.conv2d(rec[b:b + 1], head[0].weight.double().cpu(), head[0].bias.double().cpu(), padding=1)
        h = F.conv2d(torch.relu(h), head[2].weight.double().cpu(), head[2].bias.double().cpu(), padding=1)
        if str(m) in model.modality_output_projectors:
            pj = model.modality_output_projectors[str(m)]
            h = F.conv2d(h, pj.weight.double().cpu(), pj.bias.double().cpu())
        h = h[:, :out_c]
        if h.shape[1] < out_c:
            h = torch.cat([h, h.new_zeros((1, out_c - h.shape[1]) + tuple(h.shape[2:]))], 1)
        outs.append(h)
    return torch.cat(outs)


@pytest.mark.parametrize("out_c,ids", [(3, [0, 1, 2, 3, 4, 7, 1, 0, 17, 3, 2, 4, 4, 9, 1, 0]),
                                       (3, [1, 1, 4, 2]),          # colour only: gray heads absent
                                       (1, [0, 3, 3, 0, 0])])     # all gray (collate gives 1 channel out)
def test_modality_heads_match_per_sample_loop(out_c, ids):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from medvae_disentangled_multimodal_amd import ops
    dev = torch.device("cuda:0")
    model = _model(dev)
    B = len(ids)
    g = torch.Generator().manual_seed(9)
    rec0 = torch.randn(B, 3, 28, 28, generator=g)
    dout0 = torch.randn(B, out_c, 28, 28, generator=g)
    idx = torch.tensor(ids, dtype=torch.long)
    rec = rec0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    out = ops.modality_heads(rec, idx.to(dev), out_c, 5, model._head_params())
    out.backward(dout0.to(dev))
    ref_rec = rec0.double().requires_grad_()
    params = {n: p for n, p in model.named_parameters() if n.startswith(("modality_decoders", "modality_output"))}
    ref = _ref_heads(model, ref_rec, idx, out_c)
    rp = [p for p in params.values()]
    rg = torch.autograd.grad(ref, [ref_rec] + rp, dout0.double(), allow_unused=True)
    rel = lambda a, b: float((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm().clamp_min(1e-30))
    assert rel(out, ref.detach()) < 1e-5
    assert rel(rec.grad, rg[0]) < 1e-5
    present = {min(i, 4) for i in ids}
    for (n, p), r in zip(params.items(), rg[1:]):
        m = int(n.split(".")[1])
        if m in present:
            assert p.grad is not None and rel(p.grad, r) < 1e-5, n
        else:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n


def test_route_in_matches_per_sample_loop():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from medvae_disentangled_multimodal_amd import ops
    dev = torch.device("cuda:0")
    model = _model(dev)
    ids = [0, 1, 2, 3, 4, 7, 3, 0]
    B = len(ids)
    g = torch.Generator().manual_seed(4)
    x0 = torch.rand(B, 3, 28, 28, generator=g) * 2 - 1
    x0[2, 1, 5, 5] = float("nan")   # colour sample: scrubbed to 0
    x0[3, 0, 7, 9] = float("nan")   # gray sample: scrubbed before its projector
    dr0 = torch.randn(B, 3, 28, 28, generator=g)
    idx = torch.tensor(ids)
    routed = ops.modality_route_in(x0.to(dev), idx.to(dev), 3, 5, model._route_in_params())
    routed.backward(dr0.to(dev))
    xs = torch.where(torch.isnan(x0), torch.zeros_like(x0), x0).double()
    refs = []
    for b in range(B):
        m = min(ids[b], 4)
        if str(m) in model.modality_input_projectors:
            pj = model.modality_input_projectors[str(m)]
            refs.append(F.conv2d(xs[b:b + 1, :1], pj.weight.double().cpu(), pj.bias.double().cpu()))
        else:
            refs.append(xs[b:b + 1, :3])
    ref = torch.cat(refs)
    assert float((routed.double().cpu() - ref.cpu()).abs().max()) < 1e-6
    for key in ("0", "3"):
        pj = model.modality_input_projectors[key]
        w = pj.weight.double().detach().requires_grad_()
        bb = pj.bias.double().detach().requires_grad_()
        sel = [b for b in range(B) if min(ids[b], 4) == int(key)]
        o = F.conv2d(xs[sel, :1], w.cpu(), bb.cpu())
        gw, gb = torch.autograd.grad(o, [w, bb], dr0[sel].double())
        gw, gb = gw.cpu(), gb.cpu()
        assert float((pj.weight.grad.double().cpu() - gw).norm() / gw.norm()) < 1e-5
        assert float((pj.bias.grad.double().cpu() - gb).norm() / gb.norm()) < 1e-5


def test_one_channel_batch_routing_kernel_matches_grouped_form(monkeypatch):
    """a 1-channel batch (cx = 1) with colour modalities present. The routing kernel reads the
    missing channels as zeros ([x0, 0, 0]); the grouped form (MVAE_NO_ROUTING / large images) zero-pads the same
    way, so both paths give the same encoder input and latents."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import medvae_disentangled_multimodal_amd.disentangled as D
    dev = torch.device("cuda:0")
    model = _model(dev)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(6, 1, 28, 28, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    idx = torch.tensor([0, 1, 2, 3, 4, 1], device=dev)
    with torch.no_grad():
        mu_k, lv_k = model.encode(x, idx)
        monkeypatch.setattr(D, "ROUTING_KERNELS", False)
        mu_g, lv_g = model.encode(x, idx)
    # same encoder input; the two forms differ only in how the 1x1 projector is evaluated (routing kernel fp32 vs
    # the 3xBF16 conv), i.e. at the conv tolerance (2e-4) -- before the fix the colour samples differed by O(1)
    assert float((mu_k - mu_g).norm() / mu_g.norm()) < 2e-4
    assert float((lv_k - lv_g).norm() / lv_g.norm()) < 2e-4
