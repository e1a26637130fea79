"""Diagnostic: layer-by-layer activation-gradient accuracy of the HIP discriminator vs float64 (hinge real branch)."""
import os, sys
R0 = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R0, os.path.join(R0, "tests", "golden"), os.path.join(R0, "tests")):
    sys.path.insert(0, p)
import torch, torch.nn.functional as F
from golden_io import golden_state, load_case
from medvae_disentangled_multimodal_amd import ops
from medvae_disentangled_multimodal_amd.discriminator import NLayerDiscriminator
dev = torch.device("cuda:0")
meta, data = load_case("disc")
st = golden_state(meta)
rel = lambda a, b: float((a.detach().double().cpu() - b.detach().double().cpu()).norm() / b.detach().double().cpu().norm().clamp_min(1e-30))
for exact in (True, False):
    D = NLayerDiscriminator(3, 64, 3, exact_fp32=exact).to(dev)
    D.load_state_dict({k: v.to(dev) for k, v in st.items()}, strict=False)
    D.train()
    x = torch.from_numpy(data["in.x"]).to(dev).contiguous(memory_format=torch.channels_last)
    acts = []
    h = x
    with ops.math_scope(2 if exact else None):
        for m in D.main:
            h = m(h)
            h.retain_grad()
            acts.append(h)
    loss = 0.5 * ops.hinge_real(h)
    loss.backward()
    # float64 reference, same layer sequence
    W = {k: v.double() for k, v in st.items()}
    hr = x.double().cpu().requires_grad_()
    refs = []
    i = 0
    seq = []
    for idx, m in enumerate(D.main):
        name = type(m).__name__
        if name == "Conv2d":
            hr = F.conv2d(hr, W[f"main.{idx}.weight"], W.get(f"main.{idx}.bias"), stride=m.geom.stride, padding=1)
        elif name == "BatchNorm2d":
            hr = F.batch_norm(hr, None, None, W[f"main.{idx}.weight"], W[f"main.{idx}.bias"], True, 0.1, 1e-5)
            hr = F.leaky_relu(hr, 0.2)
        elif name == "LeakyReLU":
            hr = F.leaky_relu(hr, 0.2)
        else:  # fused leaky: identity
            hr = hr * 1.0
        hr.retain_grad()
        refs.append(hr)
        seq.append(name)
    (0.5 * F.relu(1 - hr).mean()).backward()
    print("exact" if exact else "3xbf16", [(n, f"a {rel(a, r):.1e} g {rel(a.grad, r.grad):.1e}") for n, a, r in zip(seq, acts, refs)])
    # per-channel pixel sums of the activation gradients (BatchNorm input gradients sum to 0 exactly)
    for i, (n, a, r) in enumerate(zip(seq, acts, refs)):
        sa = a.grad.double().cpu().sum((0, 2, 3))
        sr = r.grad.sum((0, 2, 3))
        print(f"  {i} {n}: |sum ours| {float(sa.norm()):.3e} |sum f64| {float(sr.norm()):.3e} err {float((sa - sr).norm()):.3e} |g| {float(r.grad.norm()):.3e}")
