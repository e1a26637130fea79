"""Diagnostic: per-layer accuracy of the HIP discriminator path against float64 (tests/golden/disc.npz inputs)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch, torch.nn.functional as F
from golden_io import golden_state, load_case
from oracle import torch_ref as R
from medvae_disentangled_multimodal_amd import ops
from medvae_disentangled_multimodal_amd.discriminator import NLayerDiscriminator
dev = torch.device("cuda:0")
meta, data = load_case("disc")
st = golden_state(meta)
D = NLayerDiscriminator(3, 64, 3).to(dev)
D.load_state_dict({k: v.to(dev) for k, v in st.items()}, strict=False)
D.train()
x = torch.from_numpy(data["in.x"])
xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
out = D(xd)
g = torch.Generator().manual_seed(0)
dy = torch.randn(out.shape, generator=g)
out.backward(dy.to(dev))
W = {k: v.double().requires_grad_() for k, v in st.items()}
running = {}
for k, s in meta["params"]:
    if k.endswith(".weight") and len(s) == 1:
        b = k[:-7]; running[b + ".running_mean"] = torch.zeros(s[0], dtype=torch.float64); running[b + ".running_var"] = torch.ones(s[0], dtype=torch.float64)
xr = x.double().requires_grad_()
o = R.discriminator(W, xr, running=running)
o.backward(dy.double())
rel = lambda a, b: float((a.detach().double().cpu() - b.detach()).norm() / b.detach().norm().clamp_min(1e-30))
print("logits", rel(out, o), "dx", rel(xd.grad, xr.grad))
for k, p in D.named_parameters():
    print(k, "%.2e" % rel(p.grad, W[k].grad), "norm %.3e" % float(W[k].grad.norm()))
# BatchNorm alone with a mean-dominated gradient
for c, n, hw in ((128, 2, 16 * 16), (256, 2, 8 * 8), (512, 2, 7 * 7)):
    xx = torch.randn(n, c, hw, 1, generator=g) * 3 + 5
    gy = torch.randn(n, c, hw, 1, generator=g) * 0.1 + 1.0
    gam, bet = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g)
    a = xx.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = ops.batch_norm(a, gam.to(dev), bet.to(dev), None, None, True, 0.1, 1e-5, 0.2)
    y.backward(gy.to(dev).contiguous(memory_format=torch.channels_last))
    ar = xx.double().requires_grad_()
    yr = F.leaky_relu(F.batch_norm(ar, None, None, gam.double(), bet.double(), True, 0.1, 1e-5), 0.2)
    yr.backward(gy.double())
    print("bn", c, hw, "y %.2e dx %.2e" % (rel(y, yr), rel(a.grad, ar.grad)))
