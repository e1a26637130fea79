"""Diagnostic: the adversarial test's exact sequence vs float64, with and without the generator phase."""
import os, sys
R0 = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R0, os.path.join(R0, "tests", "golden"), os.path.join(R0, "tests")):
    sys.path.insert(0, p)
import torch, torch.nn.functional as F
from golden_io import golden_state, load_case
from weights import synth_param
from oracle import torch_ref as R
from medvae_disentangled_multimodal_amd import ops
from medvae_disentangled_multimodal_amd.discriminator import NLayerDiscriminator
from medvae_disentangled_multimodal_amd.encoder_decoder import Conv2d
from medvae_disentangled_multimodal_amd.losses import LPIPSWithDiscriminator
dev = torch.device("cuda:0")
meta, data = load_case("disc")
st = golden_state(meta)
rel = lambda a, b: float((a.detach().double().cpu() - b.detach().double().cpu()).norm() / b.detach().double().cpu().norm().clamp_min(1e-30))
cl = lambda t: t.to(dev).contiguous(memory_format=torch.channels_last)
W = {k: v.double().requires_grad_() for k, v in st.items()}
x64 = torch.from_numpy(data["in.x"]).double(); feat64 = torch.from_numpy(data["in.feat"]).double()
wl = torch.from_numpy(synth_param("last.weight", (3, 8, 3, 3))); bl = torch.from_numpy(synth_param("last.bias", (3,)))
rec64 = F.conv2d(feat64, wl.double(), bl.double(), padding=1)
lr64 = R.discriminator(W, x64); lf64 = R.discriminator(W, rec64)
R.hinge_d_loss(lr64, lf64).backward()
for gen in (False, True):
    for order in ("real_first",):
        D = NLayerDiscriminator(3, 64, 3).to(dev)
        D.load_state_dict({k: v.to(dev) for k, v in st.items()}, strict=False)
        D.train()
        last = Conv2d(8, 3, 3, 1, 1).to(dev)
        with torch.no_grad():
            last.weight.copy_(wl); last.bias.copy_(bl)
        x = cl(torch.from_numpy(data["in.x"])); feat = cl(torch.from_numpy(data["in.feat"]))
        rec = last(feat)
        if gen:
            for p in D.parameters(): p.requires_grad_(False)
            g_loss = ops.neg_mean(D(rec))
            nll = ops.mse_mean(rec, x)
            dw = LPIPSWithDiscriminator.calculate_adaptive_weight(None, nll, g_loss, last)
            for p in D.parameters(): p.requires_grad_(True)
        if order == "real_first":
            lr = D(x); lf = D(rec.detach())
        else:
            lf = D(rec.detach()); lr = D(x)
        d = 0.5 * (ops.hinge_real(lr) + ops.hinge_fake(lf))
        d.backward()
        errs = {k: rel(p.grad, W[k].grad) for k, p in D.named_parameters() if not k.endswith(("2.bias", "5.bias", "8.bias"))}
        print(f"gen={gen} {order}: lr {rel(lr, lr64):.1e} lf {rel(lf, lf64):.1e} rec {rel(rec, rec64):.1e}",
              " ".join(f"{k}:{v:.1e}" for k, v in errs.items()))
