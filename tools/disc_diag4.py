"""Diagnostic: main.0 parameter gradients per hinge branch (real / fake / both) vs float64."""
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
dev = torch.device("cuda:0")
meta, data = load_case("disc")
st = golden_state(meta)
rel = lambda a, b: float((a.detach().double().cpu() - b.detach().double().cpu()).norm() / b.detach().double().cpu().norm().clamp_min(1e-30))
x64 = torch.from_numpy(data["in.x"]).double(); feat64 = torch.from_numpy(data["in.feat"]).double()
rec64 = F.conv2d(feat64, torch.from_numpy(synth_param("last.weight", (3, 8, 3, 3))).double(),
                 torch.from_numpy(synth_param("last.bias", (3,))).double(), padding=1)
def ref(which):
    W = {k: v.double().requires_grad_() for k, v in st.items()}
    l = 0
    if "real" in which: l = l + 0.5 * F.relu(1 - R.discriminator(W, x64)).mean()
    if "fake" in which: l = l + 0.5 * F.relu(1 + R.discriminator(W, rec64)).mean()
    l.backward()
    return W
def ours(which, two_forward):
    D = NLayerDiscriminator(3, 64, 3).to(dev)
    D.load_state_dict({k: v.to(dev) for k, v in st.items()}, strict=False)
    D.train()
    x = x64.float().to(dev).contiguous(memory_format=torch.channels_last)
    rec = rec64.float().to(dev).contiguous(memory_format=torch.channels_last)
    lr_ = D(x) if ("real" in which or two_forward) else None
    lf = D(rec) if ("fake" in which or two_forward) else None
    l = 0
    if "real" in which: l = l + 0.5 * ops.hinge_real(lr_)
    if "fake" in which: l = l + 0.5 * ops.hinge_fake(lf)
    l.backward()
    return dict(D.named_parameters())
for which in (("real",), ("fake",), ("real", "fake")):
    Wr = ref(which)
    for tf in (False, True):
        P = ours(which, tf)
        print(which, "two_fwd" if tf else "one_fwd", {k: f"{rel(P[k].grad, Wr[k].grad):.1e}" for k in ("main.0.weight", "main.0.bias", "main.2.weight", "main.3.bias")})
