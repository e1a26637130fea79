"""Decode-only paths (base_vae.py:79-129 decode/sample, conditional_vae.py:166-188
conditional_sample/get_modality_condition, disentangled_conditional_vae.py:456-482
sample_conditional; generate.py:18-104 drives them): decode(z) of the reference's golden latents
reproduces the golden reconstructions (the reference's decoder output) within 1e-3, and the
sampling entry points draw z ~ N(0, I) of the reference's latent shape."""
import pytest
import torch

from cases import CASES
from golden_io import golden_state, load_case, rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["base_attn", "beta_c2", "cvae_c4"])
def test_decode_matches_golden(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import medvae_disentangled_multimodal_amd as M
    dev = torch.device("cuda:0")
    meta, data = load_case(name)
    case = CASES[name]
    if case["kwargs"].get("dropout", 0.0):
        pytest.skip("dropout active in the golden forward")
    model = getattr(M, case["cls"])(**case["kwargs"])
    model.load_state_dict(golden_state(meta))
    model = model.to(dev).eval()
    z = torch.from_numpy(data["out.z"]).to(dev)
    with torch.no_grad():
        rec = model.decode(z)
    assert rel_err(rec.cpu(), data["out.reconstruction"]) < 1e-3
    torch.manual_seed(0)
    with torch.no_grad():
        s1 = model.sample(3, dev)
    torch.manual_seed(0)
    with torch.no_grad():
        s2 = model.sample(3, dev)
    assert s1.shape == (3, *rec.shape[1:]) and torch.isfinite(s1).all() and torch.equal(s1, s2)
    if case["cls"] == "ConditionalVAE":
        c = model.get_modality_condition(model.modalities[1])
        assert c.tolist() == [1.0 if i == 1 else 0.0 for i in range(model.num_modalities)]
        with torch.no_grad():
            s3 = model.conditional_sample(2, c.unsqueeze(0).repeat(2, 1).to(dev), dev)
        assert s3.shape == (2, *rec.shape[1:])


def test_disentangled_sample_conditional():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import medvae_disentangled_multimodal_amd as M
    dev = torch.device("cuda:0")
    meta, data = load_case("dis_c3")
    case = CASES["dis_c3"]
    model = getattr(M, case["cls"])(**case["kwargs"])
    model.load_state_dict(golden_state(meta))
    model = model.to(dev).eval()
    idx = torch.tensor([0, 1, 4, 3], device=dev)
    with torch.no_grad():
        s = model.sample_conditional(4, idx, dev)
    assert s.shape[0] == 4 and torch.isfinite(s).all()
