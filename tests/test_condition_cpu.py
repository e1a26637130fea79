"""The one-hot conditioning path of ConditionalVAE (src/models/conditional_vae.py:65-69, 107-136) restated bit for
bit (oracle/torch_ref.py:condition_map_exact) and pinned on the CPU: against torch's own Linear + ReLU + bilinear
interpolate (the reference's arithmetic) on random inputs, and against the condition maps the reference itself
produced for the golden cases (tests/golden/make_golden.py: out.cond_proj / out.cond_map). north_star asks the
one-hot modality-conditioning index path to be bit-exact: every comparison here is bitwise."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_io import golden_state, load_case
from oracle.torch_ref import _fma32, condition_map_exact


def _bits_equal(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.int32), b.view(np.int32))


def test_fma32_is_correctly_rounded():
    from fractions import Fraction
    rng = np.random.default_rng(0)
    a = rng.standard_normal(4000).astype(np.float32)
    b = rng.standard_normal(4000).astype(np.float32)
    c = rng.standard_normal(4000).astype(np.float32) * np.float32(1e-3)
    r = _fma32(a, b, c)
    for i in range(0, 4000, 97):
        ex = Fraction(float(a[i])) * Fraction(float(b[i])) + Fraction(float(c[i]))
        cand = [np.float32(r[i]), np.nextafter(r[i], np.float32(np.inf)), np.nextafter(r[i], np.float32(-np.inf))]
        errs = [abs(Fraction(float(v)) - ex) for v in cand]
        assert errs[0] <= min(errs), i


@pytest.mark.parametrize("H,W", [(64, 64), (28, 28), (32, 32), (28, 64)])
def test_condition_map_matches_torch_cpu_bitwise(H, W):
    g = torch.Generator().manual_seed(H * 7 + W)
    C, K, B = 3, 12, 6
    w = torch.randn(C * 64, K, generator=g) * 0.3
    b = torch.randn(C * 64, generator=g) * 0.3
    idx = torch.randint(0, K, (B,), generator=g)
    oh = F.one_hot(idx, K).float()
    pre_t = F.linear(oh, w, b)
    map_t = F.interpolate(F.relu(pre_t).view(B, C, 8, 8), size=(H, W), mode="bilinear", align_corners=False)
    pre, cmap = condition_map_exact(w.numpy(), b.numpy(), oh.numpy(), C, H, W)
    assert _bits_equal(pre, pre_t.numpy())
    assert _bits_equal(pre, (w.t()[idx] + b).numpy())  # the index path: column selection + bias
    assert _bits_equal(cmap, map_t.numpy())


@pytest.mark.parametrize("case", ["cvae_c4", "cvae_c4_full"])
def test_condition_map_matches_reference_fixture_bitwise(case):
    meta, d = load_case(case)
    W = {k: v.numpy() for k, v in golden_state(meta).items()}
    C = meta["case"]["kwargs"]["input_channels"]
    x = d["in.x"]
    pre, cmap = condition_map_exact(W["condition_proj.0.weight"], W["condition_proj.0.bias"], d["in.cond"], C,
                                    x.shape[2], x.shape[3])
    assert _bits_equal(pre, d["out.cond_proj"])
    assert _bits_equal(cmap, d["out.cond_map"])
