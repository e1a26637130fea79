"""Host-side logic that needs no GPU: `_target_` config instantiation against the reference's own
YAML (when the reference checkout is present), parameter naming / init parity with the reference,
schedulers, conv geometry and the flat parameter buffer layout."""
import json
import os

import pytest
import torch

from cases import CASES
from golden_io import GOLDEN

REF_CFG = "/root/reference/configs/model"


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference checkout not present")
@pytest.mark.parametrize("fname", ["base_vae.yaml", "beta_vae.yaml", "conditional_vae.yaml"])
def test_reference_model_yaml_instantiates(fname):
    from medvae_disentangled_multimodal_amd import config
    cfg = config.load_yaml(os.path.join(REF_CFG, fname))
    # the reference's defaults are 224x224 ImageNet-size models; keep the architecture, shrink sizes
    m = config.instantiate(cfg, hidden_channels=16, resolution=32, latent_dim=4)
    assert type(m).__name__ == cfg["_target_"].rsplit(".", 1)[1]
    names = [k for k, _ in m.state_dict().items()]
    assert names[0] == "encoder.conv_in.weight"


@pytest.mark.parametrize("name", sorted(CASES))
def test_state_dict_names_and_seeded_init_match_reference(name):
    import medvae_disentangled_multimodal_amd as M
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        meta = json.load(f)
    torch.manual_seed(0)
    m = getattr(M, CASES[name]["cls"])(**CASES[name]["kwargs"])
    sd = m.state_dict()
    assert [[k, list(v.shape)] for k, v in sd.items()] == meta["params"]
    for k, v in sd.items():
        s, s2 = meta["seeded_init_torch_seed0"][k]
        assert abs(float(v.double().sum()) - s) <= 1e-5 * max(1.0, abs(s)), k
        assert abs(float((v.double() ** 2).sum()) - s2) <= 1e-6 * max(1.0, s2), k


def test_conv_geometry_matches_reference_shapes():
    from medvae_disentangled_multimodal_amd.ops import ConvGeom
    down = ConvGeom(3, 3, 2, 0, 0, 1, 1)          # Downsample: 28->14->7->3 (SURVEY note 3)
    assert [down.out_hw(h, h)[0] for h in (28, 14, 7, 64, 32)] == [14, 7, 3, 32, 16]
    up = ConvGeom(3, 3, 1, 1, 1, 1, 1, upsample=True)
    assert up.out_hw(7, 7) == (14, 14)
    assert ConvGeom(3, 3, 1, 1, 1, 1, 1).out_hw(28, 28) == (28, 28)


def test_flat_parameters_layout_and_krsc_views():
    from medvae_disentangled_multimodal_amd.optim import FlatParameters
    conv = torch.nn.Conv2d(3, 8, 3)
    lin = torch.nn.Linear(5, 2)
    mod = torch.nn.ModuleDict({"c": conv, "l": lin})
    ref = {k: v.detach().clone() for k, v in mod.state_dict().items()}
    f = FlatParameters(mod, torch.device("cpu"))
    for k, v in mod.state_dict().items():
        assert torch.equal(v, ref[k])
    assert conv.weight.is_contiguous(memory_format=torch.channels_last)   # KRSC physical layout
    assert all(o % 4 == 0 for o in f.offsets)                             # 16-byte aligned tensors
    assert conv.weight.grad.data_ptr() == f.grad.data_ptr() + 4 * f.offsets[0]
    assert f.tensor_chunk_begin.tolist()[-1] == f.nchunks


def test_schedulers_follow_reference_defaults():
    from medvae_disentangled_multimodal_amd.schedulers import get_scheduler
    p = [torch.nn.Parameter(torch.zeros(1))]
    opt = torch.optim.SGD(p, lr=1.0)
    assert get_scheduler(opt, {"type": "none"}) is None
    s = get_scheduler(opt, {"type": "step", "step_size": 5, "gamma": 0.5})
    assert s.step_size == 5 and s.gamma == 0.5
    s = get_scheduler(opt, {"type": "multistep"})
    assert sorted(s.milestones) == [50, 100]
    with pytest.raises(ValueError):
        get_scheduler(opt, {"type": "bogus"})


def test_ops_refuse_cpu_tensors():
    from medvae_disentangled_multimodal_amd import ops
    x = torch.zeros(1, 4, 4, 4)
    w = torch.zeros(4, 4, 3, 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.conv2d(x, w, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1))


def test_distributed_sampler_semantics():
    """data.DistributedSampler == torch.utils.data.DistributedSampler(shuffle=True, drop_last=False)."""
    import torch.utils.data as tud
    from medvae_disentangled_multimodal_amd.data import DistributedSampler, standardize_labels
    ds = list(range(23))
    for world in (1, 2, 4):
        for rank in range(world):
            ref = tud.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=7)
            ref.set_epoch(3)
            mine = DistributedSampler(23, world, rank, True, 7)
            mine.set_epoch(3)
            assert mine.indices() == list(iter(ref))
    import numpy as np
    assert standardize_labels(np.array([[3], [1]])).tolist() == [3, 1]
    assert standardize_labels(np.array([[0, 1, 1], [0, 0, 0]])).tolist() == [1, 0]


def test_grad_sink_park_take_semantics():
    """GradSink (ops.py): producer parks, consumer takes; a consumer that ran first closes the sink so
    the producer returns its gradient to autograd instead (correct in either engine order)."""
    from medvae_disentangled_multimodal_amd import ops
    s = ops.GradSink()
    g = torch.ones(3)
    assert s.park(g) and s.take() is g and s.g is None and not s.closed
    s2 = ops.GradSink()
    assert s2.take() is None and s2.closed and not s2.park(g)
    s3 = ops.GradSink()  # stale park (partial backward) is replaced by the next pass's gradient
    assert s3.park(torch.zeros(3)) and s3.park(g) and s3.take() is g
