"""On-device MedMNIST batches vs the CPU oracle of the reference's __getitem__ + transforms +
collate (oracle/data_ref.py; torchvision restated, not installed). Synthetic uint8 datasets in the
MedMNIST npz layout. Evaluation transform: bit-exact. Training transform with the SAME explicit
random parameters: rotated coordinates may round differently only on exact ties (< 0.5 % of
pixels), jitter values within 2e-6."""
import math
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import data_ref as D

pytestmark = pytest.mark.gpu


def _arrays(size, seed=0):
    rng = np.random.default_rng(seed)
    return {
        "chestmnist": (rng.integers(0, 256, (5, size, size), dtype=np.uint8), rng.integers(0, 2, (5, 14))),
        "pathmnist": (rng.integers(0, 256, (4, size, size, 3), dtype=np.uint8), rng.integers(0, 9, (4, 1))),
        "octmnist": (rng.integers(0, 256, (3, size, size), dtype=np.uint8), rng.integers(0, 4, (3, 1))),
        "organamnist": (rng.integers(0, 256, (3, size, size, 3), dtype=np.uint8), rng.integers(0, 11, (3, 1))),
    }


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _oracle_batch(arrs, names, index, augs=None):
    flat = []
    for n in names:
        imgs, labels = arrs[n]
        for k in range(len(imgs)):
            flat.append((n, imgs[k]))
    ims = [D.sample(flat[i][1], flat[i][0], None if augs is None else augs[j]) for j, i in enumerate(index)]
    return D.collate(ims)


@pytest.mark.parametrize("size", [28, 64])
def test_eval_batch_bit_exact(dev, size):
    from medvae_disentangled_multimodal_amd import data
    arrs = _arrays(size)
    names = list(arrs)
    with tempfile.TemporaryDirectory() as d:  # through the npz files, MedMNIST layout
        for n, (im, lab) in arrs.items():
            np.savez(data.npz_path(d, n, size), train_images=im, train_labels=lab)
        ds = data.DeviceMedMNIST(names, "train", size, d, device=dev)
    assert len(ds) == 15
    index = [0, 6, 9, 14, 3, 12]
    x, labels, onehot, midx = ds.batch(index)
    ref = _oracle_batch(arrs, names, index)
    assert x.shape == ref.shape and x.is_contiguous(memory_format=torch.channels_last)
    diff = (x.cpu() - ref).abs()
    assert torch.equal(x.cpu(), ref), (int((diff > 0).sum()), float(diff.max()), torch.nonzero(diff)[:5].tolist())
    mods = [data.MODALITIES.index(n) for n in names for _ in range(len(arrs[n][0]))]
    assert midx.cpu().tolist() == [mods[i] for i in index]
    assert torch.equal(onehot.cpu(), torch.nn.functional.one_hot(midx.cpu(), 12).float())
    all_labels = np.concatenate([data.standardize_labels(arrs[n][1]) for n in names])
    assert labels.view(-1).cpu().tolist() == all_labels[index].tolist()
    # gray-only batch keeps 1 channel (no padding), as the collate does
    x1, *_ = ds.batch([0, 1])
    assert x1.shape[1] == 1


def test_train_batch_matches_given_parameters(dev):
    from medvae_disentangled_multimodal_amd import data
    size = 64
    arrs = _arrays(size, 1)
    names = list(arrs)
    ds = data.DeviceMedMNIST(names, "train", size, arrays=arrs, device=dev)
    index = list(range(15))
    rng = np.random.default_rng(5)
    aug = data.draw_augmentation(len(index), size, size, rng)
    # the same parameters in the oracle's form
    rng = np.random.default_rng(5)
    params = []
    for _ in index:
        flip = rng.random() < 0.5
        angle = rng.uniform(-10.0, 10.0)
        b, c = rng.uniform(0.9, 1.1), rng.uniform(0.9, 1.1)
        perm = list(rng.permutation(4))
        params.append((flip, angle, b, c, perm.index(0) < perm.index(1)))
    x, *_ = ds.batch(index, aug)
    ref = _oracle_batch(arrs, names, index, params)
    diff = (x.cpu() - ref).abs()
    assert float((diff > 2e-6).float().mean()) < 5e-3
    assert float(diff.median()) == 0.0


def test_loader_sharding_and_epochs(dev):
    from medvae_disentangled_multimodal_amd import data
    arrs = _arrays(28, 2)
    ds = data.DeviceMedMNIST(list(arrs), "train", 28, arrays=arrs, device=dev)
    seen = []
    for rank in range(2):
        dl = data.DeviceDataLoader(ds, batch_size=4, shuffle=True, augment=True, seed=3, num_replicas=2, rank=rank)
        n = 0
        for x, labels, onehot, midx in dl:
            assert x.shape[0] <= 4 and torch.isfinite(x).all()
            assert float(x.min()) >= -1.0 and float(x.max()) <= 1.0
            n += x.shape[0]
        assert n == math.ceil(15 / 2)
        seen += dl.sampler.indices()
    assert sorted(set(seen)) == list(range(15))


@pytest.mark.parametrize("size", [28, 64])
def test_eval_batch_vs_reference_fixture(dev, size):
    """The device pipeline against the vectors the reference's own __getitem__ + mixed_modality_collate_fn produced
    (tests/golden/make_ref_fixtures.py), evaluation transform = Normalize(0.5, 0.5) applied to them in float32
    (torchvision's `sub(mean).div(std)`; torchvision itself is unpinned): images bitwise, labels / one-hot / indices
    exactly."""
    from medvae_disentangled_multimodal_amd import data
    ref = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_data.npz"),
                       allow_pickle=False))
    p = f"s{size}."
    items = [str(s).split(":") for s in ref[p + "items"]]
    names = list(dict.fromkeys(n for n, _ in items))
    arrays = {n: (ref[f"{p}{n}.u8"], ref[f"{p}{n}.labels"]) for n in names}
    ds = data.DeviceMedMNIST(names, "train", size, device=dev, arrays=arrays)
    for b in ("mixed", "gray"):
        sel = ref[f"{p}collate.{b}.select"].tolist()
        x, labels, onehot, midx = ds.batch(sel)
        # Normalize runs per sample in __getitem__, before the collate pads gray samples with zero channels
        want = torch.from_numpy(ref[f"{p}collate.{b}.x"]).sub(0.5).div(0.5)
        for j, i in enumerate(sel):
            if data.target_channels(items[i][0]) < want.shape[1]:
                want[j, 1:] = 0.0
        assert x.shape == want.shape
        assert torch.equal(x.cpu().contiguous(), want), b
        assert labels.cpu().tolist() == ref[f"{p}collate.{b}.labels"].tolist()
        assert torch.equal(onehot.cpu(), torch.from_numpy(ref[f"{p}collate.{b}.onehot"]))
        assert midx.cpu().tolist() == ref[f"{p}collate.{b}.idx"].tolist()
