"""Rows (f)1 / (f)3 pinned on the reference itself: tests/golden/make_ref_fixtures.py ran the reference's own
pure-torch functions (mixed_modality_collate_fn, MedMNISTDataset.__getitem__'s channel conversion / label
standardisation / one-hot, compute_kl_metrics, the MSE / MAE of compute_reconstruction_metrics) in the build
container. Here the CPU restatements -- oracle/data_ref.py, the host logic of the device pipeline
(medvae_disentangled_multimodal_amd/data.py: modality table, target channels, label standardisation) and
oracle/torch_ref.kl_metrics -- are checked against those vectors: images / collate bitwise, labels / one-hot /
indices exactly, metrics to 1e-6 relative. (transforms.ToTensor / Normalize / the train augmentations and
torchmetrics' PSNR / SSIM stay unpinned: torchvision and torchmetrics are not installed.)"""
import os

import numpy as np
import pytest
import torch

from oracle import data_ref as D
from oracle import torch_ref as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ref_data():
    return dict(np.load(os.path.join(GOLDEN, "ref_data.npz"), allow_pickle=False))


@pytest.fixture(scope="module")
def ref_metrics():
    return dict(np.load(os.path.join(GOLDEN, "ref_metrics.npz"), allow_pickle=False))


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("size", [28, 64])
def test_getitem_and_collate_vs_reference(ref_data, size):
    from medvae_disentangled_multimodal_amd import data
    p = f"s{size}."
    items = [str(s) for s in ref_data[p + "items"]]
    imgs = []
    for it in items:
        name, k = it.split(":")
        k = int(k)
        u8 = ref_data[f"{p}{name}.u8"][k]
        img = D.convert_channels(D.to_tensor(u8), data.target_channels(name))
        assert _bits_equal(img.numpy(), ref_data[f"{p}{name}.{k}.image"]), it
        lab = data.standardize_labels(ref_data[f"{p}{name}.labels"])[k]
        assert ref_data[f"{p}{name}.{k}.label"].tolist() == [int(lab)], it
        oh = np.zeros(12, np.float32)
        oh[data.MODALITIES.index(name)] = 1
        assert _bits_equal(oh, ref_data[f"{p}{name}.{k}.onehot"]), it
        assert int(ref_data[f"{p}{name}.{k}.idx"]) == data.MODALITIES.index(name)
        imgs.append(img)
    for b in ("mixed", "gray"):
        sel = ref_data[f"{p}collate.{b}.select"].tolist()
        x = D.collate([imgs[i] for i in sel])
        assert _bits_equal(x.numpy(), ref_data[f"{p}collate.{b}.x"]), b
    assert ref_data[f"{p}collate.mixed.x"].shape[1] == 3 and ref_data[f"{p}collate.gray.x"].shape[1] == 1


@pytest.mark.parametrize("tag", ["flat", "spatial"])
def test_kl_metrics_vs_reference(ref_metrics, tag):
    mean = torch.from_numpy(ref_metrics[f"kl.{tag}.mean"])
    logvar = torch.from_numpy(ref_metrics[f"kl.{tag}.logvar"])
    got = R.kl_metrics(mean, logvar)
    for k, v in got.items():
        assert v == pytest.approx(float(ref_metrics[f"kl.{tag}.{k}"]), rel=1e-6, abs=1e-9), k


def test_mse_mae_vs_reference(ref_metrics):
    x, r = torch.from_numpy(ref_metrics["recon.x"]), torch.from_numpy(ref_metrics["recon.rec"])
    got = R.reconstruction_metrics(x, r)
    assert got["mse"] == pytest.approx(float(ref_metrics["recon.mse"]), rel=1e-6)
    assert got["mae"] == pytest.approx(float(ref_metrics["recon.mae"]), rel=1e-6)
