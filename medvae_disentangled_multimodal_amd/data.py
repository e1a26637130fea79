"""On-device MedMNIST input pipeline.

Replaces the reference's CPU DataLoader path (src/data/medmnist_data.py): MedMNISTDataModule
(:257-440) over ConcatDataset(MedMNISTDataset per dataset name) with `mixed_modality_collate_fn`
(:16-72). The uint8 images of every requested dataset are uploaded once and stay resident in HBM
(MedMNIST at 64x64 is ~4 KB/image: all twelve datasets fit easily); a batch is one HIP launch
(`mvae_decode_batch`, csrc/data.hip) that gathers the sampled images and applies the reference's
per-sample transform -- ToTensor, modality channel conversion, [train] horizontal flip / rotation
(+-10 deg, nearest) / brightness+contrast jitter (0.1) in torchvision's order, Normalize(0.5, 0.5) --
and the collate's zero-padding, and writes the (x, labels, onehot, modality_idx) batch contract.

Sampling follows DistributedSampler(shuffle=True): per epoch a permutation seeded with seed+epoch,
padded to a multiple of world_size, rank-strided. Random augmentation parameters are drawn on the host
from a seeded generator (torchvision's distributions); their exact torch RNG stream is not
reproduced (parity for augmentation is given-parameters, see tests/test_gpu_data.py).

Files: `{root}/{name}.npz` (28x28) or `{root}/{name}_{size}.npz`, MedMNIST's own layout
(`{split}_images` uint8 [N,H,W] or [N,H,W,3], `{split}_labels` [N,L]); loaded with
numpy.load(allow_pickle=False).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib, ops

# src/data/medmnist_data.py:132-149 (modality index = position in this list; one-hot length 12)
MODALITIES = ["chestmnist", "pathmnist", "octmnist", "pneumoniamnist", "dermamnist", "bloodmnist",
              "tissuemnist", "retinamnist", "breastmnist", "organamnist", "organcmnist", "organsmnist"]
# :154-184 target channels per modality (gray modalities stay 1-channel, the rest become RGB)
GRAY_MODALITIES = {"chestmnist", "pneumoniamnist", "organamnist", "organcmnist", "organsmnist"}


def target_channels(name: str) -> int:
    return 1 if name in GRAY_MODALITIES else 3


def standardize_labels(labels: np.ndarray) -> np.ndarray:
    """__getitem__'s label standardisation (:225-241): scalar/1-element labels as they are,
    multi-label rows -> argmax if any positive else 0. Returns int64 [N]."""
    lab = np.asarray(labels).reshape(len(labels), -1).astype(np.int64)
    if lab.shape[1] == 1:
        return lab[:, 0].copy()
    out = np.where(lab.sum(1) > 0, lab.argmax(1), 0)
    return out.astype(np.int64)


def npz_path(root: str, name: str, size: int) -> str:
    return os.path.join(root, f"{name}.npz" if size == 28 else f"{name}_{size}.npz")


class DistributedSampler:
    """torch.utils.data.DistributedSampler(shuffle=True, drop_last=False) index semantics."""

    def __init__(self, n: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0):
        self.n, self.num_replicas, self.rank, self.shuffle, self.seed = n, num_replicas, rank, shuffle, seed
        self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> List[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        pad = self.total_size - len(idx)
        if pad > 0:
            idx += (idx * math.ceil(pad / len(idx)))[:pad]
        return idx[self.rank:self.total_size:self.num_replicas]


def draw_augmentation(n: int, h: int, w: int, rng: np.random.Generator) -> np.ndarray:
    """Per-sample parameters of RandomHorizontalFlip(0.5), RandomRotation(10), ColorJitter(0.1, 0.1)
    in the kernel's layout (12 float32 per sample, see csrc/data.hip SampleAug)."""
    aug = np.zeros((n, 12), dtype=np.float32)
    for k in range(n):
        flip = rng.random() < 0.5
        angle = rng.uniform(-10.0, 10.0)
        rot = math.radians(-angle)  # F.rotate -> _get_inverse_affine_matrix(center, -angle, ...)
        m = np.array([math.cos(rot), math.sin(rot), -math.sin(rot), math.cos(rot)], dtype=np.float32)
        bright = rng.uniform(0.9, 1.1)
        contrast = rng.uniform(0.9, 1.1)
        perm = rng.permutation(4)  # ColorJitter.get_params: fn_idx = randperm(4)
        order = 0.0 if list(perm).index(0) < list(perm).index(1) else 1.0
        aug[k] = set_aug_row(flip, m, w, h, bright, contrast, order)
    return aug


def set_aug_row(flip: bool, m: np.ndarray, w: int, h: int, bright: float, contrast: float, order: float):
    """m = float32 [cos, sin, -sin, cos] of the inverse rotation (torchvision's theta rows)."""
    hw, hh = np.float32(0.5 * w), np.float32(0.5 * h)
    return np.array([1.0 if flip else 0.0, m[0] / hw, m[1] / hw, m[2] / hh, m[3] / hh,
                     np.float32(bright), np.float32(1.0 - bright), np.float32(contrast), np.float32(1.0 - contrast),
                     order, 0.0, 0.0], dtype=np.float32)


class DeviceMedMNIST:
    """The images of several MedMNIST datasets (one split) resident on the GPU, in ConcatDataset order."""

    def __init__(self, dataset_names: Sequence[str], split: str = "train", size: int = 28, root: str = "./data",
                 device="cuda", arrays: Optional[Dict[str, Tuple[np.ndarray, np.ndarray]]] = None):
        self.names = [n.lower() for n in dataset_names]
        self.split, self.size, self.device = split, size, torch.device(device)
        chunks, offs, nat, tgt, mod, lab = [], [], [], [], [], []
        off = 0
        self.lengths = []
        for name in self.names:
            if name not in MODALITIES:
                raise ValueError(f"Unknown dataset: {name}")
            if arrays is not None:
                imgs, labels = arrays[name]
            else:
                with np.load(npz_path(root, name, size), allow_pickle=False) as f:
                    imgs, labels = f[f"{split}_images"], f[f"{split}_labels"]
            imgs = np.ascontiguousarray(imgs, dtype=np.uint8)
            if imgs.ndim == 3:
                imgs = imgs[..., None]
            n, h, w, c = imgs.shape
            if (h, w) != (size, size):
                raise ValueError(f"{name}: images are {h}x{w}, expected {size}x{size} (no resize on device)")
            per = h * w * c
            chunks.append(imgs.reshape(-1))
            offs.append(off + np.arange(n, dtype=np.int64) * per)
            off += n * per
            nat += [c] * n
            tgt += [target_channels(name)] * n
            mod += [MODALITIES.index(name)] * n
            lab.append(standardize_labels(labels))
            self.lengths.append(n)
        dev = self.device
        self.store = torch.from_numpy(np.concatenate(chunks)).to(dev)
        self.offset = torch.from_numpy(np.concatenate(offs)).to(dev)
        self.channels = torch.tensor(nat, dtype=torch.int32, device=dev)
        self.targets = torch.tensor(tgt, dtype=torch.int32, device=dev)
        self.modality = torch.tensor(mod, dtype=torch.int32, device=dev)
        self.labels = torch.from_numpy(np.concatenate(lab)).to(dev)
        self._targets_host = np.asarray(tgt, dtype=np.int32)
        self.n = len(tgt)

    def __len__(self):
        return self.n

    def batch(self, index: Sequence[int], aug: Optional[np.ndarray] = None):
        """(x [B,C,H,W] channels_last, labels [B,1] int64, onehot [B,12], modality_idx [B] int64) for the
        given global sample indices; C = max target channels in the batch (the collate's padding)."""
        idx_np = np.asarray(index, dtype=np.int64)
        nb = len(idx_np)
        cout = int(self._targets_host[idx_np].max())
        dev = self.device
        idx = torch.from_numpy(idx_np).to(dev, non_blocking=True)
        h = w = self.size
        x = torch.empty((nb, cout, h, w), device=dev, dtype=torch.float32, memory_format=torch.channels_last)
        onehot = torch.empty((nb, len(MODALITIES)), device=dev, dtype=torch.float32)
        midx = torch.empty(nb, device=dev, dtype=torch.int64)
        labels = torch.empty(nb, device=dev, dtype=torch.int64)
        a = torch.from_numpy(np.ascontiguousarray(aug, dtype=np.float32)).to(dev) if aug is not None else None
        ws = ops.ARENA.get("decode", _lib.query("mvae_decode_batch_workspace_bytes", nb, h), dev)
        _lib.call("mvae_decode_batch", self.store.data_ptr(), self.offset.data_ptr(), self.channels.data_ptr(),
                  self.targets.data_ptr(), self.modality.data_ptr(), self.labels.data_ptr(), idx.data_ptr(),
                  ops._ptr(a), nb, h, w, cout, len(MODALITIES), x.data_ptr(), onehot.data_ptr(), midx.data_ptr(),
                  labels.data_ptr(), ws.data_ptr(), ws.numel(), ops._stream(x))
        return x, labels.view(nb, 1), onehot, midx


class DeviceDataLoader:
    """Iterates (x, labels, onehot, modality_idx) batches of a DeviceMedMNIST on the GPU:
    DistributedSampler order, drop_last=False, training augmentation when `augment`."""

    def __init__(self, dataset: DeviceMedMNIST, batch_size: int, shuffle: bool = True, augment: bool = False,
                 seed: int = 0, num_replicas: int = 1, rank: int = 0):
        self.ds, self.batch_size, self.augment = dataset, batch_size, augment
        self.sampler = DistributedSampler(len(dataset), num_replicas, rank, shuffle, seed)
        self.seed, self.rank = seed, rank

    def set_epoch(self, epoch: int):
        self.sampler.set_epoch(epoch)

    def __len__(self):
        return math.ceil(self.sampler.num_samples / self.batch_size)

    def __iter__(self) -> Iterator:
        idx = self.sampler.indices()
        rng = np.random.default_rng([self.seed, self.sampler.epoch, self.rank])
        for s in range(0, len(idx), self.batch_size):
            chunk = idx[s:s + self.batch_size]
            aug = draw_augmentation(len(chunk), self.ds.size, self.ds.size, rng) if self.augment else None
            yield self.ds.batch(chunk, aug)
