"""CPU oracle of the reference's per-sample input path (TEST INFRASTRUCTURE ONLY).

Restates src/data/medmnist_data.py: MedMNISTDataset.__getitem__ (:186-251: ToTensor, modality
channel conversion, label standardisation), the modality transform of
MedMNISTDataModule._get_modality_transform (:341-375: [train] RandomHorizontalFlip(0.5),
RandomRotation(10), ColorJitter(brightness=0.1, contrast=0.1); Normalize(0.5, 0.5)) and
mixed_modality_collate_fn (:16-72). torchvision 0.22.1 (uv.lock:4088) is not installed here: its
tensor kernels used by those transforms are restated from its published code --
F.hflip (flip of the last dim), F.rotate (_get_inverse_affine_matrix + _gen_affine_grid +
grid_sample nearest / zeros / align_corners=False), F.adjust_brightness / adjust_contrast (_blend,
rgb_to_grayscale 0.2989/0.587/0.114), F.normalize. Random draws are explicit parameters.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

GRAY = {"chestmnist", "pneumoniamnist", "organamnist", "organcmnist", "organsmnist"}


def to_tensor(img: np.ndarray) -> torch.Tensor:
    """transforms.ToTensor on an HxW or HxWx3 uint8 array -> [C,H,W] float in [0,1]."""
    t = torch.from_numpy(np.ascontiguousarray(img))
    if t.dim() == 2:
        t = t[:, :, None]
    return t.permute(2, 0, 1).contiguous().to(torch.float32).div(255)


def convert_channels(image: torch.Tensor, target: int) -> torch.Tensor:
    """__getitem__ :208-218."""
    if target == 1 and image.shape[0] == 3:
        return (0.299 * image[0] + 0.587 * image[1] + 0.114 * image[2]).unsqueeze(0)
    if target == 3 and image.shape[0] == 1:
        return image.repeat(3, 1, 1)
    return image


def rotate_nearest(img: torch.Tensor, angle: float) -> torch.Tensor:
    """torchvision.transforms.functional.rotate(img, angle, NEAREST, expand=False, center=None, fill=None)."""
    c, h, w = img.shape
    rot = math.radians(-angle)
    # _get_inverse_affine_matrix(center=[0,0], -angle, [0,0], 1.0, [0,0]), inverted
    a, b, cc, d = math.cos(rot), -math.sin(rot), math.sin(rot), math.cos(rot)
    matrix = [d, -b, 0.0, -cc, a, 0.0]
    theta = torch.tensor(matrix, dtype=torch.float32).reshape(1, 2, 3)
    # _gen_affine_grid
    base = torch.empty(1, h, w, 3, dtype=torch.float32)
    base[..., 0].copy_(torch.linspace(-w * 0.5 + 0.5, w * 0.5 + 0.5 - 1, steps=w))
    base[..., 1].copy_(torch.linspace(-h * 0.5 + 0.5, h * 0.5 + 0.5 - 1, steps=h).unsqueeze_(-1))
    base[..., 2].fill_(1)
    rescaled = theta.transpose(1, 2) / torch.tensor([0.5 * w, 0.5 * h], dtype=torch.float32)
    grid = base.view(1, h * w, 3).bmm(rescaled).view(1, h, w, 2)
    return F.grid_sample(img[None], grid, mode="nearest", padding_mode="zeros", align_corners=False)[0]


def _blend(img1: torch.Tensor, img2, ratio: float) -> torch.Tensor:
    return (ratio * img1 + (1.0 - ratio) * img2).clamp(0, 1.0)


def adjust_brightness(img: torch.Tensor, f: float) -> torch.Tensor:
    return _blend(img, torch.zeros_like(img), f)


def adjust_contrast(img: torch.Tensor, f: float) -> torch.Tensor:
    if img.shape[0] == 3:
        gray = (0.2989 * img[0] + 0.587 * img[1] + 0.114 * img[2]).to(img.dtype).unsqueeze(0)
        mean = torch.mean(gray, dim=(-3, -2, -1), keepdim=True)
    else:
        mean = torch.mean(img, dim=(-3, -2, -1), keepdim=True)
    return _blend(img, mean, f)


def transform(image: torch.Tensor, aug: Optional[Tuple[bool, float, float, float, bool]]) -> torch.Tensor:
    """aug = (flip, angle_deg, brightness, contrast, brightness_first) or None (evaluation)."""
    if aug is not None:
        flip, angle, bright, contrast, bright_first = aug
        if flip:
            image = image.flip(-1)
        image = rotate_nearest(image, angle)
        for fn in ((0, 1) if bright_first else (1, 0)):
            image = adjust_brightness(image, bright) if fn == 0 else adjust_contrast(image, contrast)
    c = image.shape[0]
    mean = torch.tensor([0.5] * c).view(c, 1, 1)
    std = torch.tensor([0.5] * c).view(c, 1, 1)
    return image.sub(mean).div(std)


def sample(img: np.ndarray, name: str, aug=None) -> torch.Tensor:
    return transform(convert_channels(to_tensor(img), 1 if name in GRAY else 3), aug)


def collate(images: Sequence[torch.Tensor]) -> torch.Tensor:
    """mixed_modality_collate_fn's image part: zero-pad channels to the batch maximum."""
    cmax = max(i.shape[0] for i in images)
    out = []
    for i in images:
        if i.shape[0] < cmax:
            i = torch.cat([i, torch.zeros((cmax - i.shape[0], *i.shape[1:]), dtype=i.dtype)], 0)
        out.append(i)
    return torch.stack(out)
