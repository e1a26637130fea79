#!/usr/bin/env python3
"""Golden vectors for the callers either side of the hot path -- the input pipeline (row f1) and the validation
metrics (row f3) -- from the REFERENCE's own pure-torch functions (build container only; /root/reference does not
exist on the GPU box).

    python3 -B tests/golden/make_ref_fixtures.py

src.data and src.utils cannot be imported here (they import lightning, medmnist, torchvision, sklearn and
torchmetrics, none installed). The functions below are pure torch, so this script parses the reference files with
`ast`, compiles only these definitions and runs them on synthetic MedMNIST-shaped inputs:
  * mixed_modality_collate_fn                        src/data/medmnist_data.py:16-72
  * MedMNISTDataset._create_modality_map,            src/data/medmnist_data.py:137-152
    _get_modality_channels, __getitem__              :154-181, :186-251 (channel conversion, label
                                                     standardisation, one-hot, modality index); `self` is a
                                                     stand-in object holding the attributes __init__ would set
                                                     (medmnist's INFO / download are not available). Images are
                                                     handed over as PIL-like uint8 images; transforms.ToTensor is
                                                     restated (uint8 / 255 -- torchvision is absent, so that one
                                                     step is unpinned), transform=None.
  * compute_kl_metrics, and the MSE / MAE half of    src/utils/metrics.py:14-73 (PSNR / SSIM come from
    compute_reconstruction_metrics                   torchmetrics, absent: unpinned; stubbed to NaN here)
Only data is written (tests/golden/ref_data.npz, ref_metrics.npz + .json metadata); no reference source is stored.
"""
from __future__ import annotations

import ast
import json
import os
import sys
import types
from typing import Any, Dict, List, Optional, Tuple

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("MEDVAE_REFERENCE", "/root/reference")


def _defs(path: str, names: List[str], cls: Optional[str] = None) -> Dict[str, ast.AST]:
    tree = ast.parse(open(path).read(), filename=path)
    body = tree.body
    if cls is not None:
        body = next(n for n in body if isinstance(n, ast.ClassDef) and n.name == cls).body
    found = {n.name: n for n in body if isinstance(n, ast.FunctionDef) and n.name in names}
    missing = set(names) - set(found)
    assert not missing, missing
    return found


def _compile(nodes: Dict[str, ast.AST], ns: dict, path: str) -> dict:
    for name, node in nodes.items():
        node = ast.fix_missing_locations(node)
        mod = ast.Module(body=[node], type_ignores=[])
        exec(compile(mod, path, "exec"), ns)
    return ns


class _PilLike:
    """What medmnist's dataset returns with transform=None: a PIL image (here: its uint8 array and a `mode`)."""

    def __init__(self, arr: np.ndarray):
        self.arr = arr
        self.mode = "L" if arr.ndim == 2 else "RGB"


class _ToTensor:
    """transforms.ToTensor restated (torchvision is absent -- this one step is unpinned): HxW[x3] uint8 ->
    [C,H,W] float32 / 255."""

    def __call__(self, pic):
        a = pic.arr.reshape(pic.arr.shape[0], pic.arr.shape[1], -1)
        return torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)


class _Transforms:
    ToTensor = _ToTensor

    def __getattr__(self, k):
        raise RuntimeError(f"torchvision.transforms.{k} is not available")


def reference_data_functions():
    path = os.path.join(REF, "src", "data", "medmnist_data.py")
    ns = {"torch": torch, "np": np, "transforms": _Transforms(), "Tuple": Tuple, "Dict": Dict, "Any": Any,
          "Optional": Optional, "List": List}
    _compile(_defs(path, ["mixed_modality_collate_fn"]), ns, path)
    meth = _compile(_defs(path, ["_create_modality_map", "_get_modality_channels", "__getitem__", "__len__"],
                          cls="MedMNISTDataset"), dict(ns), path)
    Dataset = type("RefMedMNISTDataset", (), {k: meth[k] for k in ("_create_modality_map", "_get_modality_channels",
                                                                    "__getitem__", "__len__")})
    return ns["mixed_modality_collate_fn"], Dataset


def reference_metric_functions():
    path = os.path.join(REF, "src", "utils", "metrics.py")
    nan = lambda *a, **k: torch.tensor(float("nan"))  # noqa: E731  (torchmetrics psnr / ssim: absent)
    ns = {"torch": torch, "F": F, "np": np, "Dict": Dict, "Tuple": Tuple, "Optional": Optional, "psnr": nan,
          "ssim": nan}
    _compile(_defs(path, ["compute_kl_metrics", "compute_reconstruction_metrics"]), ns, path)
    return ns["compute_kl_metrics"], ns["compute_reconstruction_metrics"]


def make_dataset(Dataset, name: str, images: List[torch.Tensor], labels: List[np.ndarray], natural_channels: int):
    ds = object.__new__(Dataset)
    ds.dataset_name = name
    ds.dataset = list(zip(images, labels))
    ds.transform = None
    ds.n_channels = natural_channels
    ds.modality_map = ds._create_modality_map()
    ds.modality_idx = ds.modality_map[name]
    ds.target_channels = ds._get_modality_channels()
    return ds


NAMES = ["chestmnist", "pathmnist", "octmnist", "pneumoniamnist", "dermamnist", "bloodmnist", "tissuemnist",
         "retinamnist", "breastmnist", "organamnist", "organcmnist", "organsmnist"]
# MedMNIST's stored layout per dataset: (natural channels, label width) -- chest is 14-way multi-label
LAYOUT = {"chestmnist": (1, 14), "pathmnist": (3, 1), "octmnist": (1, 1), "pneumoniamnist": (1, 1),
          "dermamnist": (3, 1), "bloodmnist": (3, 1), "tissuemnist": (1, 1), "retinamnist": (3, 1),
          "breastmnist": (1, 1), "organamnist": (1, 1), "organcmnist": (1, 1), "organsmnist": (3, 1)}  # organs stored RGB: exercises RGB -> gray


def data_fixture(size: int, rng: np.random.Generator):
    collate, Dataset = reference_data_functions()
    rec = {}
    items = []  # (name, item index) in fixture order
    for name in NAMES:
        ch, lw = LAYOUT[name]
        n = 3
        u8 = rng.integers(0, 256, size=(n, size, size) if ch == 1 else (n, size, size, 3), dtype=np.uint8)
        if lw > 1:
            lab = rng.integers(0, 2, size=(n, lw)).astype(np.int64)
            lab[1] = 0  # a multi-label row without positives -> label 0
        else:
            lab = rng.integers(0, 9, size=(n, 1)).astype(np.int64)
        imgs = [_PilLike(u8[k]) for k in range(n)]
        ds = make_dataset(Dataset, name, imgs, [lab[k] for k in range(n)], ch)
        rec[f"{name}.u8"] = u8
        rec[f"{name}.labels"] = lab
        for k in range(n):
            image, label, modality, midx = ds[k]
            rec[f"{name}.{k}.image"] = image.numpy()
            rec[f"{name}.{k}.label"] = label.numpy()
            rec[f"{name}.{k}.onehot"] = modality.numpy()
            rec[f"{name}.{k}.idx"] = np.array(int(midx))
            items.append((name, k, (image, label, modality, midx)))
    # collate: one mixed batch (gray + colour -> zero-padded), one all-gray batch (no padding)
    batches = {"mixed": [0, 4, 7, 12, 30, 3, 16], "gray": [0, 9, 27, 28, 33]}
    for bname, sel in batches.items():
        x, labels, onehot, midx = collate([items[i][2] for i in sel])
        rec[f"collate.{bname}.select"] = np.array(sel)
        rec[f"collate.{bname}.x"] = x.numpy()
        rec[f"collate.{bname}.labels"] = labels.numpy()
        rec[f"collate.{bname}.onehot"] = onehot.numpy()
        rec[f"collate.{bname}.idx"] = midx.numpy()
    rec["items"] = np.array([f"{n}:{k}" for n, k, _ in items])
    return rec


def metrics_fixture(rng: np.random.Generator):
    kl_fn, rec_fn = reference_metric_functions()
    rec = {}
    for tag, shape in (("flat", (6, 40)), ("spatial", (4, 16, 7, 7))):
        mean = torch.from_numpy(rng.standard_normal(shape).astype(np.float32))
        logvar = torch.from_numpy((0.5 * rng.standard_normal(shape)).astype(np.float32))
        m = kl_fn(mean, logvar)
        rec[f"kl.{tag}.mean"] = mean.numpy()
        rec[f"kl.{tag}.logvar"] = logvar.numpy()
        for k, v in m.items():
            rec[f"kl.{tag}.{k}"] = np.array(v)
    x = torch.from_numpy((rng.random((3, 3, 28, 28)) * 2 - 1).astype(np.float32))
    r = x + torch.from_numpy((0.1 * rng.standard_normal(x.shape)).astype(np.float32))
    m = rec_fn(x, r)
    rec["recon.x"], rec["recon.rec"] = x.numpy(), r.numpy()
    rec["recon.mse"], rec["recon.mae"] = np.array(m["mse"]), np.array(m["mae"])
    return rec


if __name__ == "__main__":
    torch.set_num_threads(8)
    rng = np.random.Generator(np.random.PCG64(31))
    data = {}
    for size in (28, 64):
        data.update({f"s{size}.{k}": v for k, v in data_fixture(size, rng).items()})
    np.savez(os.path.join(HERE, "ref_data.npz"), **data)
    np.savez(os.path.join(HERE, "ref_metrics.npz"), **metrics_fixture(rng))
    meta = {"reference": "parsakzr/medvae-disentangled-multimodal @ 2025-08-24", "torch": torch.__version__,
            "functions": ["src/data/medmnist_data.py:mixed_modality_collate_fn",
                          "src/data/medmnist_data.py:MedMNISTDataset.__getitem__ (+ _create_modality_map, "
                          "_get_modality_channels)",
                          "src/utils/metrics.py:compute_kl_metrics",
                          "src/utils/metrics.py:compute_reconstruction_metrics (mse, mae)"],
            "unpinned": ["transforms.ToTensor (torchvision absent: restated as uint8 / 255)",
                         "transforms.Normalize / RandomHorizontalFlip / RandomRotation / ColorJitter (torchvision)",
                         "psnr / ssim (torchmetrics absent)"]}
    with open(os.path.join(HERE, "ref_fixtures.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote ref_data.npz", len(data), "arrays; ref_metrics.npz")
