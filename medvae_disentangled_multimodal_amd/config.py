"""Hydra-style `_target_` instantiation without Hydra (not installed on the MI355X image).

The reference builds its model with `hydra.utils.instantiate(cfg.model)` (main.py:29) from YAML
files such as configs/model/base_vae.yaml whose `_target_` is `src.models.BaseVAE`. This loader reads
the same YAML (yaml.SafeLoader, no code execution), maps the reference's `src.models.*` /
`src.losses.*` targets onto this package (the drop-in swap), and calls the class with the remaining
keys as kwargs. `defaults:` lists and `# @package _global_` overlays are flattened by the caller via
`merge`.
"""
from __future__ import annotations

import copy
import importlib
from typing import Any, Dict, Optional

import yaml

_PKG = "medvae_disentangled_multimodal_amd"
TARGET_MAP = {
    "src.models.BaseVAE": f"{_PKG}.BaseVAE",
    "src.models.BetaVAE": f"{_PKG}.BetaVAE",
    "src.models.ConditionalVAE": f"{_PKG}.ConditionalVAE",
    "src.models.DisentangledConditionalVAE": f"{_PKG}.DisentangledConditionalVAE",
    "src.models.DisentangledVAELoss": f"{_PKG}.DisentangledVAELoss",
    "src.models.Encoder": f"{_PKG}.Encoder",
    "src.models.Decoder": f"{_PKG}.Decoder",
    "src.losses.VAELoss": f"{_PKG}.VAELoss",
    "src.losses.LPIPSLoss": f"{_PKG}.LPIPSLoss",
    "src.losses.LPIPSWithDiscriminator": f"{_PKG}.LPIPSWithDiscriminator",
}


def load_yaml(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.load(f, Loader=yaml.SafeLoader) or {}


def merge(base: Dict[str, Any], over: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def resolve_target(target: str):
    target = TARGET_MAP.get(target, target)
    mod, _, name = target.rpartition(".")
    return getattr(importlib.import_module(mod), name)


def instantiate(cfg: Dict[str, Any], **overrides):
    """Build `cfg['_target_'](**rest)`; nested dicts with a `_target_` are instantiated first."""
    cfg = merge(cfg, overrides)
    target = cfg.pop("_target_")
    kwargs = {k: (instantiate(v) if isinstance(v, dict) and "_target_" in v else v)
              for k, v in cfg.items() if k != "defaults"}
    if "ch_mult" in kwargs and isinstance(kwargs["ch_mult"], list):
        kwargs["ch_mult"] = tuple(kwargs["ch_mult"])
    return resolve_target(target)(**kwargs)
