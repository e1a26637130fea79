"""Learning-rate schedulers (names/defaults as of the reference (src/utils/training_utils.py:12-57), stepped per epoch."""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch


def get_scheduler(optimizer: torch.optim.Optimizer, config: Dict[str, Any]) -> Optional[Any]:
    t = (config or {}).get("type", "none")
    if t in ("none", None):
        return None
    S = torch.optim.lr_scheduler
    if t == "step":
        return S.StepLR(optimizer, step_size=config.get("step_size", 30), gamma=config.get("gamma", 0.1))
    if t == "multistep":
        return S.MultiStepLR(optimizer, milestones=config.get("milestones", [50, 100]),
                             gamma=config.get("gamma", 0.1))
    if t == "exponential":
        return S.ExponentialLR(optimizer, gamma=config.get("gamma", 0.95))
    if t == "cosine":
        return S.CosineAnnealingLR(optimizer, T_max=config.get("T_max", 100), eta_min=config.get("eta_min", 0))
    if t == "reduce_on_plateau":
        return S.ReduceLROnPlateau(optimizer, mode=config.get("mode", "min"), factor=config.get("factor", 0.5),
                                   patience=config.get("patience", 10), threshold=config.get("threshold", 1e-4))
    raise ValueError(f"Unknown scheduler type: {t}")
