"""Lightning-checkpoint interchange (main.py:51-61,110-116: ModelCheckpoint / trainer.save_checkpoint;
quick_generate.py:37-42: loading `model.`-prefixed weights).

A checkpoint written here has the layout Lightning 2.5 writes for the reference's VAELightningModule
-- `state_dict` with `model.`-prefixed parameter names (logical OIHW conv weights),
`optimizer_states` in torch.optim.Adam/AdamW's own `state_dict()` format over `model.parameters()`
order, `epoch`, `global_step`, `lr_schedulers` -- so the reference can resume from it, and a
reference checkpoint loads here (weights and Adam moments land in the flat buffers).
Loading uses `torch.load(weights_only=True)`: nothing in the file is executed; a checkpoint that
needs arbitrary unpickling is refused.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Dict

import torch

from .optim import FlatParameters

LIGHTNING_VERSION = "2.5.2"  # the reference's pin (uv.lock)


def _torch_optimizer_state(opt, flat) -> Dict[str, Any]:
    state = {}
    steps = opt.steps.cpu()
    for i, (p, off) in enumerate(zip(flat.params, flat.offsets)):
        if int(steps[i]) == 0:
            continue
        state[i] = {"step": torch.tensor(float(steps[i])),
                    "exp_avg": FlatParameters._view(opt.exp_avg, off, p).detach().contiguous().cpu(),
                    "exp_avg_sq": FlatParameters._view(opt.exp_avg_sq, off, p).detach().contiguous().cpu()}
    g = opt.param_groups[0]
    group = {"lr": g["lr"], "betas": tuple(g["betas"]), "eps": g["eps"], "weight_decay": g["weight_decay"],
             "amsgrad": False, "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
             "fused": None, "params": list(range(len(flat.params)))}
    if opt.decoupled:
        group["decoupled_weight_decay"] = True
    return {"state": state, "param_groups": [group]}


def lightning_checkpoint(module, epoch: int = 0) -> Dict[str, Any]:
    """The dict `trainer.save_checkpoint` would write for this module: the LightningModule's own state dict
    (`model.*` and the criterion's `criterion.*` -- LPIPS network, discriminator weights and BatchNorm
    buffers), one optimizer state per optimizer (the discriminator's Adam second, lightning_module.py:
    427-433)."""
    sd = OrderedDict((f"model.{k}", v.detach().contiguous().cpu()) for k, v in module.model.state_dict().items())
    crit = getattr(module, "criterion", None)
    if isinstance(crit, torch.nn.Module):
        sd.update((f"criterion.{k}", v.detach().contiguous().cpu()) for k, v in crit.state_dict().items())
    ck = {"epoch": int(epoch), "global_step": int(getattr(module, "global_step_count", 0)),
          "pytorch-lightning_version": LIGHTNING_VERSION, "state_dict": sd, "loops": {}, "callbacks": {},
          "lr_schedulers": [], "optimizer_states": []}
    if module.optimizer is not None:
        ck["optimizer_states"] = [_torch_optimizer_state(module.optimizer, module.flat)]
        if getattr(module, "optimizer_d", None) is not None:
            ck["optimizer_states"].append(_torch_optimizer_state(module.optimizer_d, module.flat_d))
        if module.scheduler is not None and hasattr(module.scheduler, "state_dict"):
            ck["lr_schedulers"] = [module.scheduler.state_dict()]
    return ck


def save_checkpoint(module, path: str, epoch: int = 0):
    torch.save(lightning_checkpoint(module, epoch), path)


def load_checkpoint(module, ckpt, strict: bool = True, load_optimizer: bool = True):
    """Load a Lightning checkpoint (path or dict) of the reference's VAELightningModule (or of this
    one) into `module`: model weights (into the flat parameter buffer) and, when present and an
    optimizer is configured, the Adam/AdamW moments and step counts."""
    if isinstance(ckpt, str):
        ckpt = torch.load(ckpt, map_location="cpu", weights_only=True)
    module._graph = None  # a captured step froze the old hyper-parameters (betas / eps / lr) as launch values
    sd = {k[len("model."):]: v for k, v in ckpt["state_dict"].items() if k.startswith("model.")}
    module.model.load_state_dict(sd, strict=strict)
    crit = getattr(module, "criterion", None)
    csd = {k[len("criterion."):]: v for k, v in ckpt["state_dict"].items() if k.startswith("criterion.")}
    if isinstance(crit, torch.nn.Module) and (csd or (strict and len(crit.state_dict()) > 0)):
        crit.load_state_dict(csd, strict=strict)
    states = ckpt.get("optimizer_states") or []
    if load_optimizer and states:
        if module.optimizer is None:
            module.configure_optimizers()
        _load_optimizer_state(module.optimizer, module.flat, states[0])
        if len(states) > 1 and getattr(module, "optimizer_d", None) is not None:
            _load_optimizer_state(module.optimizer_d, module.flat_d, states[1])
    module.global_step_count = int(ckpt.get("global_step", 0))
    return ckpt


def _load_optimizer_state(opt, flat, st):
    steps = torch.zeros(len(flat.params), dtype=torch.int32)
    with torch.no_grad():
        for i, (p, off) in enumerate(zip(flat.params, flat.offsets)):
            s = st["state"].get(i, st["state"].get(str(i)))
            if s is None:
                FlatParameters._view(opt.exp_avg, off, p).zero_()
                FlatParameters._view(opt.exp_avg_sq, off, p).zero_()
                continue
            FlatParameters._view(opt.exp_avg, off, p).copy_(s["exp_avg"])
            FlatParameters._view(opt.exp_avg_sq, off, p).copy_(s["exp_avg_sq"])
            steps[i] = int(float(s["step"]))
    opt.steps.copy_(steps)
    g = st["param_groups"][0]
    for k in ("lr", "betas", "eps", "weight_decay"):
        if k in g:
            opt.param_groups[0][k] = tuple(g[k]) if k == "betas" else g[k]
