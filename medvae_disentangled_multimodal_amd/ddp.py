"""Data-parallel training: one process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm)
or gloo (CPU tests).

The reference reaches DP only through Lightning's DDP strategy (devices > 1; configs/config.yaml:22
pins 1). Every op of the VAE is per-sample (GroupNorm, no BatchNorm, attention within an image), so the
only exchange per step is the gradient average. Because all gradients live in ONE flat buffer
(optim.FlatParameters), that exchange is one all-reduce (bucketed into a few large slices so RCCL can
pipeline them over the xGMI links) instead of hundreds of per-parameter collectives; the 1/world
average is folded into the fused optimizer kernel (grad_scale) instead of a separate pass.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

BUCKET_BYTES = 256 << 20  # 256 MiB slices: large enough to saturate xGMI rings, few enough launches


def init_from_env(backend: Optional[str] = None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    if dist.is_available() and not dist.is_initialized() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_initialized() else 1
    local = int(os.environ.get("LOCAL_RANK", rank))
    return rank, world, local


class DataParallel:
    """Attach to a VAELightningModule: broadcasts the initial parameters from rank 0 and averages
    the flat gradient buffer after every backward."""

    def __init__(self, module, group=None, bucket_bytes: int = BUCKET_BYTES):
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_elems = max(1, bucket_bytes // 4)
        if module.flat is None:
            module.configure_optimizers()
        if self.world > 1:
            dist.broadcast(module.flat.data, src=0, group=group)
        module.optimizer.grad_scale = 1.0 / self.world
        module.process_group = self

    def allreduce_gradients(self, flat):
        if self.world == 1:
            return
        g = flat.grad
        n = g.numel()
        for s in range(0, n, self.bucket_elems):
            dist.all_reduce(g[s:s + self.bucket_elems], op=dist.ReduceOp.SUM, group=self.group)
