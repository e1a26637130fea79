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
    the flat gradient buffer every step.

    Overlap: the flat buffer is cut into buckets of whole parameters in REVERSE registration order
    (the order backward produces gradients: decoder first). Every op reports each parameter whose
    flat-slot gradient it has finished (ops.GRAD_HOOK; autograd-accumulated parameters through a
    post-accumulate hook), and a bucket's all-reduce is launched asynchronously (RCCL runs it on its
    own stream, ordered after the kernels that wrote the bucket) as soon as its last parameter
    reports -- so the collective of the decoder's gradients runs while the encoder's backward is
    still computing. Buckets are launched strictly in bucket order (a ready bucket waits for its
    predecessors), so every rank issues the same sequence of collectives even when ranks use
    different parameters (the disentangled model's per-modality heads). `allreduce_gradients`
    launches whatever never reported (parameters unused this step) and makes the compute stream
    wait for all collectives before the optimizer."""

    def __init__(self, module, group=None, bucket_bytes: int = BUCKET_BYTES, overlap: bool = True):
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_elems = max(1, bucket_bytes // 4)
        if module.flat is None:
            module.configure_optimizers()
        flat = module.flat
        if self.world > 1:
            dist.broadcast(flat.data, src=0, group=group)
            if getattr(module, "flat_d", None) is not None:  # discriminator of the adversarial branch
                dist.broadcast(module.flat_d.data, src=0, group=group)
        module.optimizer.grad_scale = 1.0 / self.world
        if getattr(module, "optimizer_d", None) is not None:
            module.optimizer_d.grad_scale = 1.0 / self.world
        module.process_group = self
        self.overlap = overlap and self.world > 1
        self._plan(flat)
        self._works = []
        self._armed = False
        if self.overlap:
            from . import ops
            ops.GRAD_HOOK = self._on_grad

    def _plan(self, flat):
        """Buckets of whole parameters, reverse order, each >= bucket_elems (the last may be smaller)."""
        self.buckets = []  # (start, end) element ranges of flat.grad
        self.param_bucket = {}
        members, lo, hi = [], None, None
        for i in reversed(range(len(flat.params))):
            p, off = flat.params[i], flat.offsets[i]
            end = off + (p.numel() + 3) // 4 * 4 if i < len(flat.params) - 1 else flat.numel  # (+ the tail padding)
            members.append(i)
            lo = off
            hi = end if hi is None else hi
            if hi - lo >= self.bucket_elems:
                self._close(members, lo, hi)
                members, lo, hi = [], None, None
        if members:
            self._close(members, 0 if lo is None else lo, hi)
        self.expected = [0] * len(self.buckets)
        for b in self.param_bucket.values():
            self.expected[b] += 1

    def _close(self, members, lo, hi):
        b = len(self.buckets)
        self.buckets.append((lo, hi))
        for i in members:
            self.param_bucket[id(self.module.flat.params[i])] = b

    def begin_backward(self):
        """Arm the per-step readiness counters (call before loss.backward())."""
        self.pending = list(self.expected)
        self.launched = [False] * len(self.buckets)
        self.next_bucket = 0
        self.seen = set()
        self._works = []
        self._armed = True

    def _on_grad(self, p):
        if not self._armed:
            return
        key = id(p)
        b = self.param_bucket.get(key)
        if b is None or key in self.seen:
            return
        self.seen.add(key)
        self.pending[b] -= 1
        while self.next_bucket < len(self.buckets) and self.pending[self.next_bucket] == 0:
            self._launch(self.next_bucket)
            self.next_bucket += 1

    def _launch(self, b):
        lo, hi = self.buckets[b]
        self.launched[b] = True
        g = self.module.flat.grad[lo:hi]
        self._works.append(dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def backend(self) -> Optional[str]:
        """the process group's backend ("nccl" = RCCL on ROCm, "gloo"); None without a process group."""
        return dist.get_backend(self.group) if dist.is_initialized() else None

    def any_across_ranks(self, flags: torch.Tensor) -> torch.Tensor:
        """Element-wise OR of a small bool vector over all ranks (same call order on every rank)."""
        if self.world == 1:
            return flags
        v = flags.to(torch.int32)
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=self.group)
        return v > 0

    def allreduce_flat(self, flat):
        """Synchronous bucketed all-reduce of another flat gradient buffer (the discriminator's)."""
        if self.world == 1:
            return
        g = flat.grad
        for s in range(0, g.numel(), self.bucket_elems):
            dist.all_reduce(g[s:s + self.bucket_elems], op=dist.ReduceOp.SUM, group=self.group)

    def allreduce_gradients(self, flat):
        if self.world == 1:
            return
        if not self.overlap or not self._armed:
            g = flat.grad
            n = g.numel()
            for s in range(0, n, self.bucket_elems):
                dist.all_reduce(g[s:s + self.bucket_elems], op=dist.ReduceOp.SUM, group=self.group)
            return
        for b in range(self.next_bucket, len(self.buckets)):  # incl. parameters that produced no gradient
            self._launch(b)
        self.next_bucket = len(self.buckets)
        for w in self._works:
            w.wait()
        self._works = []
        self._armed = False
