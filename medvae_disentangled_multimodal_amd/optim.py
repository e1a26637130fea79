"""Flat parameter / gradient storage and the fused Adam/AdamW step.

`FlatParameters` re-homes every parameter of a module into ONE contiguous fp32 buffer (4-D conv
weights keep channels_last = KRSC strides) and gives each parameter a gradient view into ONE flat
gradient buffer. The HIP ops accumulate weight gradients straight into those views, the data-parallel
all-reduce is a single collective over the flat gradient buffer, and the optimizer is one fused
multi-tensor kernel (non-finite zeroing, global-norm clip, Adam/AdamW).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional

import torch

from . import _lib
from .ops import ARENA

CHUNK = 65536
ALIGN = 4  # floats (16 bytes): every tensor starts 16B-aligned for float4 loads


def _after_autograd_accumulate(p: torch.Tensor):
    """Parameters whose gradient autograd accumulates (torch glue ops): keep the result in the flat
    slot even if autograd swapped in a new .grad tensor, then report the gradient as complete."""
    mg = p._mvae_main_grad
    if p.grad is not None and p.grad.data_ptr() != mg.data_ptr():
        mg.copy_(p.grad)
        p.grad = mg
    from . import ops
    ops._grad_done(p)


class FlatParameters:
    def __init__(self, module: torch.nn.Module, device=None):
        self.module = module
        named = [(n, p) for n, p in module.named_parameters()]
        if device is None:
            device = named[0][1].device
        self.device = torch.device(device)
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offs
        # whole 8-element groups: the one-launch weight conversions of a step (ops.prep_flat_weights: split4 / packed
        # bf16) take the buffer in 16-B output groups of 8 fp32 elements; the padding stays zero
        o = (o + 7) // 8 * 8
        self.numel = o
        self.data = torch.zeros(o, device=self.device, dtype=torch.float32)
        self.grad = torch.zeros(o, device=self.device, dtype=torch.float32)
        for p, off in zip(self.params, offs):
            dv = self._view(self.data, off, p)
            dv.copy_(p.detach().to(self.device, torch.float32))
            p.data = dv
            gv = self._view(self.grad, off, p)
            p._mvae_main_grad = gv
            p.grad = gv
            if p.requires_grad:
                p.register_post_accumulate_grad_hook(_after_autograd_accumulate)
        # chunk table for the multi-tensor kernels
        ct, cs, cl, tcb = [], [], [], [0]
        for t, (p, off) in enumerate(zip(self.params, offs)):
            n = p.numel()
            for s in range(0, n, CHUNK):
                ct.append(t)
                cs.append(off + s)
                cl.append(min(CHUNK, n - s))
            tcb.append(len(ct))
        dev = self.device
        self.chunk_tensor = torch.tensor(ct, dtype=torch.int32, device=dev)
        self.chunk_start = torch.tensor(cs, dtype=torch.int64, device=dev)
        self.chunk_len = torch.tensor(cl, dtype=torch.int32, device=dev)
        self.tensor_chunk_begin = torch.tensor(tcb, dtype=torch.int32, device=dev)
        self.nchunks = len(ct)
        self.used = torch.ones(len(self.params), dtype=torch.int32, device=dev)

    @staticmethod
    def _view(buf: torch.Tensor, off: int, p: torch.Tensor) -> torch.Tensor:
        n = p.numel()
        flat = buf[off:off + n]
        if p.dim() == 4:
            o, i, kh, kw = p.shape
            return flat.view(o, kh, kw, i).permute(0, 3, 1, 2)  # logical OIHW, physical OHWI (KRSC)
        return flat.view(p.shape)

    def zero_grad(self):
        self.grad.zero_()
        for p in self.params:  # re-attach in case a caller set .grad = None
            if p.grad is None or p.grad.data_ptr() != p._mvae_main_grad.data_ptr():
                p.grad = p._mvae_main_grad

    def index_of(self, name: str) -> int:
        return self.names.index(name)


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam / AdamW semantics over a FlatParameters buffer in one fused kernel chain.
    `step()` also applies the LightningModule hooks that precede it in the reference:
    per-tensor non-finite zeroing (on_before_optimizer_step) and global-norm clipping."""

    def __init__(self, flat: FlatParameters, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 decoupled: bool = False, max_grad_norm: Optional[float] = None):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(flat.params, defaults)
        self.flat = flat
        self.decoupled = decoupled
        self.max_grad_norm = max_grad_norm
        dev = flat.device
        self.exp_avg = torch.zeros(flat.numel, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(flat.numel, device=dev, dtype=torch.float32)
        self.steps = torch.zeros(len(flat.params), dtype=torch.int32, device=dev)
        self.scalars = torch.zeros(2, device=dev, dtype=torch.float32)
        self.grad_scale = 1.0

    @property
    def last_total_norm(self) -> torch.Tensor:
        return self.scalars[0]

    def zero_grad(self, set_to_none: bool = True):
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, closure=None, used: Optional[torch.Tensor] = None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        f = self.flat
        used = f.used if used is None else used
        nbytes = _lib.query("mvae_multi_tensor_adam_workspace_bytes", f.nchunks, len(f.params))
        ws = ARENA.get("adam", nbytes, f.device)
        clip = self.max_grad_norm
        st = torch.cuda.current_stream(f.device).cuda_stream
        b1, b2 = g["betas"]
        _lib.call("mvae_multi_tensor_adam", f.data.data_ptr(), f.grad.data_ptr(), self.exp_avg.data_ptr(),
                  self.exp_avg_sq.data_ptr(), f.chunk_tensor.data_ptr(), f.chunk_start.data_ptr(),
                  f.chunk_len.data_ptr(), f.nchunks, f.tensor_chunk_begin.data_ptr(), len(f.params),
                  used.data_ptr(), self.steps.data_ptr(), float(self.grad_scale),
                  float(clip) if clip else 0.0, 1 if (clip is not None and clip > 0) else 0, float(g["lr"]),
                  float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), 1 if self.decoupled else 0,
                  ws.data_ptr(), ws.numel(), self.scalars.data_ptr(), st)
        return loss

    def state_dict(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "steps": self.steps,
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.steps.copy_(sd["steps"])
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)


def AdamW(flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_grad_norm=None):
    return FusedAdam(flat, lr, betas, eps, weight_decay, decoupled=True, max_grad_norm=max_grad_norm)


def Adam(flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None):
    return FusedAdam(flat, lr, betas, eps, weight_decay, decoupled=False, max_grad_norm=max_grad_norm)
