#!/usr/bin/env python3
"""Which part of a training step breaks HIP-graph capture: tools/graph_bisect.py <variant>
variants: cvae_fwd, cvae_fwdbwd, cvae_step, dis_fwd, dis_fwdbwd, dis_step"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import faulthandler; faulthandler.enable()
import torch
import medvae_disentangled_multimodal_amd as M
from medvae_disentangled_multimodal_amd import ops
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_graph import CASES, _batch, _module

v = sys.argv[1]
dev = torch.device("cuda:0")
cls, kw, loss = CASES[0] if v.startswith("dis") else CASES[1]
mod = _module(cls, kw, loss, dev)
batch = _batch(cls, dev)
mod.fit_step(batch, 0)
torch.cuda.synchronize()
static = [t.clone() for t in batch]
g = torch.cuda.CUDAGraph()
part = v.split("_")[1]
with torch.cuda.graph(g):
    if part == "step":
        out = mod.fit_step(static, 1)
    else:
        mod.optimizer.zero_grad()
        l = mod.training_step(static, 1)
        if part == "fwdbwd":
            l.backward()
print(v, "captured", flush=True)
g.replay()
torch.cuda.synchronize()
print(v, "replayed ok", flush=True)
