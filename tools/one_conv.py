#!/usr/bin/env python3
"""Run one conv pass (fwd/dgrad/wgrad) of one cfg-4 layer shape repeatedly (profiling target)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import ops
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import SHAPES

ap = argparse.ArgumentParser()
ap.add_argument("--shape", type=int, default=1)
ap.add_argument("--pass_", default="fwd")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--precision", default="32")
a = ap.parse_args()
ops.set_precision(a.precision)
n, ci, co, h, k, s, pads, ups = SHAPES[a.shape]
dev = torch.device("cuda:0")
g = ops.ConvGeom(k, k, s, pads[0], pads[1], pads[2], pads[3], ups)
x = torch.randn(n, ci, h, h, device=dev).contiguous(memory_format=torch.channels_last)
w = (torch.randn(co, ci, k, k, device=dev) * 0.02).contiguous(memory_format=torch.channels_last)
b = torch.zeros(co, device=dev)
ho, wo = g.out_hw(h, h)
dy = torch.randn(n, co, ho, wo, device=dev).contiguous(memory_format=torch.channels_last)
dw = torch.zeros_like(w)
for _ in range(a.reps):
    if a.pass_ == "fwd":
        ops.conv2d_forward_raw(x, w, b, None, g)
    elif a.pass_ == "dgrad":
        ops.conv2d_dgrad_raw(dy, w, x.shape, g)
    else:
        ops.conv2d_wgrad_raw(dy, x, dw, 0.0, g)
torch.cuda.synchronize()
