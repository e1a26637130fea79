#!/usr/bin/env python3
"""Wave-quantization probe: time one conv pass of a layer shape at several batch sizes (HIP events). A launch whose tile
count is just past a multiple of the resident slots (256 CUs x tiles per CU) pays a nearly empty last round.
usage: tools/quant_probe.py cin cout h [batches...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import ops

dev = torch.device("cuda:0")
ops.set_precision("32")
ci, co, h = (int(v) for v in sys.argv[1:4])
batches = [int(v) for v in sys.argv[4:]] or [256, 250, 240, 192, 128]
g = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
for n in batches:
    x = torch.randn(n, ci, h, h, device=dev).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, 3, 3, device=dev) * 0.02).contiguous(memory_format=torch.channels_last)
    b = torch.zeros(co, device=dev)
    dy = torch.randn(n, co, h, h, device=dev).contiguous(memory_format=torch.channels_last)
    dw = torch.zeros_like(w)
    row = []
    for name, fn in (("fwd", lambda: ops.conv2d_forward_raw(x, w, b, None, g)),
                     ("dgrad", lambda: ops.conv2d_dgrad_raw(dy, w, x.shape, g)),
                     ("wgrad", lambda: ops.conv2d_wgrad_raw(dy, x, dw, 0.0, g))):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 50
        row.append(f"{name} {us:7.1f}us {us / n:6.3f}us/img")
    print(n, " | ".join(row), flush=True)
