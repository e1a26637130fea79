#!/usr/bin/env python3
"""Time the conv weight-gradient GEMM (+ its split-K reduce and bias reduce) on c2 / c3 / c4 layer shapes.
usage: tools/wgrad_bench.py [reps]   (A/B: MVAE_SPLIT_LEGACY=1 in a second process)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import ops
dev = torch.device("cuda:0")
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
SHAPES = [  # n, cin, cout, h, k
    (512, 32, 32, 28, 3), (512, 64, 64, 14, 3), (512, 128, 128, 7, 3), (512, 128, 128, 7, 1), (512, 64, 32, 28, 3),
    (512, 32, 64, 14, 3), (512, 64, 32, 14, 3),
    (256, 128, 128, 28, 3), (256, 256, 256, 14, 3), (256, 512, 512, 7, 3),
    (256, 2048, 2048, 8, 3), (256, 256, 256, 64, 3),
]
tot = 0.0
for n, ci, co, h, k in SHAPES:
    p = (k - 1) // 2
    g = ops.ConvGeom(k, k, 1, p, p, p, p)
    x = torch.randn(n, ci, h, h, device=dev).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, co, h, h, device=dev).contiguous(memory_format=torch.channels_last)
    dw = torch.zeros(co, ci, k, k, device=dev).contiguous(memory_format=torch.channels_last)
    db = torch.zeros(co, device=dev)
    fn = lambda: ops.conv2d_wgrad_raw(dy, x, dw, 0.0, g, db=db)
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / REPS
    tot += us
    fl = 2.0 * n * h * h * co * ci * k * k
    print(f"{(n, ci, co, h, k)}  {us:8.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
print("legacy" if os.environ.get("MVAE_SPLIT_LEGACY") else "new", f"total {tot:.0f} us")
