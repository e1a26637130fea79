#!/usr/bin/env python3
"""Time the GroupNorm fwd / bwd C-ABI calls on the c2 / c3 level shapes (HIP events), per path.
usage: tools/gn_bench.py [reps]   (env knobs of norm.hip apply: MVAE_GN_RES_GRID ...)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import _lib
dev = torch.device("cuda:0")
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
SHAPES = [(512, 32, 28, True), (512, 64, 14, True), (512, 128, 7, True), (256, 128, 28, True), (256, 256, 14, False),
          (256, 512, 7, True)]
if os.environ.get("GN_BENCH_C4"):
    SHAPES = [(256, 2048, 8, True), (256, 1024, 16, True), (256, 512, 32, True), (256, 256, 64, True),
              (256, 256, 64, False), (256, 512, 64, False)]
st = torch.cuda.current_stream().cuda_stream
tot = {0: [0.0, 0.0], 1: [0.0, 0.0]}
for n, c, h, add in SHAPES:
    G = 32
    x = torch.randn(n, h, h, c, device=dev)
    dy = torch.randn_like(x)
    ad = torch.randn_like(x) if add else None
    gamma = torch.ones(c, device=dev); beta = torch.zeros(c, device=dev)
    y = torch.empty_like(x); dx = torch.empty_like(x)
    mean = torch.empty(n * G, device=dev); rstd = torch.empty_like(mean)
    dg = torch.zeros(c, device=dev); db = torch.zeros(c, device=dev)
    ws = torch.empty(_lib.query("mvae_group_norm_workspace_bytes", n, h * h, c), dtype=torch.uint8, device=dev)
    row = []
    for path in (1, 0):
        _lib.call("mvae_set_group_norm_path", path)
        def fwd():
            _lib.call("mvae_group_norm_fwd_nhwc", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                      mean.data_ptr(), rstd.data_ptr(), n, h * h, c, G, 1e-6, 1, 0.0, 0, 1, ws.data_ptr(), ws.numel(), st)
        def bwd():
            _lib.call("mvae_group_norm_bwd_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                      mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), ad.data_ptr() if add else None, dg.data_ptr(),
                      db.data_ptr(), n, h * h, c, G, 1, 0.0, 0, ws.data_ptr(), ws.numel(), st)
        for fn, k in ((fwd, 0), (bwd, 1)):
            fn(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REPS):
                fn()
            e1.record(); torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / REPS
            nbytes = x.numel() * 4 * (2 if k == 0 else (4 if add else 3))
            row.append(f"{'SR'[path == 0]}{'fb'[k]} {us:7.1f}us {nbytes / us / 1e6:5.2f}TB/s")
            tot[path][k] += us
    _lib.call("mvae_set_group_norm_path", 0)
    print((n, c, h, add), " | ".join(row), flush=True)
print(os.environ.get("MVAE_GN_RES_GRID", "-"), os.environ.get("MVAE_GN_RES_FWD_IT", "-"), "total us: streaming fwd %.0f bwd %.0f | resident fwd %.0f bwd %.0f" % (
    tot[1][0], tot[1][1], tot[0][0], tot[0][1]))
