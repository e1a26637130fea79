#!/usr/bin/env python3
"""Stress: resident GroupNorm backward with the residual-branch gradient vs the streaming path, N repetitions."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from test_gpu_kernels import _gn_raw, rel
dev = torch.device("cuda:0")
bad = {}
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    for (n, c, h, add) in [(2, 2048, 4, True), (2, 1024, 4, True), (3, 32, 28, True), (2, 2048, 4, False)]:
        g = torch.Generator().manual_seed(rep * 131 + c + h)
        G = min(32, c)
        x = (torch.randn(n, h, h, c, generator=g) * 1.5 + 0.3).to(dev)
        gamma = (1 + 0.2 * torch.randn(c, generator=g)).to(dev)
        beta = (0.1 * torch.randn(c, generator=g)).to(dev)
        dy = torch.randn(n, h, h, c, generator=g).to(dev)
        ad = torch.randn(n, h, h, c, generator=g).to(dev) if add else None
        r1 = _gn_raw(1, x, gamma, beta, dy, ad, G, True, 0.0, 77)[3]
        r0 = _gn_raw(0, x, gamma, beta, dy, ad, G, True, 0.0, 77)[3]
        if rel(r0, r1) > 1e-5:
            bad[(n, c, h, add)] = bad.get((n, c, h, add), 0) + 1
print(os.environ.get("MVAE_HIP_LIB", "default"), "failures:", bad, flush=True)
