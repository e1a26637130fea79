#!/usr/bin/env python3
"""Diagnostic for the fused single-tile attention (csrc/attn.hip): with V = identity (n = C = 64) the forward output is
P itself; prints where O deviates from float64 softmax (by row / column block) in each GEMM arithmetic."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from medvae_disentangled_multimodal_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for prec in ("32", "32-exact", "bf16-mixed"):
    for n in (64, 49, 17):
        g = torch.Generator().manual_seed(n)
        b, c = 2, 64
        q = torch.randn(b, n, c, generator=g)
        k = torch.randn(b, n, c, generator=g)
        v = torch.zeros(b, n, c)
        for j in range(n):
            v[:, j, j] = 1.0
        s = torch.bmm(q.double(), k.double().transpose(1, 2)) * c ** -0.5
        p = torch.softmax(s, 2)
        o_ref = torch.zeros(b, n, c, dtype=torch.float64)
        o_ref[:, :, :n] = p
        qd, kd, vd = (t.to(dev).contiguous() for t in (q, k, v))
        o = torch.empty_like(qd)
        lse = torch.empty(b, 64, device=dev)
        prev = ops.set_precision(prec)
        try:
            ops._lib.call("mvae_attention_small_fwd", qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), o.data_ptr(),
                          lse.data_ptr(), b, n, c, c ** -0.5, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            ops.restore_math_mode(prev)
        d = (o.double().cpu() - o_ref).abs()
        lse_ref = torch.logsumexp(s, 2)
        print(prec, n, "max err", float(d.max()), "nan", bool(torch.isnan(o).any()),
              "rows<32", float(d[:, :32].max()), "rows>=32", float(d[:, 32:].max()) if n > 32 else None,
              "cols<32", float(d[:, :, :32].max()), "cols>=32", float(d[:, :, 32:].max()),
              "lse err", float((lse[:, :n].double().cpu() - lse_ref).abs().max()), flush=True)
        if float(d.max()) > 1e-3:
            i = int(d.flatten().argmax())
            bb, rr, cc = i // (n * c), (i // c) % n, i % c
            print("   worst at b", bb, "row", rr, "col", cc, "got", float(o[bb, rr, cc]), "ref", float(o_ref[bb, rr, cc]))
