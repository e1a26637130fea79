#!/usr/bin/env python3
"""Attention core timing at the configs' geometries (c4 / c5 16x16x1024 and mid blocks 8x8x2048, c2 7x7x512, c3
7x7x128): the fused single-tile kernels (csrc/attn.hip, n <= 64), the query-block fused kernels (csrc/attn_tile.hip,
64 <= n <= 256) and the unfused path (batched GEMMs around the row softmax), forward and backward, HIP events on the
launch stream. tools/attn_bench.py [precision]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from medvae_disentangled_multimodal_amd import ops  # noqa: E402

SHAPES = [("c4_16x16x1024", 256, 1024, 16), ("c4_8x8x2048", 256, 2048, 8), ("c2_7x7x512", 256, 512, 7),
          ("c3_7x7x128", 512, 128, 7)]
VARIANTS = {"small": (True, False), "tile": (False, True), "unfused": (False, False)}  # (ATTN_FUSED, ATTN_TILE)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "32"
    ops.set_precision(prec)
    dev = torch.device("cuda:0")
    out = {}
    for lab, b, c, h in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        q, k, v, go = (torch.randn(b, c, h, h, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
                       for _ in range(4))
        n = h * h
        fl_f, fl_b = 4.0 * n * n * c * b, 8.0 * n * n * c * b
        row = {}
        ops.ATTN_FUSED_MAXC = 1 << 30
        for name, (fused, tile) in VARIANTS.items():
            ops.ATTN_FUSED, ops.ATTN_TILE = fused, tile
            if (name == "small" and not ops._attn_small_ok(q, n, c)) or (name == "tile" and not ops._attn_use_tile(q, n, c)):
                continue
            qq, kk, vv = (t.detach().requires_grad_() for t in (q, k, v))
            tf = timed(lambda: ops.attention_core(qq, kk, vv))
            o = ops.attention_core(qq, kk, vv)

            def bwd():
                torch.autograd.grad(o, (qq, kk, vv), go, retain_graph=True)
            tb = timed(bwd)
            row[name] = {"fwd_us": round(tf * 1e3, 1), "bwd_us": round(tb * 1e3, 1),
                                                    "fwd_TF/s": round(fl_f / tf / 1e9, 1),
                                                    "bwd_TF/s": round(fl_b / tb / 1e9, 1)}
        out[lab] = row
        print(prec, lab, json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
