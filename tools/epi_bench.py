#!/usr/bin/env python3
"""GEMM epilogue cost on the c4 conv layers: the same 3x3 forward conv timed plain, with the residual add, with the
GroupNorm-statistics epilogue, and with both (HIP events on the launch stream). tools/epi_bench.py [precision]"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from medvae_disentangled_multimodal_amd import ops  # noqa: E402

SHAPES = [(256, 256, 64), (256, 512, 32), (256, 1024, 16), (256, 2048, 8)]


def timed(fn, reps=5):
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
    g = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
    out = {}
    for n, c, h in SHAPES:
        x = torch.randn(n, c, h, h, device=dev).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device=dev) / math.sqrt(9 * c)).contiguous(memory_format=torch.channels_last)
        b = torch.randn(c, device=dev)
        res = torch.randn_like(x)
        part = torch.empty(n * h * h // 32 * (c // 4) * 2, device=dev, dtype=torch.float64)
        wk = ops._krsc(w)
        row = {}
        for rep in range(2):  # interleaved twice (the first launches of a process run at a lower clock)
            for lab, r, p in (("stats", None, part), ("plain", None, None), ("res", res, None),
                              ("res+stats", res, part)):
                ms = timed(lambda: ops.conv2d_forward_raw(x, wk, b, r, g, False, p))
                row[f"{lab}_{rep}"] = round(ms * 1e3, 1)
        out[f"{c}x{h}"] = row
        print(prec, f"{c}x{h}", json.dumps(row), flush=True)
        del x, w, res, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
