#!/usr/bin/env python3
"""The achievable library GEMM rate on this box (tools-only measurement, not product): torch.matmul (hipBLASLt /
rocBLAS) on uniform random [-1, 1) operands, bf16 and fp32, at the plain 4096^3 / 8192^3 squares and at the GEMM shapes
of the c4 / c5 convolutions (M = pixels, N = cout, K = taps * cin: the implicit-GEMM problem as if the im2col were
free; 1x1 convs exactly). The target the conv GEMMs are measured against.
usage: tools/blas_ceiling.py [--reps 20]"""
import argparse
import json

import torch

SHAPES = [  # name, M, N, K
    ("square 4096", 4096, 4096, 4096),
    ("square 8192", 8192, 8192, 8192),
    ("c4 3x3 64x64x256 (im2col)", 256 * 64 * 64, 256, 9 * 256),
    ("c4 3x3 32x32x512 (im2col)", 256 * 32 * 32, 512, 9 * 512),
    ("c4 3x3 16x16x1024 (im2col)", 256 * 16 * 16, 1024, 9 * 1024),
    ("c4 3x3 8x8x2048 (im2col)", 256 * 8 * 8, 2048, 9 * 2048),
    ("c4 1x1 16x16 1024->1024", 256 * 16 * 16, 1024, 1024),
    ("c4 1x1 32x32 512->1024", 256 * 32 * 32, 1024, 512),
    ("wgrad 8x8x2048 (K = pixels)", 2048, 9 * 2048, 256 * 8 * 8),
    ("wgrad 64x64x256 (K = pixels)", 256, 9 * 256, 256 * 64 * 64),
]


def bench(m, n, k, dt, reps, dev):
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    a = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(dt)
    b = (torch.rand(k, n, device=dev, generator=g) * 2 - 1).to(dt)
    c = torch.empty(m, n, device=dev, dtype=dt)
    for _ in range(3):
        torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b, out=c)
    e1.record()
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) / reps * 1e-3
    return 2.0 * m * n * k / s / 1e12, s * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.backends.cuda.matmul.allow_tf32 = False
    for name, m, n, k in SHAPES:
        for dt in (torch.bfloat16, torch.float32):
            if dt == torch.float32 and m * n * k > 1 << 37:
                reps = max(2, a.reps // 5)
            else:
                reps = a.reps
            tf, ms = bench(m, n, k, dt, reps, dev)
            print(json.dumps({"shape": name, "M": m, "N": n, "K": k, "dtype": str(dt).split(".")[1],
                              "TFLOP/s": round(tf, 1), "ms": round(ms, 3)}), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
