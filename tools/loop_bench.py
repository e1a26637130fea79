#!/usr/bin/env python3
"""GEMM main-loop throughput on the conv entry point, per arithmetic: a 1x1 "conv" over [1, 64, 64, K] is a plain
4096 x N x K GEMM (the gather degenerates to row-major loads), next to the c4 / c5 3x3 layers. Times one launch kind
repeatedly with HIP events on the launch stream. tools/loop_bench.py [precision: bf16-mixed | 32 | 32-exact]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from medvae_disentangled_multimodal_amd import ops  # noqa: E402

# (label, n, h, w, cin, cout, k)
CASES = [("gemm4k", 1, 64, 64, 4096, 4096, 1), ("gemm8k_k", 2, 64, 64, 8192, 4096, 1),
         ("c4_8x8x2048", 256, 8, 8, 2048, 2048, 3), ("c4_16x16x1024", 256, 16, 16, 1024, 1024, 3),
         ("c4_64x64x256", 256, 64, 64, 256, 256, 3)]


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16-mixed"
    ops.set_precision(prec)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for lab, n, h, w, c, co, k in CASES:
        p = k // 2
        fmt = ops._dma_fmt()
        if fmt:
            xb = torch.empty(ops._dma_bytes(n * h * w * c), dtype=torch.uint8, device=dev)
            wb = torch.empty(ops._dma_bytes(co * c * k * k), dtype=torch.uint8, device=dev)
            xs = torch.randn(n * h * w * c, device=dev)
            ws = torch.randn(co * c * k * k, device=dev) / (c * k * k) ** 0.5
            fn = "mvae_split_planar" if fmt == 3 else "mvae_pack_bf16"
            ops._lib.call(fn, xs.data_ptr(), xb.data_ptr(), xs.numel(), st)
            ops._lib.call(fn, ws.data_ptr(), wb.data_ptr(), ws.numel(), st)
            flag = ops._dma_flag()
            del xs, ws
        else:
            xb = torch.randn(n * h * w * c, device=dev)
            wb = torch.randn(co * c * k * k, device=dev) / (c * k * k) ** 0.5
            flag = 0
        y = torch.empty(n, co, h, w, device=dev).contiguous(memory_format=torch.channels_last)

        def run():
            ops._conv_call(xb.data_ptr(), wb.data_ptr(), None, None, y, n, h, w, c, co, k, k, 1, p, p, h, w, flag, st)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fl = 2.0 * n * h * w * c * co * k * k
        res[lab] = round(fl / ms / 1e9, 1)
        del xb, wb, y
        torch.cuda.empty_cache()
    print(os.environ.get("MVAE_HIP_LIB", "default"), prec, "TF/s", json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
