#!/usr/bin/env python3
"""Conv passes at c4 / c5 layer shapes through the model's autograd path, timed by the per-launch HIP events of
ops._timed: TF/s per pass (fwd / dgrad / wgrad). tools/dma_exp.py [precision: bf16-mixed (default, the LDS-DMA loop)
| 32 (3xBF16)]. Used to A/B main-loop variants (MVAE_HIP_LIB=variants/<v>/libmvae_hip.so)."""
import json, math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import ops

SHAPES = [(256, 2048, 2048, 8), (256, 1024, 1024, 16), (256, 256, 256, 64)]


def main():
    dev = torch.device("cuda:0")
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16-mixed"
    ops.set_precision(prec)
    out = {}
    for n, ci, co, h in SHAPES:
        g = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
        x = torch.randn(n, ci, h, h, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_()
        w = (torch.randn(co, ci, 3, 3, device=dev) / math.sqrt(ci * 9)).contiguous(
            memory_format=torch.channels_last).requires_grad_()
        dy = torch.randn(n, co, h, h, device=dev).contiguous(memory_format=torch.channels_last)
        for it in range(4):
            ops.PROFILE = [] if it == 3 else None
            y = ops.conv2d(x, w, None, g)
            y.backward(dy)
            torch.cuda.synchronize()
        fl = 2.0 * n * h * h * co * ci * 9
        res = {}
        for tag, flops, s, e, shape, ref in ops.PROFILE:
            res[tag] = round(flops / (s.elapsed_time(e) * 1e-3) / 1e12, 1)
        ops.PROFILE = None
        out[f"{ci}x{h}"] = res
        del x, w, dy, y
        torch.cuda.empty_cache()
    print(os.environ.get("MVAE_HIP_LIB", "default"), prec, json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
