#!/usr/bin/env python3
"""Per-shape timing of the implicit-GEMM conv passes (fwd / dgrad / wgrad) on the GPU, for the
conv layer classes of BASELINE config 4 (multi_modal_cvae @ 64x64, bs 256). Prints TFLOP/s per
pass (algorithmic FLOPs = 2*M*N*K of the reference conv)."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from medvae_disentangled_multimodal_amd import ops

SHAPES = [  # n, cin, cout, h, k, stride, pads, ups
    (256, 256, 256, 64, 3, 1, (1, 1, 1, 1), False),
    (256, 512, 512, 32, 3, 1, (1, 1, 1, 1), False),
    (256, 1024, 1024, 16, 3, 1, (1, 1, 1, 1), False),
    (256, 2048, 2048, 8, 3, 1, (1, 1, 1, 1), False),
    (256, 1024, 1024, 16, 1, 1, (0, 0, 0, 0), False),
    (256, 512, 512, 32, 3, 1, (1, 1, 1, 1), True),     # upsample conv 32 -> 64
    (256, 256, 256, 64, 3, 2, (0, 0, 1, 1), False),    # downsample 64 -> 32
]


def bench(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda:0")
    res = []
    for n, ci, co, h, k, s, pads, ups in SHAPES:
        g = ops.ConvGeom(k, k, s, pads[0], pads[1], pads[2], pads[3], ups)
        x = torch.randn(n, ci, h, h, device=dev).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, k, k, device=dev) * 0.02).contiguous(memory_format=torch.channels_last)
        b = torch.zeros(co, device=dev)
        ho, wo = g.out_hw(h, h)
        dy = torch.randn(n, co, ho, wo, device=dev).contiguous(memory_format=torch.channels_last)
        dw = torch.zeros_like(w)
        fl = 2.0 * n * ho * wo * co * ci * k * k
        tf = bench(lambda: ops.conv2d_forward_raw(x, w, b, None, g))
        td = bench(lambda: ops.conv2d_dgrad_raw(dy, w, x.shape, g))
        tw = bench(lambda: ops.conv2d_wgrad_raw(dy, x, dw, 0.0, g))
        r = dict(shape=f"{ci}->{co} k{k} s{s} {h}x{h}{' ups' if ups else ''}", gflop=round(fl / 1e9, 1),
                 fwd_tf=round(fl / tf / 1e12, 1), dgrad_tf=round(fl / td / 1e12, 1), wgrad_tf=round(fl / tw / 1e12, 1),
                 ms=[round(tf * 1e3, 2), round(td * 1e3, 2), round(tw * 1e3, 2)])
        if k == 3 and s == 1 and not ups:  # the training path: GroupNorm output handed over pre-split (3xBF16 hi/lo)
            xs = torch.empty_like(x)
            ops._lib.call("mvae_split_bf16", x.data_ptr(), xs.data_ptr(), x.numel(), ops._stream(x))
            tfs = bench(lambda: ops.conv2d_forward_raw(xs, w, b, None, g, True))
            tws = bench(lambda: ops.conv2d_wgrad_raw(dy, xs, dw, 0.0, g, x_split=True))
            r.update(fwd_split_tf=round(fl / tfs / 1e12, 1), wgrad_split_tf=round(fl / tws / 1e12, 1))
            del xs
        print(json.dumps(r), flush=True)
        res.append(r)
        del x, w, dy, dw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
