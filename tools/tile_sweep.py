#!/usr/bin/env python3
"""Tile-config sweep of the conv GEMMs on c2 / c3 / c4 layer shapes: one process per forced tile
(MVAE_GEMM_TILE=0..4: 256x256, 256x128, 128x256, 128x128, 64x64; -1 = the heuristic). Prints TF/s per pass."""
import json, os, subprocess, sys, time
SHAPES = [  # n, cin, cout, h
    (256, 512, 512, 7), (256, 256, 256, 14), (256, 128, 128, 28),          # c2
    (512, 128, 128, 7), (512, 64, 64, 14), (512, 32, 32, 28),              # c3
    (256, 2048, 2048, 8), (256, 1024, 1024, 16),                           # c4
]
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    from medvae_disentangled_multimodal_amd import ops
    dev = torch.device("cuda:0")
    g = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
    out = {}
    for n, ci, co, h in SHAPES:
        x = torch.randn(n, ci, h, h, device=dev).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 3, 3, device=dev) * 0.02).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, co, h, h, device=dev).contiguous(memory_format=torch.channels_last)
        dw = torch.zeros_like(w)
        fl = 2.0 * n * h * h * co * ci * 9
        res = []
        for fn in (lambda: ops.conv2d_forward_raw(x, w, None, None, g), lambda: ops.conv2d_dgrad_raw(dy, w, x.shape, g),
                   lambda: ops.conv2d_wgrad_raw(dy, x, dw, 0.0, g)):
            fn(); torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            res.append(round(fl / ((time.perf_counter() - t) / 10) / 1e12, 1))
        out[f"{n}x{ci}->{co}@{h}"] = res
    print(json.dumps(out))
    sys.exit(0)
rows = {}
for tile in (-1, 0, 1, 2, 3, 4):
    env = dict(os.environ, MVAE_GEMM_TILE=str(tile))
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        print("tile", tile, "failed", r.stderr[-500:]); continue
    rows[tile] = json.loads(r.stdout.strip().splitlines()[-1])
for shp in rows[-1]:
    print(f"{shp:22s}", "  ".join(f"t{t}:{'/'.join(str(v) for v in rows[t][shp])}" for t in rows))
