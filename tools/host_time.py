#!/usr/bin/env python3
"""Host dispatch time vs GPU time per training step (is a config launch-bound?).
usage: tools/host_time.py <config> [steps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
import medvae_disentangled_multimodal_amd as M
cfg = dict(bench.CONFIGS[sys.argv[1]])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda:0")
torch.manual_seed(42)
model = getattr(M, cfg["cls"])(**cfg["kwargs"]).to(dev)
mod = M.VAELightningModule(model, cfg["opt"], {"type": "none"}, cfg["loss"], gradient_clip_val=cfg["clip"],
                           precision=cfg.get("precision", "32"))
mod.configure_optimizers()
gen = torch.Generator(device=dev).manual_seed(1)
batches = [bench.make_batch(cfg, dev, gen) for _ in range(2)]
for i in range(5):
    mod.fit_step(batches[i % 2], i)
torch.cuda.synchronize()
host, wall = [], []
for i in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mod.fit_step(batches[i % 2], i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.append(t1 - t0); wall.append(t2 - t0)
host.sort(); wall.sort()
print(f"{sys.argv[1]}: host dispatch median {1e3 * host[len(host) // 2]:.2f} ms, step (synced) median "
      f"{1e3 * wall[len(wall) // 2]:.2f} ms, min {1e3 * wall[0]:.2f} max {1e3 * wall[-1]:.2f}")
