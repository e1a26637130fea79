#!/usr/bin/env python3
"""torch.profiler view of one bench config's training step: which host-side ops launch the small device
kernels (copies, fills, torch elementwise glue). usage: tools/torch_prof.py --config c3"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
import medvae_disentangled_multimodal_amd as M

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--rows", type=int, default=45)
a = ap.parse_args()
dev = torch.device("cuda:0")
cfg = dict(bench.CONFIGS[a.config])
torch.manual_seed(42)
model = getattr(M, cfg["cls"])(**cfg["kwargs"]).to(dev)
mod = M.VAELightningModule(model, cfg["opt"], {"type": "none"}, cfg["loss"], gradient_clip_val=cfg["clip"],
                           precision=cfg.get("precision", "32"))
mod.configure_optimizers()
gen = torch.Generator(device=dev).manual_seed(1234)
batch = bench.make_batch(cfg, dev, gen)
for i in range(3):
    mod.fit_step(batch, i)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
    for i in range(2):
        mod.fit_step(batch, 3 + i)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="count", row_limit=a.rows, max_name_column_width=70))
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=70))
