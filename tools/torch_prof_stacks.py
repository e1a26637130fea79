#!/usr/bin/env python3
"""Which Python call sites issue torch's small device kernels (copies, fills, elementwise glue) in one config's
training step: torch.profiler with stacks, grouped by the top frames. usage: tools/torch_prof_stacks.py --config c3"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
import medvae_disentangled_multimodal_amd as M

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
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
with torch.profiler.profile(activities=acts, with_stack=True) as prof:
    mod.fit_step(batch, 3)
    torch.cuda.synchronize()
ev = prof.key_averages(group_by_stack_n=6)
rows = []
for e in ev:
    if e.key in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add_", "aten::add", "aten::where", "aten::clone",
                 "aten::mul", "aten::clamp", "aten::isnan", "aten::isfinite", "aten::cat", "aten::zeros", "aten::sub",
                 "aten::div", "aten::eq", "aten::ne", "aten::logical_and", "aten::ones_like", "aten::zeros_like",
                 "aten::full_like", "aten::exp", "aten::sum", "aten::abs", "aten::mean", "aten::neg"):
        rows.append((e.count, e.key, [s for s in e.stack if "medvae" in s or "bench" in s or "torch/autograd" in s][:4]))
rows.sort(key=lambda r: -r[0])
for c, k, st in rows[:60]:
    print(f"{c:4d} {k:18s} {' <- '.join(x.split('/')[-1] for x in st)}")
