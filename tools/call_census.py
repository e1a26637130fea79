"""Which library entry points (and how often) one training step of a bench config calls: a spy on _lib.call during one
eager fit_step after a warm-up step. Usage: python tools/call_census.py [config] -- e.g. c4 (prints name, count, and the
size arguments of the implicit-GEMM weight-gradient calls)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from medvae_disentangled_multimodal_amd import _lib  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    import medvae_disentangled_multimodal_amd as M
    cfg = dict(bench.CONFIGS[name])
    dev = torch.device("cuda:0")
    torch.manual_seed(42)
    model = getattr(M, cfg["cls"])(**cfg["kwargs"]).to(dev)
    mod = M.VAELightningModule(model, cfg["opt"], {"type": "none"}, cfg["loss"], gradient_clip_val=cfg["clip"],
                               precision=cfg.get("precision", "32"))
    mod.configure_optimizers()
    gen = torch.Generator(device=dev).manual_seed(1234)
    batches = [bench.make_batch(cfg, dev, gen) for _ in range(2)]
    step = mod.fit_step
    step(batches[0], 0)
    torch.cuda.synchronize()
    seen = collections.Counter()
    wg = collections.Counter()
    orig = _lib.call

    def spy(fn, *args):
        seen[fn] += 1
        if fn == "mvae_conv2d_wgrad_nhwc":
            wg[tuple(args[5:17])] += 1
        return orig(fn, *args)
    _lib.call = spy
    step(batches[1], 1)
    torch.cuda.synchronize()
    _lib.call = orig
    for k, v in seen.most_common():
        print(f"{v:5d}  {k}")
    print("mvae_conv2d_wgrad_nhwc (n, h, w, c, co, kh, kw, stride, pad_t, pad_l, ho, wo):")
    for k, v in wg.most_common():
        print(f"{v:5d}  {k}")


if __name__ == "__main__":
    main()
