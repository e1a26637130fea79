"""Probe for the 4-rank data-parallel test (tests/test_gpu_ddp.py::test_dp_four_ranks_real_hip_step): the same model and
forced-Winograd settings, single process ("single") or 4 gloo ranks on the one card ("dp4"), printing each phase so a
hang or fault names where it happened. Usage: python tools/dp4_probe.py single|dp4 [--no-wino]"""
import faulthandler
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
WINO = "--no-wino" not in sys.argv
if WINO:
    os.environ.update({"MVAE_WINOGRAD_MIN_C": "32", "MVAE_WINOGRAD_MIN_C_WIDE": "32", "MVAE_WINOGRAD_MIN_MACS": "0"})

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def log(*a):
    print(f"[{os.getpid()} {time.strftime('%H:%M:%S')}]", *a, flush=True)


def run(rank, world, init_file):
    faulthandler.dump_traceback_later(90, exit=True)
    from test_gpu_ddp import _cdata, _cmodule
    if world > 1:
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    from medvae_disentangled_multimodal_amd import ddp
    dev = torch.device("cuda:0")
    mod = _cmodule(dev)
    log(rank, "module built")
    if world > 1:
        ddp.DataParallel(mod, bucket_bytes=256 << 10)
    x, eps, oh = _cdata()
    b = x.shape[0] // world
    sl = slice(b * rank, b * rank + b)
    batch = (x[sl].to(dev), torch.zeros(b, 1, dtype=torch.long, device=dev), oh[sl].to(dev))
    for s in range(2):
        mod.optimizer.zero_grad()
        loss = mod.training_step(batch, s, eps=eps[s, sl].to(dev))
        torch.cuda.synchronize()
        log(rank, "step", s, "forward ok", float(loss))
        mod.fit_step(batch, s, eps=eps[s, sl].to(dev))
        torch.cuda.synchronize()
        log(rank, "step", s, "fit_step ok")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    if sys.argv[1] == "single":
        run(0, 1, None)
    else:
        with tempfile.TemporaryDirectory() as d:
            ctx = mp.get_context("spawn")
            ps = [ctx.Process(target=run, args=(r, 4, os.path.join(d, "init"))) for r in range(4)]
            for p in ps:
                p.start()
            for p in ps:
                p.join(timeout=150)
            log("exit codes", [p.exitcode for p in ps])
            sys.exit(0 if all(p.exitcode == 0 for p in ps) else 1)
