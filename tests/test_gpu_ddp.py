"""Data-parallel step on the GPU: two ranks on cuda:0 (gloo carries the collectives between the
processes; the RCCL path is the same DataParallel code with backend "nccl", exercised by the
driver's multi-GPU bench). Checks the overlapped, readiness-driven bucket all-reduce launched from
inside backward by the HIP ops: the averaged flat gradient of 2 ranks x batch 2 equals the single
process gradient of the concatenated batch of 4 (every op is per-sample and the loss is a mean),
within the 3xBF16 tolerance; and the whole DP optimisation step leaves identical parameters on
both ranks."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

KW = dict(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=(1, 2), num_res_blocks=1,
          attn_resolutions=[8], dropout=0.0, resolution=16)


def _data():
    g = torch.Generator().manual_seed(3)
    x = torch.rand(4, 3, 16, 16, generator=g) * 2 - 1
    eps = torch.randn(4, 8, 8, 8, generator=g)
    return x, eps


def _module(dev):
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(0)
    model = M.BaseVAE(**KW).to(dev)
    mod = M.VAELightningModule(model, {"type": "adamw", "lr": 1e-3}, {"type": "none"}, {"type": "vae"},
                               gradient_clip_val=1.0)
    mod.configure_optimizers()
    return mod


def _worker(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    from medvae_disentangled_multimodal_amd import ddp
    dev = torch.device("cuda:0")
    mod = _module(dev)
    dp = ddp.DataParallel(mod, bucket_bytes=64 << 10)  # many buckets
    x, eps = _data()
    sl = slice(2 * rank, 2 * rank + 2)
    batch = (x[sl].to(dev), torch.zeros(2, 1, dtype=torch.long, device=dev))
    mod.optimizer.zero_grad()
    loss = mod.training_step(batch, 0, eps=eps[sl].to(dev))
    dp.begin_backward()
    loss.backward()
    launched_in_backward = sum(dp.launched)
    dp.allreduce_gradients(mod.flat)
    grad = (mod.flat.grad * mod.optimizer.grad_scale).cpu()
    mod.optimizer.step()
    torch.cuda.synchronize()
    torch.save({"grad": grad, "params": mod.flat.data.cpu(), "early": launched_in_backward,
                "nb": len(dp.buckets)}, f"{out_file}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_dp_overlapped_allreduce_matches_global_batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        out = os.path.join(d, "out")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, 2, init_file, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        r0 = torch.load(f"{out}.0", weights_only=True)
        r1 = torch.load(f"{out}.1", weights_only=True)
    assert r0["early"] > 0 and r0["nb"] > 4  # buckets really launched from inside backward
    assert torch.equal(r0["params"], r1["params"])  # identical update on both ranks

    dev = torch.device("cuda:0")
    mod = _module(dev)
    x, eps = _data()
    mod.optimizer.zero_grad()
    loss = mod.training_step((x.to(dev), torch.zeros(4, 1, dtype=torch.long, device=dev)), 0, eps=eps.to(dev))
    loss.backward()
    ref = mod.flat.grad.cpu().double()
    got = r0["grad"].double()
    assert float((got - ref).norm() / ref.norm()) < 1e-3
    # the whole DP step (non-finite zeroing, global clip, AdamW) against the single-process step on the concatenated
    # batch. Adam's first step moves each element by ~lr*sign(g): where the exact gradient is zero (here the conv
    # biases in front of 1-channel-per-group GroupNorms) the sign is rounding noise and may differ between any two
    # summation orders, so those elements are bounded by the step size; every element with a real gradient
    # (|g| > 1e-3 max|g| of its tensor) must agree to 1e-5 relative.
    p0 = mod.flat.data.detach().clone().cpu()
    mod.optimizer.step()
    torch.cuda.synchronize()
    single = mod.flat.data.detach().cpu().double()
    dp_p = r0["params"].double()
    lr = mod.optimizer.param_groups[0]["lr"]
    signal = torch.zeros_like(ref, dtype=torch.bool)
    for prm, off in zip(mod.flat.params, mod.flat.offsets):
        g = ref[off:off + prm.numel()]
        signal[off:off + prm.numel()] = g.abs() > 1e-3 * g.abs().max()
    assert float(signal.double().mean()) > 0.9
    assert float((dp_p[signal] - single[signal]).norm() / single[signal].norm()) < 1e-5
    assert float((dp_p - single).abs().max()) <= 2 * lr * 1.001
    assert not torch.equal(p0.double(), single)


DKW = dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8, hidden_channels=32, ch_mult=(1, 2),
           num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=16)


def _worker_modalities(rank, world, init_file, out_file):
    """Rank 0 sees modalities {0, 1}, rank 1 sees {2, 3, 4}: every head is used on exactly one rank."""
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ddp
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = M.DisentangledConditionalVAE(**DKW).to(dev)
    mod = M.VAELightningModule(model, {"type": "adam", "lr": 5e-4}, {"type": "none"},
                               {"type": "disentangled_vae"}, gradient_clip_val=0.5)
    mod.configure_optimizers()
    ddp.DataParallel(mod, bucket_bytes=64 << 10)
    g = torch.Generator().manual_seed(11 + rank)
    idx = torch.tensor([0, 1, 0, 1] if rank == 0 else [2, 3, 4, 2])
    x = torch.rand(4, 3, 16, 16, generator=g) * 2 - 1
    eps = torch.randn(4, 16, 8, 8, generator=g)
    oh = torch.nn.functional.one_hot(idx, 12).float()
    batch = (x.to(dev), torch.zeros(4, 1, dtype=torch.long, device=dev), oh.to(dev), idx.to(dev))
    for step in range(2):
        mod.fit_step(batch, step, eps=eps.to(dev))
    torch.cuda.synchronize()
    torch.save({"params": mod.flat.data.cpu(), "used": mod._used_mask().cpu(),
                "steps": mod.optimizer.steps.cpu()}, f"{out_file}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_dp_rank_dependent_modalities_keep_replicas_identical():
    """the per-modality parameter mask (clip norm / Adam update / step count) is OR-ed over ranks, so
    parameters stay bitwise identical when ranks see different modalities."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        out = os.path.join(d, "out")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker_modalities, args=(r, 2, init_file, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        r0 = torch.load(f"{out}.0", weights_only=True)
        r1 = torch.load(f"{out}.1", weights_only=True)
    assert torch.equal(r0["used"], r1["used"]) and bool(r0["used"].bool().all()) is False  # embedding unused
    assert torch.equal(r0["steps"], r1["steps"])
    assert torch.equal(r0["params"], r1["params"])


def _worker_graphed(rank, world, init_file, out_file):
    """The DP step replayed from captured graphs (fit_step_graphed, "split" mode: gloo cannot be captured, so graph 1
    = forward + backward, the exchange eager, graph 2 = the optimizer step) against the eager DP step, same inputs:
    4 steps whose modality sets change per step and rank, so the usage mask the optimizer graph reads changes too."""
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ddp
    dev = torch.device("cuda:0")
    idx_sets = [[0, 1, 0, 1], [2, 3, 4, 2], [0, 0, 0, 0], [4, 3, 4, 3]]
    batches = []
    for s in range(4):
        g = torch.Generator().manual_seed(100 * s + rank)
        idx = torch.tensor(idx_sets[(s + rank) % 4])
        x = torch.rand(4, 3, 16, 16, generator=g) * 2 - 1
        eps = torch.randn(4, 16, 8, 8, generator=g)
        oh = torch.nn.functional.one_hot(idx, 12).float()
        batches.append(((x.to(dev), torch.zeros(4, 1, dtype=torch.long, device=dev), oh.to(dev), idx.to(dev)),
                        eps.to(dev)))
    res = {}
    for graphed in (False, True):
        torch.manual_seed(0)
        model = M.DisentangledConditionalVAE(**DKW).to(dev)
        mod = M.VAELightningModule(model, {"type": "adam", "lr": 5e-4}, {"type": "none"},
                                   {"type": "disentangled_vae"}, gradient_clip_val=0.5)
        mod.configure_optimizers()
        ddp.DataParallel(mod, bucket_bytes=64 << 10)
        losses = []
        for s, (batch, eps) in enumerate(batches):
            step = mod.fit_step_graphed if graphed and s > 0 else mod.fit_step
            losses.append(float(step(batch, s, eps=eps)))
        torch.cuda.synchronize()
        res["graphed" if graphed else "eager"] = {"params": mod.flat.data.cpu(), "losses": torch.tensor(losses),
                                                  "steps": mod.optimizer.steps.cpu(),
                                                  "mode": mod._dp_capture_mode() if graphed else ""}
        mod.teardown()
    torch.save(res, f"{out_file}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_dp_graphed_step_matches_eager_dp_step():
    """the captured step under data parallelism. Replays run the same kernels in the same order as the
    eager DP step, so parameters, losses and per-parameter step counts are bitwise equal, and identical across ranks.
    (The RCCL "whole" capture -- the bucket all-reduces inside the one graph -- needs one GPU per rank and is not
    exercised on a 1-GPU box.)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        out = os.path.join(d, "out")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker_graphed, args=(r, 2, init_file, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        r0 = torch.load(f"{out}.0", weights_only=True)
        r1 = torch.load(f"{out}.1", weights_only=True)
    assert r0["graphed"]["mode"] == "split"
    for r in (r0, r1):
        assert torch.equal(r["graphed"]["params"], r["eager"]["params"])
        assert torch.equal(r["graphed"]["losses"], r["eager"]["losses"])
        assert torch.equal(r["graphed"]["steps"], r["eager"]["steps"])
    assert torch.equal(r0["graphed"]["params"], r1["graphed"]["params"])


# a ConditionalVAE of the c4 family (concat conditioning, attention, 3 levels) small enough for 4 ranks on one card; the
# workers and the single-process reference force the Winograd convs (the c4 bench's conv form) onto its 3x3 convs
CKW = dict(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4), num_res_blocks=1, attn_resolutions=[8],
           dropout=0.0, resolution=32, condition_method="concat")
WINO_ENV = {"MVAE_WINOGRAD_MIN_C": "32", "MVAE_WINOGRAD_MIN_C_WIDE": "32", "MVAE_WINOGRAD_MIN_MACS": "0"}


def _cdata(n=8):
    g = torch.Generator().manual_seed(21)
    x = torch.rand(n, 3, 32, 32, generator=g) * 2 - 1
    eps = torch.randn(2, n, 8, 8, 8, generator=g)  # one draw per step
    oh = torch.nn.functional.one_hot(torch.arange(n) % 12, 12).float()
    return x, eps, oh


def _cmodule(dev):
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(5)
    model = M.ConditionalVAE(**CKW).to(dev)
    mod = M.VAELightningModule(model, {"type": "adamw", "lr": 1e-3, "weight_decay": 1e-5, "betas": [0.5, 0.999]},
                               {"type": "none"}, {"type": "vae"}, gradient_clip_val=1.0)
    mod.configure_optimizers()
    return mod


def _worker4(rank, world, init_file, out_file):
    os.environ.update(WINO_ENV)  # (before the package is imported: its dispatch rules read them at import)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    from medvae_disentangled_multimodal_amd import _lib, ddp, ops
    dev = torch.device("cuda:0")
    mod = _cmodule(dev)
    dp = ddp.DataParallel(mod, bucket_bytes=256 << 10)
    seen = set()
    orig = _lib.call

    def spy(name, *args):
        seen.add(name)
        return orig(name, *args)
    _lib.call = spy
    x, eps, oh = _cdata()
    b = x.shape[0] // world
    sl = slice(b * rank, b * rank + b)
    batch = (x[sl].to(dev), torch.zeros(b, 1, dtype=torch.long, device=dev), oh[sl].to(dev))
    mod.fit_step(batch, 0, eps=eps[0, sl].to(dev))
    grad = mod.flat.grad.cpu()  # (the fused step leaves the exchanged gradient scaled by 1/world -- and clipped -- in place)
    p1 = mod.flat.data.cpu()
    mod.fit_step(batch, 1, eps=eps[1, sl].to(dev))
    torch.cuda.synchronize()
    _lib.call = orig
    torch.save({"grad": grad, "p1": p1, "p2": mod.flat.data.cpu(), "scale": float(mod.optimizer.grad_scale),
                "nb": len(dp.buckets), "wino": "mvae_winograd_wgrad_gemm" in seen,
                "steps": mod.optimizer.steps.cpu()}, f"{out_file}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_dp_four_ranks_real_hip_step(monkeypatch):
    """4 data-parallel ranks on the one card (gloo collectives, the HIP step of a c4-family ConditionalVAE with its 3x3
    convs on the Winograd form): the gradient scale is 1/4, the replicas stay bitwise identical over two fused AdamW
    steps, the averaged gradient of 4 x 2 images equals the single-process gradient of the concatenated 8 within 1e-3,
    and the parameters after each step equal the single-process steps' (elements with a real gradient to 1e-4 of the
    update; Adam's sign-noise elements within one step size -- see the 2-rank test)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 4
    with tempfile.TemporaryDirectory() as d:
        init_file, out = os.path.join(d, "init"), os.path.join(d, "out")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker4, args=(r, world, init_file, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    assert all(r["scale"] == 0.25 and r["wino"] and r["nb"] > 1 for r in rs)
    for r in rs[1:]:
        assert torch.equal(r["p1"], rs[0]["p1"]) and torch.equal(r["p2"], rs[0]["p2"])
        assert torch.equal(r["steps"], rs[0]["steps"])

    from medvae_disentangled_multimodal_amd import ops
    for k, v in WINO_ENV.items():
        monkeypatch.setattr(ops, k[5:], float(v) if "MACS" in k else int(v))
    dev = torch.device("cuda:0")
    mod = _cmodule(dev)
    x, eps, oh = _cdata()
    batch = (x.to(dev), torch.zeros(8, 1, dtype=torch.long, device=dev), oh.to(dev))
    p0 = mod.flat.data.cpu().double()
    mod.fit_step(batch, 0, eps=eps[0].to(dev))
    ref = mod.flat.grad.cpu().double()  # (the same in-place clip)
    assert float((rs[0]["grad"].double() - ref).norm() / ref.norm()) < 1e-3
    single1 = mod.flat.data.cpu().double()
    mod.fit_step(batch, 1, eps=eps[1].to(dev))
    torch.cuda.synchronize()
    single2 = mod.flat.data.cpu().double()
    lr = mod.optimizer.param_groups[0]["lr"]
    signal = torch.zeros_like(ref, dtype=torch.bool)
    for prm, off in zip(mod.flat.params, mod.flat.offsets):
        gg = ref[off:off + prm.numel()]
        signal[off:off + prm.numel()] = gg.abs() > 1e-3 * gg.abs().max()
    assert float(signal.double().mean()) > 0.9
    # (the 2 x 4 and 8-image batches round differently through the 3xBF16 F(4x4) convs, ~5e-5 per conv: the
    # parameters agree far inside the north-star 1e-3, and so does each step's UPDATE (measured 2.5e-4 after the first
    # step, 1.2e-3 after the second: Adam's moments carry the first step's difference into the second)
    for dp_p, single, base, steps in ((rs[0]["p1"].double(), single1, p0, 1), (rs[0]["p2"].double(), single2, p0, 2)):
        assert float((dp_p - single).norm() / single.norm()) < 1e-3  # (measured 2.3e-4: sign-noise elements)
        upd = single - base
        err = float((dp_p - single)[signal].norm() / upd[signal].norm())
        assert err < 1e-3 * steps, (steps, err)
        assert float((dp_p - single).abs().max()) <= 2 * steps * lr * 1.001
