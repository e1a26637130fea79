"""Data-parallel plumbing on CPU (gloo, world_size 2): initial-parameter broadcast, the bucketed
all-reduce of the ONE flat gradient buffer, and the 1/world average folded into the optimizer's
grad_scale. The averaged gradient must equal the gradient of the concatenated global batch (the DDP
parity argument of SURVEY.md section 8(e): every op of the VAE is per-sample and the loss is a mean)."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Mod:
    """Stand-in for VAELightningModule: only the attributes ddp.DataParallel touches."""

    def __init__(self, model):
        from medvae_disentangled_multimodal_amd.optim import FlatParameters

        class _Opt:
            grad_scale = 1.0
        self.model = model
        self.flat = FlatParameters(model, torch.device("cpu"))
        self.optimizer = _Opt()
        self.process_group = None

    def configure_optimizers(self):
        pass


def _worker(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    from medvae_disentangled_multimodal_amd import ddp
    torch.manual_seed(100 + rank)  # different init on each rank: broadcast must fix it
    model = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    mod = _Mod(model)
    dp = ddp.DataParallel(mod, bucket_bytes=64)  # tiny buckets: exercise the slicing
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 7, generator=g)
    y = torch.randn(8, 3, generator=g)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    mod.flat.zero_grad()
    loss = torch.nn.functional.mse_loss(model(xs), ys)
    dp.begin_backward()
    loss.backward()
    # overlap: every bucket whose parameters all reported was launched during backward, in order
    assert all(dp.launched), dp.launched
    assert dp.next_bucket == len(dp.buckets) > 1
    dp.allreduce_gradients(mod.flat)
    avg = mod.flat.grad * mod.optimizer.grad_scale
    if rank == 0:
        torch.save({"params": mod.flat.data.clone(), "grad": avg.clone()}, out_file)
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_plan_covers_flat_buffer():
    from medvae_disentangled_multimodal_amd import ddp
    model = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3), torch.nn.Linear(3, 9))
    mod = _Mod(model)
    dp = ddp.DataParallel.__new__(ddp.DataParallel)
    dp.module, dp.bucket_elems = mod, 16
    dp._plan(mod.flat)
    # contiguous, non-overlapping, reverse order, covering the whole buffer, whole parameters only
    spans = sorted(dp.buckets)
    assert spans[0][0] == 0 and spans[-1][1] == mod.flat.numel
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert dp.buckets[0][1] == mod.flat.numel  # the decoder-side (last) parameters go first
    assert sum(dp.expected) == len(mod.flat.params)


def test_flat_gradient_allreduce_matches_global_batch():
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        out_file = os.path.join(d, "out.pt")
        mp.spawn(_worker, args=(2, init_file, out_file), nprocs=2, join=True)
        res = torch.load(out_file, weights_only=True)
    # reference: rank-0 initial weights (broadcast), the full batch of 8, one process
    torch.manual_seed(100)
    ref = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    flat_ref = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    from medvae_disentangled_multimodal_amd.optim import FlatParameters
    f = FlatParameters(ref, torch.device("cpu"))
    assert torch.allclose(res["params"], f.data)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 7, generator=g)
    y = torch.randn(8, 3, generator=g)
    f.zero_grad()
    torch.nn.functional.mse_loss(ref(x), y).backward()
    assert torch.allclose(res["grad"], f.grad, rtol=1e-5, atol=1e-7)
    assert flat_ref.numel() <= f.numel


def _worker_unused(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    from medvae_disentangled_multimodal_amd import ddp
    torch.manual_seed(5)
    a, b = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)  # b (last => first bucket) is used by rank 0 only
    model = torch.nn.ModuleList([a, b])
    mod = _Mod(model)
    dp = ddp.DataParallel(mod, bucket_bytes=16)
    x = torch.full((2, 4), float(rank + 1))
    mod.flat.zero_grad()
    out = a(x)
    if rank == 0:
        out = b(out)
    dp.begin_backward()
    out.sum().backward()
    dp.allreduce_gradients(mod.flat)  # same collective sequence on both ranks: no hang
    if rank == 0:
        torch.save({"b_w": b.weight._mvae_main_grad.clone(), "a_b": a.bias._mvae_main_grad.clone()}, out_file)
    dist.barrier()
    dist.destroy_process_group()


def test_overlap_with_rank_dependent_unused_parameters():
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        out_file = os.path.join(d, "out.pt")
        mp.spawn(_worker_unused, args=(2, init_file, out_file), nprocs=2, join=True)
        res = torch.load(out_file, weights_only=True)
    torch.manual_seed(5)
    a, b = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)
    h0 = a(torch.full((2, 4), 1.0))
    b(h0).sum().backward()
    gb0 = b.weight.grad.clone()
    a.zero_grad()
    b.zero_grad()
    a(torch.full((2, 4), 2.0)).sum().backward()
    ga1 = a.bias.grad.clone()
    a.zero_grad()
    b(a(torch.full((2, 4), 1.0))).sum().backward()
    ga0 = a.bias.grad.clone()
    assert torch.allclose(res["b_w"], gb0, atol=1e-6)         # only rank 0 contributed
    assert torch.allclose(res["a_b"], ga0 + ga1, atol=1e-6)   # summed over ranks


W8_IDS = ([0, 1, 0, 1, 0, 0, 1, 1, 0, 1, 1, 0, 0, 1, 0, 0, 1, 1, 0, 1, 3, 1, 0, 0, 1, 0, 1, 1, 0, 1, 0, 0],  # step 0
          [1, 0, 0, 1, 1, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 0, 1, 0, 0, 1, 1, 0, 0, 1, 0, 1, 1, 0, 1, 0, 0, 1])  # step 1
# head 2 is used by no rank (never updated), head 3 only by rank 5 at step 0 (updated on every replica at step 0 only)


class _Heads(torch.nn.Module):
    """A shared trunk and per-modality heads (the disentangled model's routing in miniature)."""

    def __init__(self):
        super().__init__()
        self.trunk = torch.nn.Linear(6, 8)
        self.heads = torch.nn.ModuleList([torch.nn.Linear(8, 3) for _ in range(4)])

    def forward(self, x, ids):
        h = torch.tanh(self.trunk(x))
        return torch.stack([self.heads[int(i)](h[j]) for j, i in enumerate(ids)])


def _w8_data(step):
    g = torch.Generator().manual_seed(11 + step)
    return torch.randn(32, 6, generator=g), torch.randn(32, 3, generator=g), torch.tensor(W8_IDS[step])


def _w8_opt_step(model, opt, grads, used_heads, clip):
    """torch AdamW over the parameters the used-mask keeps (the rest get no update and no step count, like
    FusedAdam's `used` mask), after the global-norm clip of lightning_module.py:452-466"""
    for name, p in model.named_parameters():
        keep = not name.startswith("heads.") or used_heads[int(name.split(".")[1])]
        p.grad = grads[name].clone() if keep else None
    torch.nn.utils.clip_grad_norm_([p for p in model.parameters() if p.grad is not None], clip)
    opt.step()


def _worker_w8(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    from medvae_disentangled_multimodal_amd import ddp
    torch.manual_seed(300 + rank)  # different init everywhere: the broadcast must fix it
    model = _Heads()
    mod = _Mod(model)
    dp = ddp.DataParallel(mod, bucket_bytes=96)
    assert mod.optimizer.grad_scale == 1.0 / 8 and len(dp.buckets) > 3
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, betas=(0.5, 0.999), weight_decay=1e-5)
    used_log = []
    for step in range(2):
        x, y, ids = _w8_data(step)
        sl = slice(rank * 4, rank * 4 + 4)
        mod.flat.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x[sl], ids[sl]), y[sl])
        dp.begin_backward()
        loss.backward()
        dp.allreduce_gradients(mod.flat)
        present = torch.zeros(4, dtype=torch.bool)
        present[ids[sl]] = True
        used = dp.any_across_ranks(present)  # the per-modality used-mask, OR-ed over ranks
        used_log.append(used.tolist())
        grads = {n: p._mvae_main_grad * mod.optimizer.grad_scale for n, p in model.named_parameters()}
        _w8_opt_step(model, opt, grads, used.tolist(), 1.0)
    mine = mod.flat.data.clone()
    allp = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allp, mine)
    if rank == 0:
        torch.save({"params": mine, "replicas_equal": all(torch.equal(mine, q) for q in allp), "used": used_log},
                   out_file)
    dist.barrier()
    dist.destroy_process_group()


def test_dp_world8_matches_concatenated_batch_and_replicas_agree():
    """8 gloo ranks (the node's real width): bucket plan, grad_scale 1/8, rank-dependent unused parameters with the
    OR-ed used-mask, two AdamW steps; the replicas stay bitwise identical and equal the single-process steps on the
    concatenated 8x batch."""
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "init")
        out_file = os.path.join(d, "out.pt")
        mp.spawn(_worker_w8, args=(8, init_file, out_file), nprocs=8, join=True)
        res = torch.load(out_file, weights_only=True)
    assert res["replicas_equal"]
    assert res["used"] == [[True, True, False, True], [True, True, False, False]]
    torch.manual_seed(300)  # rank 0's initial weights (the broadcast)
    ref = _Heads()
    head2 = ref.heads[2].weight.detach().clone()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, betas=(0.5, 0.999), weight_decay=1e-5)
    for step in range(2):
        x, y, ids = _w8_data(step)
        ref.zero_grad()
        torch.nn.functional.mse_loss(ref(x, ids), y).backward()
        used = [bool((ids == h).any()) for h in range(4)]
        _w8_opt_step(ref, opt, {n: p.grad for n, p in ref.named_parameters()}, used, 1.0)
    from medvae_disentangled_multimodal_amd.optim import FlatParameters
    f = FlatParameters(ref, torch.device("cpu"))
    assert torch.equal(ref.heads[2].weight.detach(), head2)  # never used: never moved
    err = ((res["params"] - f.data).norm() / f.data.norm()).item()
    assert err < 1e-5, err


def test_dp_capture_mode_selection(monkeypatch):
    """fit_step_graphed's data-parallel capture mode: single process -> "single"; any backend ->
    "split" (two graphs around an eager exchange: the mode whose run is bitwise-tested); MVAE_DP_CAPTURE=whole records
    the bucket all-reduces inside the one step graph (RCCL capture, opt-in: never run on this build's 1-GPU boxes)."""
    from medvae_disentangled_multimodal_amd.lightning_module import VAELightningModule

    class PG:
        def __init__(self, world, backend):
            self.world, self._b = world, backend

        def backend(self):
            return self._b

    mod = VAELightningModule.__new__(VAELightningModule)
    monkeypatch.delenv("MVAE_DP_CAPTURE", raising=False)
    mod.process_group = None
    assert mod._dp_capture_mode() == "single"
    mod.process_group = PG(1, "nccl")
    assert mod._dp_capture_mode() == "single"
    mod.process_group = PG(2, "nccl")
    assert mod._dp_capture_mode() == "split"
    mod.process_group = PG(2, "gloo")
    assert mod._dp_capture_mode() == "split"
    monkeypatch.setenv("MVAE_DP_CAPTURE", "split")
    mod.process_group = PG(8, "nccl")
    assert mod._dp_capture_mode() == "split"
    monkeypatch.setenv("MVAE_DP_CAPTURE", "whole")
    mod.process_group = PG(2, "gloo")
    assert mod._dp_capture_mode() == "whole"
