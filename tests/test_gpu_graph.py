"""The graph-replayed training step (VAELightningModule.fit_step_graphed): one captured HIP graph of the whole
optimisation step must give exactly the eager step's results (same kernels, same inputs), advance the device
dropout salt once per replay, and re-capture when the learning rate changes."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DIS = dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4),
           num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28, modality_separation_weight=0.1,
           contrastive_weight=0.05)
CVAE = dict(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4), num_res_blocks=1,
            attn_resolutions=[14], dropout=0.0, resolution=28, condition_method="concat")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _module(cls, kw, loss, dev):
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(11)
    model = getattr(M, cls)(**kw).to(dev)
    opt = dict(type="adam", lr=5e-4, weight_decay=0.0, betas=[0.9, 0.999])
    mod = M.VAELightningModule(model, opt, {"type": "none"}, loss, gradient_clip_val=0.5)
    mod.configure_optimizers()
    return mod


def _batch(cls, dev, B=16):
    g = torch.Generator().manual_seed(5)
    x = (torch.randint(0, 256, (B, 3, 28, 28), generator=g).float() / 255 * 2 - 1).to(dev)
    labels = torch.zeros(B, 1, dtype=torch.long, device=dev)
    if cls == "DisentangledConditionalVAE":
        idx = torch.tensor([0, 1, 2, 3, 4, 1, 2, 4, 0, 3, 1, 2, 4, 4, 1, 2][:B], device=dev)
        return (x, labels, torch.nn.functional.one_hot(idx, 12).float(), idx)
    idx = torch.arange(B, device=dev) % 12
    return (x, labels, torch.nn.functional.one_hot(idx, 12).float())


CASES = [("DisentangledConditionalVAE", DIS, dict(type="disentangled_vae", recon_loss_type="mse", kl_weight=1.0,
                                                  recon_weight=1.0, separation_weight=0.1, contrastive_weight=0.05)),
         ("ConditionalVAE", CVAE, dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0))]


@pytest.mark.parametrize("cls,kw,loss", CASES)
def test_graphed_steps_match_eager_steps(dev, cls, kw, loss):
    batch = _batch(cls, dev)
    a = _module(cls, kw, loss, dev)
    b = _module(cls, kw, loss, dev)
    r = 28 // 2 ** (len(kw["ch_mult"]) - 1)
    g = torch.Generator().manual_seed(8)
    eps = [torch.randn(16, a.model.latent_dim, r, r, generator=g).to(dev) for _ in range(4)]
    assert torch.equal(a.flat.data, b.flat.data)
    la = [a.fit_step(batch, i, eps=eps[i]) for i in range(4)]
    lb = [b.fit_step(batch, 0, eps=eps[0])] + [b.fit_step_graphed(batch, i, eps=eps[i]).clone() for i in range(1, 4)]
    torch.cuda.synchronize()
    # the HIP kernels are deterministic; torch glue (the contrastive term's small mm) may pick another BLAS kernel
    # under capture, hence a rounding-level tolerance rather than bitwise equality
    for x, y in zip(la, lb):
        assert abs(float(x) - float(y)) <= 1e-5 * abs(float(x)) + 1e-7, (float(x), float(y))
    d = (a.flat.data - b.flat.data).abs().max()
    assert float(d) <= 1e-5, float(d)
    assert torch.allclose(a.optimizer.exp_avg, b.optimizer.exp_avg, rtol=1e-4, atol=1e-9)
    assert a.global_step_count == b.global_step_count == 4


def test_graph_salt_advances_and_lr_change_recaptures(dev):
    kw = dict(DIS, dropout=0.1)
    mod = _module("DisentangledConditionalVAE", kw, CASES[0][2], dev)
    batch = _batch("DisentangledConditionalVAE", dev)
    mod.fit_step(batch, 0)
    l1 = float(mod.fit_step_graphed(batch, 1))
    g1 = mod._graph["graph"]
    s1 = int(mod._graph["salt"].item())
    l2 = float(mod.fit_step_graphed(batch, 2))
    assert int(mod._graph["salt"].item()) == s1 + 1  # one advance per replay: fresh dropout masks
    assert mod._graph["graph"] is g1
    mod.optimizer.param_groups[0]["lr"] = 1e-4  # a scheduler step: the frozen lr must not be replayed
    l3 = float(mod.fit_step_graphed(batch, 3))
    assert mod._graph["graph"] is not g1
    assert all(v == v and abs(v) < 1e6 for v in (l1, l2, l3))


def test_graph_survives_eager_calls_that_grow_the_arena(dev):
    """a replay writes into the scratch buffers baked into the graph. An eager evaluate at twice
    the batch grows (replaces) those arena buffers between replays; the graph must keep its own buffers alive, so
    graphed steps interleaved with the large eager call give the eager-only steps' results."""
    from medvae_disentangled_multimodal_amd import ops
    cls, kw, loss = CASES[1]
    batch, big = _batch(cls, dev), _batch(cls, dev, B=32)
    a = _module(cls, kw, loss, dev)
    b = _module(cls, kw, loss, dev)
    r = 28 // 2 ** (len(kw["ch_mult"]) - 1)
    g = torch.Generator().manual_seed(9)
    eps = [torch.randn(16, a.model.latent_dim, r, r, generator=g).to(dev) for _ in range(4)]
    la = [a.fit_step(batch, i, eps=eps[i]) for i in range(4)]
    lb = [b.fit_step(batch, 0, eps=eps[0]), b.fit_step_graphed(batch, 1, eps=eps[1]).clone()]
    gen0 = ops.ARENA.generation
    ea = b.evaluate(big)  # eager, 2x batch: outgrows the scratch buffers the graph captured
    assert ops.ARENA.generation > gen0 and b._graph["arena"], "the test needs an arena reallocation"
    junk = torch.full((64 << 20,), float("nan"), device=dev)  # reuse freed memory, if any was freed
    lb += [b.fit_step_graphed(batch, i, eps=eps[i]).clone() for i in (2, 3)]
    torch.cuda.synchronize()
    del junk
    for x, y in zip(la, lb):
        assert abs(float(x) - float(y)) <= 1e-5 * abs(float(x)) + 1e-7, (float(x), float(y))
    assert float((a.flat.data - b.flat.data).abs().max()) <= 1e-5
    assert all(torch.isfinite(v).all() for v in ea.values() if torch.is_tensor(v))


def test_graph_key_covers_optimizer_hyperparameters(dev):
    """betas / eps / weight decay / clip norm are frozen into the captured launches; changing
    any of them (e.g. a checkpoint load) must re-capture."""
    cls, kw, loss = CASES[1]
    mod = _module(cls, kw, loss, dev)
    batch = _batch(cls, dev)
    mod.fit_step(batch, 0)
    mod.fit_step_graphed(batch, 1)
    g1 = mod._graph["graph"]
    mod.fit_step_graphed(batch, 2)
    assert mod._graph["graph"] is g1
    mod.optimizer.param_groups[0]["betas"] = (0.5, 0.999)
    mod.fit_step_graphed(batch, 3)
    g2 = mod._graph["graph"]
    assert g2 is not g1
    mod.optimizer.max_grad_norm = 2.0
    mod.fit_step_graphed(batch, 4)
    assert mod._graph["graph"] is not g2


def test_failed_capture_falls_back_with_the_step_count_intact(dev, monkeypatch):
    """A capture that fails after the recorded fit_step advanced the host step counter (here: at capture_end) leaves
    the counter where it was, runs the step eagerly and stays eager for that key; an error of the step itself (not a
    capture error) propagates."""
    cls, kw, loss = CASES[1]
    mod = _module(cls, kw, loss, dev)
    batch = _batch(cls, dev)
    mod.fit_step(batch, 0)
    assert mod.global_step_count == 1

    orig = torch.cuda.CUDAGraph.capture_end

    def boom(self, *a, **k):  # (the capture itself ends, so the stream leaves capture mode, then the failure)
        orig(self, *a, **k)
        raise RuntimeError("hipErrorStreamCaptureInvalidated: capture failed (test)")

    monkeypatch.setattr(torch.cuda.CUDAGraph, "capture_end", boom)
    with pytest.warns(UserWarning, match="capture failed"):
        mod.fit_step_graphed(batch, 1)
    assert mod.global_step_count == 2  # one eager step, not one plus the recorded one
    assert getattr(mod, "_graph", None) is None
    mod.fit_step_graphed(batch, 2)  # (same key: eager without another capture attempt)
    assert mod.global_step_count == 3
    monkeypatch.undo()
    torch.cuda.synchronize()

    from medvae_disentangled_multimodal_amd import lightning_module as LM
    assert LM._is_capture_error(RuntimeError("operation not permitted when stream is capturing"))
    assert not LM._is_capture_error(RuntimeError("conv2d: a pre-split input needs cin % 4 == 0"))
