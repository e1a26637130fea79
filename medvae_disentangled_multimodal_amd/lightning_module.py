"""Training module with the reference LightningModule contract (src/lightning_module.py:18-477).

`VAELightningModule(model, optimizer_config, scheduler_config, loss_config)` keeps the reference's
constructor, `forward`, `training_step(batch, batch_idx) -> loss`, `configure_optimizers`,
loss-type switch and `train/<key>` logging keys. Dispatch is by capability (what the model's forward
takes), not `isinstance` against the reference classes.

The optimizer hooks of the reference -- zero non-finite grads per tensor (on_before_optimizer_step,
:468-477), global-norm clipping (configure_gradient_clipping, :452-466) and Adam/AdamW (:390-408) --
run as ONE fused device-side kernel chain (`FusedAdam.step`) over a flat parameter buffer, in that
order and with the reference's per-tensor semantics. `fit_step` is the whole hot path of one
Lightning optimisation step: zero_grad -> training_step -> backward -> [all-reduce] -> fused step.
"""
from __future__ import annotations

import inspect
import os
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn as nn

from .disentangled import DisentangledConditionalVAE
from . import ops
from .losses import DisentangledVAELoss, LPIPSLoss, LPIPSWithDiscriminator, VAELoss
from .optim import Adam, AdamW, FlatParameters, FusedAdam
from .schedulers import get_scheduler

try:  # Lightning is optional: the module works stand-alone
    import lightning as L  # type: ignore
    _Base = L.LightningModule
except Exception:  # pragma: no cover - not installed in this image
    _Base = nn.Module


_CAPTURE_ERR_MARKS = ("captur", "graph", "not permitted when stream")


def _is_capture_error(e: BaseException) -> bool:
    """An error raised by recording the step (HIP stream capture / graph instantiation, or a collective the runtime
    cannot record), as opposed to an error of the step itself, which must propagate."""
    msg = str(e).lower()
    return any(m in msg for m in _CAPTURE_ERR_MARKS)


def _model_kind(model: nn.Module) -> str:
    if isinstance(model, DisentangledConditionalVAE) or hasattr(model, "modality_decoders"):
        return "indices"
    params = list(inspect.signature(model.forward).parameters)
    if len(params) >= 2 and params[1] in ("condition", "modality_indices"):
        return "condition"
    return "plain"



# The step's gradient zeroing (3.7 GB for c4's 927 M parameters) on a side stream, overlapped with the forward.
# Off under graph capture (the captured step keeps one stream). MVAE_ZERO_GRAD_SIDE=0: on the current stream.
ZERO_GRAD_SIDE = os.environ.get("MVAE_ZERO_GRAD_SIDE", "1") != "0"
_ZERO_SIDE = {}


def _zero_side(g):
    if not ZERO_GRAD_SIDE or g is None or not g.is_cuda or torch.cuda.is_current_stream_capturing() or \
            ops.PROFILE is not None:
        return None
    side = _ZERO_SIDE.get(g.device)
    if side is None:
        side = _ZERO_SIDE[g.device] = torch.cuda.Stream(g.device)
    return side

class VAELightningModule(_Base):
    def __init__(self, model: nn.Module, optimizer_config: Dict[str, Any], scheduler_config: Dict[str, Any],
                 loss_config: Dict[str, Any], gradient_clip_val: Optional[float] = None,
                 precision="32", **kwargs):
        """`precision` stands in for the Lightning Trainer's flag ("32" or "bf16-mixed"): it selects
        the GEMM arithmetic of the step (ops.set_precision)."""
        super().__init__()
        if precision not in ops._PRECISION:
            raise ValueError(f"precision {precision!r} is not supported on the MI355X path")
        self.precision = precision
        self.global_step_count = 0
        self.model = model
        self.optimizer_config = dict(optimizer_config)
        self.scheduler_config = dict(scheduler_config or {"type": "none"})
        self.loss_config = dict(loss_config)
        self.gradient_clip_val = gradient_clip_val
        self._kind = _model_kind(model)
        self._setup_loss()
        self.automatic_optimization = True
        self.flat: Optional[FlatParameters] = None
        self.optimizer: Optional[FusedAdam] = None
        self.scheduler = None
        self.logged: Dict[str, torch.Tensor] = {}
        self.process_group = None  # set by ddp.DataParallel
        self._usage = None

    def _setup_loss(self):
        t = self.loss_config.get("type", "vae")
        if t == "vae":
            self.criterion = VAELoss(recon_loss_type=self.loss_config.get("recon_loss_type", "mse"),
                                     kl_weight=self.loss_config.get("kl_weight", 1.0),
                                     recon_weight=self.loss_config.get("recon_weight", 1.0))
        elif t == "disentangled_vae":
            self.criterion = DisentangledVAELoss(
                recon_loss_type=self.loss_config.get("recon_loss_type", "mse"),
                kl_weight=self.loss_config.get("kl_weight", 1.0),
                recon_weight=self.loss_config.get("recon_weight", 1.0),
                separation_weight=self.loss_config.get("separation_weight", 0.1),
                contrastive_weight=self.loss_config.get("contrastive_weight", 0.05))
        elif t == "lpips":
            # the reference passes posteriors/priors kwargs LPIPSLoss cannot take (TypeError there);
            # here the objective is the perceptual distance alone
            self.criterion = LPIPSLoss(net=self.loss_config.get("lpips_net", "alex"),
                                       weights=self.loss_config.get("lpips_weights"),
                                       allow_synthetic=self.loss_config.get("allow_synthetic_lpips", False))
        elif t == "lpips_discriminator":
            self.criterion = LPIPSWithDiscriminator(
                discriminator_factor=self.loss_config.get("discriminator_factor", 1.0),
                perceptual_factor=self.loss_config.get("perceptual_factor", 1.0),
                kl_factor=self.loss_config.get("kl_factor", 1.0),
                discriminator_iter_start=self.loss_config.get("discriminator_iter_start", 50001),
                use_biomedclip_loss=self.loss_config.get("use_biomedclip_loss", False),
                discriminator_config=self.loss_config.get("discriminator", {}),
                lpips_weights=self.loss_config.get("lpips_weights"),
                allow_synthetic_lpips=self.loss_config.get("allow_synthetic_lpips", False),
                lpips_net=self.loss_config.get("lpips_net", "alex"))
        else:
            raise ValueError(f"Unknown/unsupported loss type on the MI355X path: {t}")
        self.use_discriminator = t == "lpips_discriminator"
        self.flat_d = None
        self.optimizer_d = None

    # ---------------------------------------------------------------------------------------
    def forward(self, x, condition=None, **kw):
        if self._kind != "plain" and condition is not None:
            return self.model(x, condition, **kw)
        return self.model(x, **kw)

    def log(self, name, value, **kwargs):  # Lightning-compatible signature; keeps device tensors
        self.logged[name] = value.detach() if torch.is_tensor(value) else value

    def training_step(self, batch, batch_idx: int, eps: Optional[torch.Tensor] = None):
        if len(batch) == 4:
            x, labels, modality, modality_indices = batch
        elif len(batch) == 3:
            x, labels, modality = batch
            modality_indices = None
        else:
            x, labels = batch[0], batch[1] if len(batch) > 1 else None
            modality, modality_indices = None, None
        kw = {} if eps is None else {"eps": eps}
        if self._kind == "indices" and modality is not None:
            if modality_indices is None:
                modality_indices = torch.argmax(modality, dim=1)
            self._usage = modality_indices
            outputs = self.model(x, modality_indices, **kw)
        elif self._kind == "condition" and modality is not None:
            outputs = self.model(x, modality, **kw)
        else:
            outputs = self.model(x, **kw)
        if isinstance(self.criterion, DisentangledVAELoss):
            loss_dict = self.criterion(outputs, x)
        elif isinstance(self.criterion, LPIPSWithDiscriminator):
            # generator objective (lightning_module.py:131-149); the discriminator step has nothing to
            # learn before discriminator_iter_start (its loss is a constant 0)
            loss_g, log = self.criterion(inputs=x, reconstructions=outputs["reconstruction"], latent=outputs["z"],
                                         posteriors=outputs["posterior"], optimizer_idx=0,
                                         global_step=self.global_step_count, split="train")
            for k, v in log.items():
                self.log(k, v)
            self._last_outputs = outputs
            return loss_g
        elif isinstance(self.criterion, LPIPSLoss):
            p = self.criterion(x, outputs["reconstruction"])
            loss_dict = {"loss": p, "p_loss": p}
        else:
            loss_dict = self.criterion(inputs=x, reconstructions=outputs["reconstruction"],
                                       posteriors=outputs["posterior"], priors=outputs["prior"])
        loss = loss_dict["loss"]
        if not isinstance(self.criterion, DisentangledVAELoss):  # (that total is already guarded by the criterion)
            loss = torch.where(torch.isfinite(loss), loss, 1e6)
        for k, v in loss_dict.items():
            self.log(f"train/{k}", v, prog_bar=True, logger=True, on_step=True, on_epoch=True)
        self._last_outputs = outputs
        return loss

    # ---------------------------------------------------------------------------------------
    def _forward_batch(self, batch, eps=None):
        if len(batch) == 4:
            x, labels, modality, modality_indices = batch
        elif len(batch) == 3:
            x, labels, modality = batch
            modality_indices = None
        else:
            x, modality, modality_indices = batch[0], None, None
        kw = {} if eps is None else {"eps": eps}
        if self._kind == "indices" and modality is not None:
            if modality_indices is None:
                modality_indices = torch.argmax(modality, dim=1)
            self._usage = modality_indices
            return x, self.model(x, modality_indices, **kw)
        if self._kind == "condition" and modality is not None:
            return x, self.model(x, modality, **kw)
        return x, self.model(x, **kw)

    def _eval_step(self, batch, split: str):
        """validation_step / test_step (lightning_module.py:220-386): reconstruction + KL metrics on
        the device (metrics.py), the objective for the `{split}/loss` monitor."""
        from .metrics import compute_kl_metrics_device, compute_reconstruction_metrics_device
        x, outputs = self._forward_batch(batch)
        rec = outputs["reconstruction"]
        mean = outputs["mean"] if "mean" in outputs else outputs["mu"]
        logvar = outputs["logvar"]
        for k, v in compute_reconstruction_metrics_device(x, rec).items():
            self.log(f"{split}/{k}", v, prog_bar=False, logger=True, on_epoch=True)
        for k, v in compute_kl_metrics_device(mean, logvar).items():
            self.log(f"{split}/{k}", v, prog_bar=False, logger=True, on_epoch=True)
        if isinstance(self.criterion, DisentangledVAELoss):
            loss = self.criterion(outputs, x)["loss"]
        elif isinstance(self.criterion, LPIPSWithDiscriminator):
            loss, _ = self.criterion(inputs=x, reconstructions=rec, latent=outputs["z"],
                                     posteriors=outputs["posterior"], optimizer_idx=0,
                                     global_step=self.global_step_count, split=split)
        elif isinstance(self.criterion, LPIPSLoss):
            loss = self.criterion(x, rec)
        else:
            loss = self.criterion(inputs=x, reconstructions=rec, posteriors=outputs["posterior"],
                                  priors=outputs["prior"])["loss"]
        loss = torch.where(torch.isfinite(loss), loss, 1e6)
        self.log(f"{split}/loss", loss, prog_bar=True, logger=True, on_epoch=True)
        return outputs

    def validation_step(self, batch, batch_idx: int):
        return self._eval_step(batch, "val")

    def test_step(self, batch, batch_idx: int):
        return self._eval_step(batch, "test")

    @torch.no_grad()
    def evaluate(self, batch, split: str = "val"):
        """Stand-alone validation of one batch (what Lightning's loop does around validation_step):
        eval mode, no autograd, the configured precision; returns the logged `{split}/*` tensors."""
        was_training = self.model.training
        self.model.eval()
        prev = ops.set_precision(self.precision)
        try:
            self._eval_step(batch, split)
        finally:
            ops.restore_math_mode(prev)
            self.model.train(was_training)
        return {k: v for k, v in self.logged.items() if k.startswith(f"{split}/")}

    # ---------------------------------------------------------------------------------------
    def teardown(self, stage: Optional[str] = None):
        """Lightning's end-of-fit / test hook: drop the captured step and free the converted weight copies (~2 x the
        conv weights' bytes, see ops.release_weight_buffers)."""
        self._graph = None
        ops.release_weight_buffers()

    def configure_optimizers(self):
        self._graph = None  # a captured step holds the previous optimizer's buffers and hyper-parameters
        ops.release_weight_buffers()  # (rebuilt by the next prepared step, for this optimizer's flat buffer)
        if self.flat is None:
            self.flat = FlatParameters(self.model)
        oc = self.optimizer_config
        betas = tuple(oc.get("betas", (0.9, 0.999)))
        if oc["type"] == "adam":
            opt = Adam(self.flat, lr=oc["lr"], betas=betas, weight_decay=oc.get("weight_decay", 0))
        elif oc["type"] == "adamw":
            opt = AdamW(self.flat, lr=oc["lr"], betas=betas, weight_decay=oc.get("weight_decay", 1e-4))
        else:
            raise ValueError(f"Unknown optimizer: {oc['type']}")
        opt.max_grad_norm = self.gradient_clip_val
        self.optimizer = opt
        if self.use_discriminator and self.optimizer_d is None:
            # lightning_module.py:427-433: Adam(lr * 0.5, betas (0.5, 0.999)) over the discriminator
            disc = self.criterion.discriminator.to(self.flat.device)
            self.flat_d = FlatParameters(disc)
            self.optimizer_d = Adam(self.flat_d, lr=oc["lr"] * 0.5, betas=(0.5, 0.999))
        self.scheduler = get_scheduler(opt, self.scheduler_config)
        if self.scheduler is not None:
            return [opt], [{"scheduler": self.scheduler, "monitor": "val/loss", "interval": "epoch",
                            "frequency": 1}]
        return [opt]

    def _used_mask(self) -> Optional[torch.Tensor]:
        if self._kind != "indices" or self._usage is None:
            return None
        f = self.flat
        if not hasattr(self, "_param_mod"):
            self._param_mod = torch.tensor([self.model.parameter_modality(n) for n in f.names],
                                           dtype=torch.long, device=f.device)
        present = self.model.modality_presence(self._usage.to(f.device))
        if self.process_group is not None:
            # a head used on ANY rank receives the averaged gradient on every rank: the mask (clip norm, Adam
            # update and step count) must be the same everywhere or the replicas drift apart
            present = self.process_group.any_across_ranks(present)
        pm = self._param_mod
        used = (pm == -1) | ((pm >= 0) & present[pm.clamp_min(0)])
        return used.to(torch.int32)

    def fit_step_graphed(self, batch, batch_idx: int = 0, eps: Optional[torch.Tensor] = None) -> torch.Tensor:
        """fit_step replayed from captured HIP graphs: the optimisation step (forward, loss, backward, gradient
        exchange, non-finite zeroing, clip, Adam/AdamW) is captured once and then replayed, so the host issues one
        or two graph launches per step instead of ~800 kernel launches (the small 28x28 configs are host-bound
        otherwise). Same arithmetic and the same kernels as fit_step; dropout masks stay fresh per step through the
        device dropout salt the graph advances (ops.dropout_salt); the reparameterisation noise comes from torch's
        graph-safe generator. Requires static batch shapes (the batch is copied into the graph's input buffers), a
        constant learning rate (a change re-captures), automatic optimisation, and at least one eager fit_step
        before the first call (library / allocator / communicator state is built eagerly).

        Data-parallel (ddp.DataParallel attached), two capture modes:
          "whole" (RCCL, the "nccl" backend): ONE graph holding the step AND its bucketed gradient all-reduces,
                  launched from the backward's readiness hooks exactly as in the eager step (RCCL collectives are
                  capturable: they are kernels on RCCL's stream, ordered by events the capture records)
          "split" (any other backend -- gloo cannot be captured -- or MVAE_DP_CAPTURE=split): graph 1 = forward +
                  backward, then the exchange eagerly (synchronous bucketed all-reduce + the per-modality usage OR),
                  graph 2 = the optimizer step reading the exchanged gradients and the usage mask from static
                  buffers."""
        if self.use_discriminator:
            raise RuntimeError("fit_step_graphed: adversarial steps run eagerly (fit_step)")
        if self.optimizer is None or self.global_step_count == 0:
            raise RuntimeError("fit_step_graphed: run at least one eager fit_step first")
        ins = list(batch) + ([eps] if eps is not None else [])
        mode = self._dp_capture_mode()
        # everything the captured launches freeze as host values: shapes, the optimizer's hyper-parameters
        # (lr, betas, eps, weight decay), clip norm and gradient scale, the GEMM arithmetic, the exchange mode
        opt = self.optimizer
        hyper = tuple(sorted((k, tuple(v) if isinstance(v, (list, tuple)) else v)
                             for k, v in opt.param_groups[0].items() if k != "params"))
        key = (tuple((tuple(t.shape), t.dtype, t.device) for t in ins), eps is not None, hyper,
               opt.max_grad_norm, getattr(opt, "grad_scale", None), id(opt), id(self.flat), self.precision, mode,
               id(self.process_group))
        if getattr(self, "_graph_failed", None) == key:  # this step's capture failed before: eager steps
            return self.fit_step(batch, batch_idx, eps=eps)
        g = getattr(self, "_graph", None)
        if g is None or g["key"] != key:
            err = None
            try:
                g = self._capture_step(ins, len(batch), batch_idx, key, mode)
            except RuntimeError as e:
                if not _is_capture_error(e):
                    raise
                err, g = e, None
            # the fall-back decision is collective: a rank that replays its graphs while a peer runs the eager exchange
            # would issue a different collective sequence (every rank falls back when any capture failed)
            pg = self.process_group
            if pg is not None and getattr(pg, "world", 1) > 1:
                failed = torch.tensor([err is not None], device=ins[0].device)
                if bool(pg.any_across_ranks(failed)[0]) and err is None:
                    err = RuntimeError("a peer rank's step capture failed")
            if err is not None:  # (e.g. a collective the runtime cannot record): eager steps from here on
                import warnings
                warnings.warn(f"fit_step_graphed: step capture failed ({err}); running eager steps")
                self._graph = None
                self._graph_failed = key
                torch.cuda.synchronize(ins[0].device)
                return self.fit_step(batch, batch_idx, eps=eps)
        for dst, src in zip(g["inputs"], ins):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
        if mode == "split":
            g["graph"].replay()  # forward + backward
            prev = ops.set_precision(self.precision)
            try:
                self.process_group.allreduce_gradients(self.flat)
                used = self._used_mask()
                if used is not None:
                    g["used"].copy_(used)
            finally:
                ops.restore_math_mode(prev)
            g["graph_opt"].replay()
        else:
            g["graph"].replay()
        self.global_step_count += 1
        return g["loss"]

    def _dp_capture_mode(self) -> str:
        """"single" (no data parallelism), "whole" or "split" (see fit_step_graphed)."""
        pg = self.process_group
        if pg is None or getattr(pg, "world", 1) == 1:
            return "single"
        # "whole" (the bucket all-reduces recorded inside the step graph) is opt-in: RCCL capture has not run on this
        # build's 1-GPU boxes, while "split" is bitwise-tested against the eager DP step (tests/test_gpu_ddp.py)
        forced = os.environ.get("MVAE_DP_CAPTURE")
        if forced in ("whole", "split"):
            return forced
        return "split"

    def _capture_step(self, ins, nb, batch_idx, key, mode="single"):
        dev = ins[0].device
        static = [t.clone() for t in ins]
        salt = ops.dropout_salt(dev)
        self._last_outputs = None  # no autograd graph of an earlier step may outlive into the capture
        ops.refresh_weight_tables(self.flat.data)  # (the batched weight re-layout table is uploaded outside the capture)
        torch.cuda.synchronize(dev)
        self._graph = None  # release an outdated graph (and the arena buffers it pinned) before recording
        graph = torch.cuda.CUDAGraph()
        step0 = self.global_step_count
        pinned = ops.ARENA.pinning = []  # the graph keeps every scratch buffer it bakes in (ops._Arena)
        eps_in = static[nb] if len(static) > nb else None
        rec = dict(inputs=static, salt=salt, key=key, arena=pinned)
        try:
            if mode != "split":
                with torch.cuda.graph(graph):  # recorded, not executed: capturing performs no optimisation step
                    salt.add_(1)
                    loss = self.fit_step(static[:nb], batch_idx, eps=eps_in)
            else:
                graph_opt = torch.cuda.CUDAGraph()
                used = torch.ones(len(self.flat.params), dtype=torch.int32, device=dev)
                prev = ops.set_precision(self.precision)
                try:
                    with torch.cuda.graph(graph):
                        salt.add_(1)
                        loss = self._forward_backward(static[:nb], batch_idx, eps_in, exchange=False)
                    with torch.cuda.graph(graph_opt, pool=graph.pool()):
                        self._optimizer_phase(used=used if self._kind == "indices" else None, exchange=False)
                finally:
                    ops.flat_weights_stale()
                    ops.restore_math_mode(prev)
                loss = loss.detach()
                rec.update(graph_opt=graph_opt, used=used)
        finally:
            ops.ARENA.pinning = None
            # (recording executes no step: the host-side counter the recorded fit_step advanced -- it drives the LR
            # schedule and the discriminator start -- is restored whether or not the capture completed; the optimizer's
            # step counts live on the device and were not touched)
            self.global_step_count = step0
        rec.update(graph=graph, loss=loss)
        self._graph = rec
        return self._graph

    def _adversarial_fit_step(self, batch, eps=None) -> torch.Tensor:
        """The reference's manual-optimisation step (lightning_module.py:131-175) once the
        discriminator is active: generator step (VAE optimizer), then discriminator step. As under
        Lightning's manual optimisation, no automatic gradient clipping; global_step counts both
        optimizer steps."""
        disc = self.criterion.discriminator
        self.model.train()
        disc.train()
        x, outputs = self._forward_batch(batch, eps)
        rec = outputs["reconstruction"]
        loss_g, log_g = self.criterion(inputs=x, reconstructions=rec, latent=outputs["z"],
                                       posteriors=outputs["posterior"], optimizer_idx=0,
                                       global_step=self.global_step_count, last_layer=self.model.decoder.conv_out,
                                       split="train")
        self.optimizer.zero_grad()
        if self.process_group is not None:
            self.process_group.begin_backward()
        loss_g.backward()
        if self.process_group is not None:
            self.process_group.allreduce_gradients(self.flat)
        clip = self.optimizer.max_grad_norm
        self.optimizer.max_grad_norm = None
        try:
            self.optimizer.step(used=self._used_mask())
        finally:
            self.optimizer.max_grad_norm = clip
        loss_d, log_d = self.criterion(inputs=x, reconstructions=rec.detach(), latent=outputs["z"].detach(),
                                       posteriors=outputs["posterior"], optimizer_idx=1,
                                       global_step=self.global_step_count, last_layer=None, split="train")
        self.optimizer_d.zero_grad()
        loss_d.backward()
        if self.process_group is not None:
            self.process_group.allreduce_flat(self.flat_d)
        self.optimizer_d.step()
        for k, v in {**log_g, **log_d}.items():
            self.log(k, v)
        self._last_outputs = outputs
        self.global_step_count += 2
        return loss_g

    def _forward_backward(self, batch, batch_idx, eps, exchange: bool = True) -> torch.Tensor:
        """fit_step's first phase: gradients of this rank's batch in the flat buffer (exchange: the data-parallel
        bucket all-reduces launched from the backward's readiness hooks)."""
        self.model.train()
        side = _zero_side(self.flat.grad)
        if side is not None:
            # the flat gradient is zeroed on a side stream, concurrent with the forward (which never touches it), and
            # joined before the backward's first gradient write
            side.wait_stream(torch.cuda.current_stream(self.flat.grad.device))
            with torch.cuda.stream(side):
                self.optimizer.zero_grad()
        else:
            self.optimizer.zero_grad()
        ops.prep_flat_weights(self.flat.data)  # every conv weight in the GEMM format, one launch
        loss = self.training_step(batch, batch_idx, eps=eps)
        if side is not None:
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(side)
        if exchange and self.process_group is not None:
            self.process_group.begin_backward()
        loss.backward()
        return loss

    def _optimizer_phase(self, used: Optional[torch.Tensor] = None, exchange: bool = True):
        """fit_step's second phase: finish the gradient exchange, then the fused optimizer step (used: the usage mask
        buffer the split graph capture reads; default: computed here)."""
        if exchange and self.process_group is not None:
            self.process_group.allreduce_gradients(self.flat)
        ops.flat_weights_stale()
        self.optimizer.step(used=self._used_mask() if used is None else used)

    def fit_step(self, batch, batch_idx: int = 0, eps: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One optimisation step of Lightning's loop, fused (automatic optimisation, or the
        reference's manual generator/discriminator pair once the discriminator is active)."""
        if self.optimizer is None:
            self.configure_optimizers()
        if self.use_discriminator and self.global_step_count >= self.criterion.discriminator_iter_start:
            prev = ops.set_precision(self.precision)
            try:
                return self._adversarial_fit_step(batch, eps)
            finally:
                ops.restore_math_mode(prev)
        self.model.train()
        prev = ops.set_precision(self.precision)
        try:
            loss = self._forward_backward(batch, batch_idx, eps)
            self._optimizer_phase()
        finally:
            ops.flat_weights_stale()
            ops.restore_math_mode(prev)
        self.global_step_count += 1
        # hand back values, not the step's autograd graph: a graph kept alive past the step pins its AccumulateGrad
        # nodes to this step's stream, which breaks the capture of the next step (fit_step_graphed)
        if isinstance(self._last_outputs, dict):
            self._last_outputs = {k: v.detach() for k, v in self._last_outputs.items() if torch.is_tensor(v)}
        return loss.detach()
