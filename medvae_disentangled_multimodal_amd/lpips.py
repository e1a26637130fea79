"""LPIPS perceptual distance (net="alex" or "vgg") on the MI355X kernels.

Restates the third-party `lpips` 0.1.4 package (pinned by the reference, uv.lock:1585) that
`LPIPSLoss` (src/losses/vae_losses.py:67-94) wraps, with torchvision's feature stacks:

  alex (the reference's default): conv1 11x11/4 p2 -> ReLU [relu1] -> maxpool 3/2 -> conv2 5x5 p2
      -> ReLU [relu2] -> maxpool 3/2 -> conv3 -> ReLU [relu3] -> conv4 -> ReLU [relu4] -> conv5 -> ReLU [relu5]
  vgg (BASELINE config 5): VGG16 conv3x3 stacks (2,2,3,3,3 convs of 64,128,256,512,512 channels)
      with 2x2/2 max pools between, taps relu1_2, relu2_2, relu3_3, relu4_3, relu5_3
    x -> ScalingLayer ((x - shift) / scale) -> taps f_l
    d(x0, x1) = sum_l mean_{h,w} sum_c w_l[c] * (f0/|f0| - f1/|f1|)^2     (|f| + 1e-10 per pixel)

The pretrained backbone + linear-layer weights cannot be fetched offline. `LPIPS` loads them from a
state dict in the lpips package's own naming (`net.slice1.0.weight`, ..., `lin0.model.1.weight`)
when given one; otherwise it refuses unless `allow_synthetic=True`, which builds deterministic
synthetic weights (benchmarks and parity tests only -- parity against the real package is
unpinned). The linear layers' dropout is inactive (lpips builds the network in
eval mode). Weights are frozen: only the gradient w.r.t. the second (reconstruction) input flows.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from . import ops
from .encoder_decoder import Conv2d

ALEX_CHANNELS = (64, 192, 384, 256, 256)
VGG_CHANNELS = (64, 128, 256, 512, 512)
# (slice, index inside torchvision's `features`) of every conv, per lpips.pretrained_networks slice
_ALEX_CONVS = ((1, 0), (2, 3), (3, 6), (4, 8), (5, 10))
_VGG_CONVS = ((1, 0), (1, 2), (2, 5), (2, 7), (3, 10), (3, 12), (3, 14), (4, 17), (4, 19), (4, 21),
              (5, 24), (5, 26), (5, 28))
_VGG_CFG = ((3, 64), (64, 64), (64, 128), (128, 128), (128, 256), (256, 256), (256, 256), (256, 512), (512, 512),
            (512, 512), (512, 512), (512, 512), (512, 512))
_SHIFT = (-0.030, -0.088, -0.188)
_SCALE = (0.458, 0.448, 0.450)


class LPIPS(nn.Module):
    def __init__(self, net: str = "alex", weights: Optional[Dict[str, torch.Tensor]] = None,
                 allow_synthetic: bool = False, seed: int = 0):
        super().__init__()
        if net not in ("alex", "vgg"):
            raise NotImplementedError(f"LPIPS net={net!r}: 'alex' (reference default) and 'vgg' are built")
        self.net = net
        if net == "alex":
            self.conv1 = Conv2d(3, 64, 11, stride=4, padding=2)
            self.conv2 = Conv2d(64, 192, 5, padding=2)
            self.conv3 = Conv2d(192, 384, 3, padding=1)
            self.conv4 = Conv2d(384, 256, 3, padding=1)
            self.conv5 = Conv2d(256, 256, 3, padding=1)
            chans = ALEX_CHANNELS
        else:
            self.vgg = nn.ModuleList([Conv2d(ci, co, 3, padding=1) for ci, co in _VGG_CFG])
            chans = VGG_CHANNELS
        self.lins = nn.ParameterList([nn.Parameter(torch.empty(c)) for c in chans])
        self.register_buffer("shift", torch.tensor(_SHIFT, dtype=torch.float32))
        self.register_buffer("scale", torch.tensor(_SCALE, dtype=torch.float32))
        self.register_buffer("inv_scale", 1.0 / self.scale, persistent=False)
        # state dicts use the lpips package's names (LPIPS(net=...).state_dict()), so a reference
        # checkpoint's `criterion.perceptual_loss.lpips.*` keys load and written checkpoints match them
        self._register_state_dict_hook(LPIPS._to_package_names)
        self._register_load_state_dict_pre_hook(LPIPS._from_package_names, with_module=True)
        self.register_load_state_dict_post_hook(LPIPS._refresh_inv_scale)
        if weights is None:
            path = os.environ.get("MVAE_LPIPS_WEIGHTS")
            if path:
                weights = load_weight_file(path)
        if weights is not None:
            self.load_lpips_state_dict(weights)
            self.pretrained = True
        elif allow_synthetic:
            self._synthetic(seed)
            self.pretrained = False
        else:
            raise RuntimeError("LPIPS needs the pretrained lpips/AlexNet weights: pass `weights=` (lpips state "
                               "dict) or set MVAE_LPIPS_WEIGHTS; allow_synthetic=True builds deterministic "
                               "synthetic weights for benchmarking only")
        for p in self.parameters():
            p.requires_grad_(False)

    def convs(self) -> List[Conv2d]:
        if self.net == "vgg":
            return list(self.vgg)
        return [self.conv1, self.conv2, self.conv3, self.conv4, self.conv5]

    @torch.no_grad()
    def _synthetic(self, seed: int):
        g = torch.Generator().manual_seed(int(seed))
        for conv in self.convs():
            fan_in = conv.weight[0].numel()
            bound = (6.0 / fan_in) ** 0.5  # He-uniform: keeps ReLU activations O(1) through the stack
            conv.weight.copy_((torch.rand(conv.weight.shape, generator=g) * 2 - 1) * bound)
            conv.bias.copy_((torch.rand(conv.bias.shape, generator=g) * 2 - 1) * 0.1)
        for lin in self.lins:
            c = lin.numel()
            lin.copy_(torch.rand(c, generator=g) / c)  # non-negative, like the trained linear layers

    def _conv_names(self):
        """(internal prefix, lpips-package prefix) of every conv: `conv1` <-> `net.slice1.0`, `vgg.3` <->
        `net.slice2.7` (lpips.pretrained_networks slices over torchvision's `features` indices)."""
        names = _ALEX_CONVS if self.net == "alex" else _VGG_CONVS
        internal = [f"conv{i + 1}" for i in range(5)] if self.net == "alex" else [f"vgg.{i}" for i in range(13)]
        return [(a, f"net.slice{sl}.{idx}") for a, (sl, idx) in zip(internal, names)]

    @staticmethod
    def _to_package_names(module, state_dict, prefix, local_metadata):
        for ours, theirs in module._conv_names():
            for t in ("weight", "bias"):
                state_dict[f"{prefix}{theirs}.{t}"] = state_dict.pop(f"{prefix}{ours}.{t}")
        for k in range(len(module.lins)):
            w = state_dict.pop(f"{prefix}lins.{k}").reshape(1, -1, 1, 1)
            state_dict[f"{prefix}lin{k}.model.1.weight"] = w
            state_dict[f"{prefix}lins.{k}.model.1.weight"] = w  # lpips registers its lin layers twice
        for b in ("shift", "scale"):
            state_dict[f"{prefix}scaling_layer.{b}"] = state_dict.pop(f"{prefix}{b}").reshape(1, 3, 1, 1)
        return state_dict

    @staticmethod
    def _from_package_names(module, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                            error_msgs):
        """Translate lpips-package keys to the module's own (both spellings load)."""
        for ours, theirs in module._conv_names():
            for t in ("weight", "bias"):
                if f"{prefix}{theirs}.{t}" in state_dict:
                    state_dict[f"{prefix}{ours}.{t}"] = state_dict.pop(f"{prefix}{theirs}.{t}")
        for k in range(len(module.lins)):
            dup = state_dict.pop(f"{prefix}lins.{k}.model.1.weight", None)
            w = state_dict.pop(f"{prefix}lin{k}.model.1.weight", dup)
            if w is not None:
                state_dict[f"{prefix}lins.{k}"] = w.reshape(-1)
        for b in ("shift", "scale"):
            if f"{prefix}scaling_layer.{b}" in state_dict:
                state_dict[f"{prefix}{b}"] = state_dict.pop(f"{prefix}scaling_layer.{b}").reshape(-1)
        if f"{prefix}inv_scale" in state_dict and f"{prefix}scale" not in state_dict:  # round-2 checkpoints
            state_dict[f"{prefix}scale"] = 1.0 / state_dict.pop(f"{prefix}inv_scale")
        state_dict.pop(f"{prefix}inv_scale", None)

    @staticmethod
    def _refresh_inv_scale(module, incompatible_keys):
        with torch.no_grad():
            module.inv_scale.copy_(1.0 / module.scale)

    def internal_weights(self) -> Dict[str, torch.Tensor]:
        """Weights under the module's own names (the oracle's lpips_alex / lpips_vgg take these)."""
        out = {f"{ours}.{t}": getattr(c, t) for (ours, _), c in zip(self._conv_names(), self.convs())
               for t in ("weight", "bias")}
        out.update({f"lins.{k}": w for k, w in enumerate(self.lins)})
        return out

    @torch.no_grad()
    def load_lpips_state_dict(self, sd: Dict[str, torch.Tensor]):
        """Load weights named as in the lpips package (LPIPS(net=...).state_dict()); the ScalingLayer
        buffers are optional (lpips hard-codes them)."""
        sd = dict(sd)
        for b in ("shift", "scale"):
            sd.setdefault(f"scaling_layer.{b}", getattr(self, b).detach().clone().view(1, 3, 1, 1))
        self.load_state_dict(sd, strict=False)
        missing = [f"{t}.{x}" for _, t in self._conv_names() for x in ("weight", "bias") if f"{t}.{x}" not in sd]
        missing += [f"lin{k}.model.1.weight" for k in range(len(self.lins))
                    if f"lin{k}.model.1.weight" not in sd and f"lins.{k}.model.1.weight" not in sd]
        if missing:
            raise KeyError(f"lpips weights missing: {missing[:4]}")

    def features(self, x: torch.Tensor) -> List[torch.Tensor]:
        if self.net == "vgg":
            taps, h, i = [], x, 0
            for block, n in enumerate((2, 2, 3, 3, 3)):
                if block:
                    h = ops.max_pool(h, 2, 2)
                for _ in range(n):
                    h = ops.relu(self.vgg[i](h))
                    i += 1
                taps.append(h)
            return taps
        h = ops.relu(self.conv1(x))
        f1 = h
        h = ops.relu(self.conv2(ops.max_pool3s2(h)))
        f2 = h
        h = ops.relu(self.conv3(ops.max_pool3s2(h)))
        f3 = h
        h = ops.relu(self.conv4(h))
        f4 = h
        h = ops.relu(self.conv5(h))
        return [f1, f2, f3, f4, h]

    def forward(self, in0: torch.Tensor, in1: torch.Tensor, pre_a: float = 1.0, pre_b: float = 0.0) -> torch.Tensor:
        """lpips.LPIPS.forward(in0, in1) -> [B,1,1,1]; `pre_a*x + pre_b` is applied before the
        ScalingLayer (LPIPSLoss passes x*2-1)."""
        x0 = ops.lpips_scale(in0, self.shift, self.inv_scale, pre_a, pre_b)
        x1 = ops.lpips_scale(in1, self.shift, self.inv_scale, pre_a, pre_b)
        if not in0.requires_grad:
            with torch.no_grad():
                f0 = self.features(x0)
        else:
            f0 = self.features(x0)
        f1 = self.features(x1)
        score = None
        for a, b, w in zip(f0, f1, self.lins):
            d = ops.lpips_dist(a, b, w)
            score = d if score is None else score + d
        return score.view(-1, 1, 1, 1)


def load_weight_file(path: str) -> Dict[str, torch.Tensor]:
    """lpips weights from safetensors or a torch file (weights_only: nothing in the file executes)."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)
