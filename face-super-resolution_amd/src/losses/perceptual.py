"""Perceptual loss with VGG19 features (reference src/losses/perceptual.py:13-169), on the
HIP path (src/hip/vgg.py).

Same classes, constructor arguments and module tree as the reference: `VGGFeatureExtractor`
keeps `features` (an nn.Sequential of vgg19.features[:max_idx + 1], state-dict keys
'features.{i}.weight'), the `mean` / `std` buffers and a train() that stays in eval mode;
`PerceptualLoss` keeps `feature_extractor`, `layers`, `weights` and `criterion`.

Weights.  The reference loads torchvision's ImageNet VGG19 (perceptual.py:48), a network
download.  Here `vgg_weights` (or the FEN_VGG19_WEIGHTS environment variable) names a local
torchvision-format state dict (.pth read with torch.load(weights_only=True), or
.safetensors); without one the extractor is randomly initialised like torchvision's VGG
(kaiming-normal fan_out, zero bias) and a warning says so -- fine for benchmarks, not for
training a real model.

Compute: the frozen extractor, the loss and the gradient w.r.t. `pred` run as one recorded
HIP program per call (bf16 by default).  Only conv feature layers are wired (conv1_2 ...
conv5_4); gradients flow to `pred` only (the target is data).  There is no CPU path.
"""
from __future__ import annotations

import os
import warnings
from typing import Dict, List, Optional, Union

import torch
import torch.nn as nn

from ..hip.vgg import LAYER_MAP, VGG19_CFG, VGGPerceptual, feature_indices

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32}


def _build_features(max_idx: int) -> nn.Sequential:
    mods, cin = [], 3
    for v in VGG19_CFG:
        if v == "M":
            mods.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            mods += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*mods[:max_idx + 1])


def _load_state(src) -> Dict[str, torch.Tensor]:
    if isinstance(src, dict):
        return src
    path = str(src)
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


class VGGFeatureExtractor(nn.Module):
    """VGG19 feature extractor (perceptual.py:13-101)."""

    LAYER_MAP = LAYER_MAP

    def __init__(self, layers: List[str] = ['conv3_4', 'conv4_4'], normalize: bool = True,
                 requires_grad: bool = False, vgg_weights: Union[str, dict, None] = None,
                 precision: str = "bf16"):
        super().__init__()
        self.layers = list(layers)
        self.normalize = normalize
        max_idx = max(self.LAYER_MAP.get(layer, 0) for layer in self.layers)
        self.features = _build_features(max_idx)
        self.layer_indices = [self.LAYER_MAP[layer] for layer in self.layers]
        src = vgg_weights if vgg_weights is not None else os.environ.get("FEN_VGG19_WEIGHTS")
        if src is not None:
            sd = _load_state(src)
            mine = {k: v for k, v in sd.items() if k.startswith("features.")
                    and int(k.split(".")[1]) <= max_idx}
            self.load_state_dict(mine, strict=False)
        else:
            warnings.warn("VGG19 ImageNet weights are not available offline; the perceptual loss uses randomly "
                          "initialised VGG19 features (pass vgg_weights= or set FEN_VGG19_WEIGHTS)")
            g = torch.Generator().manual_seed(0)
            for m in self.features:
                if isinstance(m, nn.Conv2d):
                    std = (2.0 / (m.out_channels * 9)) ** 0.5
                    with torch.no_grad():
                        m.weight.copy_(torch.randn(m.weight.shape, generator=g) * std)
                        m.bias.zero_()
        if not requires_grad:
            for p in self.features.parameters():
                p.requires_grad = False
            self.features.eval()
        self.register_buffer('mean', torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1))
        self.register_buffer('std', torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1))
        self.compute_dtype = _DTYPES[precision]
        self._hip = None

    def train(self, mode: bool = True):
        """Stays in eval mode (perceptual.py:74-77)."""
        return self

    def hip_program(self, layer_weights: Optional[Dict[str, float]] = None, criterion: str = "l1",
                    layers: Optional[List[str]] = None) -> VGGPerceptual:
        """The HIP builder over this module's (frozen) weights; re-packed when they change."""
        dev = self.features[0].weight.device
        if dev.type != "cuda":
            raise RuntimeError("the HIP perceptual loss runs on a ROCm GPU tensor (got CPU); there is no CPU path")
        layers = list(layers or self.layers)
        params = {f"features.{i}.{n}": getattr(m, n) for i, m in enumerate(self.features)
                  if isinstance(m, nn.Conv2d) for n in ("weight", "bias")}
        key = (dev, tuple(layers), criterion, tuple(sorted((layer_weights or {}).items())),
               tuple(p._version for p in params.values()), self.normalize)
        if self._hip is None or self._hip[0] != key:
            from ..hip.program import Ctx
            ctx = Ctx(self.compute_dtype, dev)
            prog = VGGPerceptual(ctx, {k: v.detach() for k, v in params.items()}, layers=layers,
                                 weights=layer_weights, criterion=criterion, normalize=self.normalize)
            self._hip = (key, prog)
        return self._hip[1]

    def forward(self, x: torch.Tensor) -> Dict[str, torch.Tensor]:
        """{layer name: NCHW fp32 feature} of x (B,3,H,W) in [0,1] (perceptual.py:79-101)."""
        from ..hip.program import Ctx
        feature_indices(self.layers)          # conv layers only on the HIP path
        prog = self.hip_program()
        ctx = Ctx(self.compute_dtype, x.device)
        _, feats = prog.forward(x.detach().float().contiguous(), ctx)
        return {name: feats[self.LAYER_MAP[name]].float().permute(0, 3, 1, 2).contiguous()
                for name in self.layers}


class _PerceptualFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, pred, target, module):
        from ..hip.program import Ctx
        fe = module.feature_extractor
        prog = fe.hip_program(module.weights, module.criterion_name, module.layers)
        B, _, H, W = pred.shape
        x2 = torch.cat([pred.detach().float(), target.detach().float()]).contiguous()
        ctx = Ctx(fe.compute_dtype, pred.device)
        loss = torch.zeros(1, device=pred.device)
        dpred = (torch.zeros(B, H, W, 16, device=pred.device, dtype=fe.compute_dtype)
                 if pred.requires_grad else None)
        prog.build(x2, loss, dpred, ctx=ctx)
        fctx.dpred = dpred
        return loss[0].clone()

    @staticmethod
    def backward(fctx, g):
        d = fctx.dpred[..., :3].float().permute(0, 3, 1, 2).contiguous()
        return d * g, None, None


class PerceptualLoss(nn.Module):
    """Weighted L1 / L2 distance between VGG19 features of pred and target
    (perceptual.py:104-169)."""

    def __init__(self, layers: List[str] = ['conv3_4', 'conv4_4'], weights: Optional[Dict[str, float]] = None,
                 criterion: str = 'l1', normalize: bool = True, vgg_weights: Union[str, dict, None] = None,
                 precision: str = "bf16"):
        super().__init__()
        self.feature_extractor = VGGFeatureExtractor(layers=layers, normalize=normalize, requires_grad=False,
                                                     vgg_weights=vgg_weights, precision=precision)
        self.layers = list(layers)
        self.weights = weights or {layer: 1.0 for layer in layers}
        if criterion == 'l1':
            self.criterion = nn.L1Loss()
        elif criterion == 'l2':
            self.criterion = nn.MSELoss()
        else:
            raise ValueError(f"Unknown criterion: {criterion}")
        self.criterion_name = criterion

    def forward(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if not pred.is_cuda:
            raise RuntimeError("the HIP perceptual loss runs on a ROCm GPU tensor (got CPU); there is no CPU path")
        return _PerceptualFn.apply(pred, target, self)

    def fused_spec(self, weight: float) -> dict:
        """The FENEngine `perceptual=` dict for this loss scaled by `weight`."""
        fe = self.feature_extractor
        params = {f"features.{i}.{n}": getattr(m, n).detach() for i, m in enumerate(fe.features)
                  if isinstance(m, nn.Conv2d) for n in ("weight", "bias")}
        return dict(weight=weight, layers=self.layers, criterion=self.criterion_name, normalize=fe.normalize,
                    params=params, layer_weights=self.weights)


__all__ = ["VGGFeatureExtractor", "PerceptualLoss"]
