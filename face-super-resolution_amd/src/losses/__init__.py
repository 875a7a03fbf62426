"""Loss surface of the reference (src/losses/combined.py:16-302) restricted to the hot path.

The stage-1 generator step's loss is L1 (combined.py:38-47) + the VGG19 perceptual term
(perceptual.py, stage1_psnr_config.yaml:40-50).  L1 is fused into the conv_last epilogue
(sign(sr-hr)/N written by the kernel, fen_conv_desc.hr); the perceptual term runs on the
HIP VGG path (src/hip/vgg.py) and its gradient joins L1's in the same dL/dsr buffer; the
stage-2 SSIM term (ssim_loss.py:174-226) runs on the HIP SSIM kernel (src/losses/ssim.py,
fused into the engine's dL/dsr as well).  MS-SSIM / L2 / Charbonnier are outside the built
path: asking for them raises instead of silently training something else.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LossConfig:
    l1_weight: float = 1.0
    l2_weight: float = 0.0
    perceptual_weight: float = 0.01
    ssim_weight: float = 0.1
    ms_ssim_weight: float = 0.0
    use_charbonnier: bool = False
    charbonnier_eps: float = 1e-3
    perceptual_layers: list = field(default_factory=lambda: ["conv3_4", "conv4_4"])
    ssim_window_size: int = 11
    vgg_weights: Optional[str] = None      # local torchvision VGG19 state dict (no download offline)


class _L1(torch.autograd.Function):
    """mean |pred - target| on fen_l1_loss (fixed-order partial sums, fen_colsum); the gradient
    sign(pred - target) / n x the upstream gradient, read on the device.  No gradient to target
    (the reference's HR images never require one; asking for it raises)."""

    @staticmethod
    def forward(fctx, pred, target):
        from ..hip import lib as L
        from ..hip.program import ptr
        if target.requires_grad:
            raise NotImplementedError("HIP L1Loss: no gradient with respect to the target")
        p, t = pred.detach().float().contiguous(), target.detach().float().contiguous()
        lib, s = L.load(), torch.cuda.current_stream().cuda_stream
        nparts = lib.fen_feat_loss_parts()
        part = torch.empty(nparts, device=p.device)
        loss = torch.empty((), device=p.device)
        L.check(lib.fen_l1_loss(p.numel(), ptr(p), ptr(t), None, 0.0, None, ptr(part), s), "l1_loss")
        L.check(lib.fen_colsum(nparts, 1, ptr(part), 1.0 / p.numel(), ptr(loss), 0, s), "l1_loss sum")
        fctx.save_for_backward(p, t)
        fctx.dtype = pred.dtype
        return loss

    @staticmethod
    def backward(fctx, gout):
        from ..hip import lib as L
        from ..hip.program import ptr
        p, t = fctx.saved_tensors
        lib, s = L.load(), torch.cuda.current_stream().cuda_stream
        g = torch.empty_like(p)
        part = torch.empty(lib.fen_feat_loss_parts(), device=p.device)
        gout = gout.detach().float().contiguous()
        L.check(lib.fen_l1_loss(p.numel(), ptr(p), ptr(t), ptr(gout), 1.0 / p.numel(), ptr(g), ptr(part), s),
                "l1_loss grad")
        return g.to(fctx.dtype), None


class L1Loss(nn.Module):
    """mean |pred - target| (combined.py:38-47), on the HIP kernel for GPU tensors ('mean'; the
    other reductions and CPU tensors through torch, which the HIP path never hands it)."""

    def __init__(self, reduction: str = "mean"):
        super().__init__()
        self.reduction = reduction

    def forward(self, pred, target):
        if self.reduction == "mean" and pred.is_cuda and pred.shape == target.shape:
            return _L1.apply(pred, target)
        return F.l1_loss(pred, target, reduction=self.reduction)


class CombinedLoss(nn.Module):
    """Weighted loss with component tracking (combined.py:80-203): L1 and perceptual terms.
    `fused_l1_weight` / `fused_perceptual` tell the Trainer it may use the fused HIP step."""

    def __init__(self, config: LossConfig):
        super().__init__()
        self.config = config
        if config.ms_ssim_weight or config.l2_weight or config.use_charbonnier:
            raise NotImplementedError(
                "only the L1, perceptual and SSIM terms are built on the MI355X path (MS-SSIM / L2 / Charbonnier "
                "are not); set ms_ssim_weight=0, l2_weight=0, use_charbonnier=False")
        self.l1 = L1Loss()
        self.perceptual = None
        if config.perceptual_weight > 0:
            from .perceptual import PerceptualLoss
            self.perceptual = PerceptualLoss(layers=list(config.perceptual_layers), vgg_weights=config.vgg_weights)
        self.ssim = None
        if config.ssim_weight > 0:
            from .ssim import SSIMLoss
            self.ssim = SSIMLoss(window_size=config.ssim_window_size)

    @property
    def fused_l1_weight(self) -> float:
        return float(self.config.l1_weight)

    @property
    def fused_ssim_weight(self) -> float:
        return float(self.config.ssim_weight) if self.ssim is not None else 0.0

    @property
    def fused_perceptual(self) -> Optional[dict]:
        if self.perceptual is None:
            return None
        return self.perceptual.fused_spec(float(self.config.perceptual_weight))

    def forward(self, pred, target) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        l1 = self.l1(pred, target)
        total = l1 * self.config.l1_weight
        comps = {"l1": l1.detach()}
        if self.perceptual is not None:
            pl = self.perceptual(pred, target)
            total = total + self.config.perceptual_weight * pl
            comps["perceptual"] = pl.detach()
        if self.ssim is not None:
            sl = self.ssim(pred, target)
            total = total + self.config.ssim_weight * sl
            comps["ssim"] = sl.detach()
        comps["total"] = total.detach()
        return total, comps


def create_loss_function(l1_weight: float = 1.0, perceptual_weight: float = 0.01, ssim_weight: float = 0.1,
                         use_charbonnier: bool = False, charbonnier_eps: float = 1e-3,
                         perceptual_layers=None, **kwargs) -> CombinedLoss:
    """Factory with the reference's signature (combined.py:278-302)."""
    cfg = LossConfig(l1_weight=l1_weight, perceptual_weight=perceptual_weight, ssim_weight=ssim_weight,
                     use_charbonnier=use_charbonnier, charbonnier_eps=charbonnier_eps,
                     perceptual_layers=list(perceptual_layers or ["conv3_4", "conv4_4"]))
    return CombinedLoss(cfg)


from .perceptual import PerceptualLoss, VGGFeatureExtractor  # noqa: E402
from .ssim import MSSSIMLoss, SSIMLoss, ssim  # noqa: E402

__all__ = ["LossConfig", "L1Loss", "CombinedLoss", "create_loss_function", "PerceptualLoss", "VGGFeatureExtractor",
           "SSIMLoss", "MSSSIMLoss", "ssim"]
