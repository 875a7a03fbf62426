"""FaceEnhanceNet with the reference's module API (tomasz-pres/face-super-resolution
src/models/custom.py), running on MI355X through libfen_hip.so.

Drop-in contract: same FaceEnhanceNetConfig fields and defaults, same
constructor / factory / Lite variant, identical module tree and state_dict keys (OIHW
fp32 parameters), same seeded initialisation, same forward semantics (global bicubic
skip, eval-only clamp), `get_attention_maps`, `get_model_info`, `from_pretrained`.
New, defaulted config fields: `precision` ('fp32' reproduces the reference numerics;
'bf16' is the MI355X throughput mode; 'fp16' -- the reference's own AMP dtype, same MFMA rate,
3 more mantissa bits -- is the inference mode that holds PSNR parity within 0.01 dB).
"""
from __future__ import annotations

from dataclasses import dataclass, fields
from typing import Any, Dict, Optional

import torch
import torch.nn as nn

from ..hip.autograd import HeadFn, Runtime, TailFn
from ..hip.net import NetSpec
from .blocks import RCAB, ChannelAttention, ResidualGroup, UpsampleModule, compute_dtype, initialize_weights  # noqa: F401


@dataclass
class FaceEnhanceNetConfig:
    """Configuration for FaceEnhanceNet (reference custom.py:22-43) + `precision`."""
    num_channels: int = 64
    num_groups: int = 3
    blocks_per_group: int = 4
    kernel_size: int = 3
    reduction_ratio: int = 4
    scale_factor: int = 4
    res_scale: float = 0.2
    in_channels: int = 3
    out_channels: int = 3
    init_scale: float = 0.1
    num_rcab_blocks: int = 8
    precision: str = "fp32"


class FaceEnhanceNet(nn.Module):
    """conv_first -> num_groups ResidualGroups -> conv_after_body (+skip) -> PixelShuffle
    upsampler -> conv_last, plus a global bicubic skip (reference custom.py:46-190)."""

    def __init__(self, config: Optional[FaceEnhanceNetConfig] = None, **kwargs):
        super().__init__()
        if config is None:
            config = FaceEnhanceNetConfig()
        for key, value in kwargs.items():
            if hasattr(config, key):
                setattr(config, key, value)
        self.config = config
        self.scale_factor = config.scale_factor
        self.num_channels = config.num_channels
        prec = config.precision
        k = config.kernel_size
        self.conv_first = nn.Conv2d(config.in_channels, config.num_channels, k, padding=k // 2)
        self.residual_groups = nn.ModuleList([
            ResidualGroup(num_channels=config.num_channels, num_blocks=config.blocks_per_group, kernel_size=k,
                          reduction_ratio=config.reduction_ratio, res_scale=config.res_scale, precision=prec)
            for _ in range(config.num_groups)
        ])
        self.conv_after_body = nn.Conv2d(config.num_channels, config.num_channels, k, padding=k // 2)
        self.upsample = UpsampleModule(num_channels=config.num_channels, scale_factor=config.scale_factor,
                                       precision=prec)
        self.conv_last = nn.Conv2d(config.num_channels, config.out_channels, k, padding=k // 2)
        self._initialize_weights()
        self._rt = Runtime(self, NetSpec.from_config(config), compute_dtype(prec))

    def _initialize_weights(self) -> None:
        """kaiming(fan_out, relu) for every conv/linear, zero biases, conv_last = 0
        (reference custom.py:129-145; this overrides the upsampler's ICNR init, as there)."""
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        nn.init.constant_(self.conv_last.weight, 0)
        if self.conv_last.bias is not None:
            nn.init.constant_(self.conv_last.bias, 0)

    @property
    def compute_dtype(self) -> torch.dtype:
        return self._rt.dtype

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: LR [B,3,H,W] in [0,1] (fp32, on the GPU) -> SR [B,3,sH,sW] fp32."""
        feat0 = HeadFn.apply(x, self.conv_first.weight, self.conv_first.bias, self._rt)
        feat = feat0
        for group in self.residual_groups:
            feat = group(feat)
        tail = [p for n, p in self.named_parameters() if n.startswith(("conv_after_body.", "upsample.", "conv_last."))]
        needs_grad = torch.is_grad_enabled() and (feat.requires_grad or any(p.requires_grad for p in tail))
        fused_clamp = (not self.training) and not needs_grad
        self._rt.grad_mode = needs_grad
        out = TailFn.apply(feat, feat0, x.contiguous().float(), self._rt, fused_clamp, *tail)
        if not self.training and not fused_clamp:
            out = torch.clamp(out, 0.0, 1.0)  # eval clamp kept differentiable (custom.py:187-188)
        return out

    @torch.no_grad()
    def get_attention_maps(self, x: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Per-RCAB channel-attention vectors [B,C] keyed 'group{g}_rcab{b}' (custom.py:192-230)."""
        maps: Dict[str, torch.Tensor] = {}
        for g, grp in enumerate(self.residual_groups):
            grp._attn = {}
        try:
            self.forward(x)
            for g, grp in enumerate(self.residual_groups):
                for k, v in grp._attn.items():
                    maps[f"group{g}_rcab{k.split('_rcab')[1]}"] = v.clone()
        finally:
            for grp in self.residual_groups:
                grp._attn = None
        return maps

    def get_model_info(self) -> Dict[str, Any]:
        """Model statistics (reference custom.py:232-256)."""
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        size_in = 64
        return {
            "name": "FaceEnhanceNet",
            "total_params": total,
            "trainable_params": trainable,
            "size_mb": total * 4 / (1024 ** 2),
            "num_groups": self.config.num_groups,
            "blocks_per_group": self.config.blocks_per_group,
            "total_rcab_blocks": self.config.num_groups * self.config.blocks_per_group,
            "num_channels": self.config.num_channels,
            "scale_factor": self.scale_factor,
            "input_size": f"{size_in}x{size_in}",
            "output_size": f"{size_in * self.scale_factor}x{size_in * self.scale_factor}",
        }

    @classmethod
    def from_pretrained(cls, checkpoint_path: str, device: Optional[str] = None) -> "FaceEnhanceNet":
        """Load a reference-format checkpoint (custom.py:258-292).  Only tensors and plain
        containers are unpickled (weights_only=True)."""
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        known = {f.name for f in fields(FaceEnhanceNetConfig)}
        if isinstance(ckpt, dict) and isinstance(ckpt.get("config"), dict):
            cfg = FaceEnhanceNetConfig(**{k: v for k, v in ckpt["config"].items() if k in known})
        else:
            cfg = FaceEnhanceNetConfig()
        model = cls(cfg)
        if "model_state_dict" in ckpt:
            model.load_state_dict(ckpt["model_state_dict"])
        elif "state_dict" in ckpt:
            model.load_state_dict(ckpt["state_dict"])
        else:
            model.load_state_dict(ckpt)
        if device:
            model = model.to(device)
        return model


def create_face_enhance_net(num_rcab_blocks: int = 8, num_channels: int = 64, scale_factor: int = 4,
                            **kwargs) -> FaceEnhanceNet:
    """Factory (reference custom.py:295-319)."""
    cfg = FaceEnhanceNetConfig(num_rcab_blocks=num_rcab_blocks, num_channels=num_channels,
                               scale_factor=scale_factor, **kwargs)
    return FaceEnhanceNet(cfg)


class FaceEnhanceNetLite(FaceEnhanceNet):
    """32 channels, reduction 2 (reference custom.py:322-333)."""

    def __init__(self, **kwargs):
        cfg = FaceEnhanceNetConfig(num_channels=32, num_rcab_blocks=4, reduction_ratio=2, **kwargs)
        super().__init__(cfg)
