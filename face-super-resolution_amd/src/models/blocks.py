"""Building blocks of FaceEnhanceNet with the reference's module API, HIP-backed.

Same classes, constructor signatures, attribute names and parameter shapes as the
reference (tomasz-pres/face-super-resolution src/models/blocks.py), so state_dicts and
hooks interchange.  The parameters are ordinary nn.Conv2d / nn.PReLU / nn.Linear members
(construction consumes the global RNG exactly like the reference, so a seeded model is
bit-identical); forward/backward run on the MI355X through libfen_hip.so.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..hip.autograd import ChannelAttentionFn, GroupFn, RCABFn, Runtime, UpsampleFn
from ..hip.net import NetSpec

_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
           "fp16": torch.float16, "float16": torch.float16}


def compute_dtype(precision: str) -> torch.dtype:
    try:
        return _DTYPES[precision]
    except KeyError:
        raise ValueError(f"precision must be one of {sorted(_DTYPES)}, got {precision!r}") from None


def icnr_init(tensor: torch.Tensor, scale_factor: int = 2) -> torch.Tensor:
    """ICNR init for a conv feeding PixelShuffle (reference blocks.py:14-41): one kaiming
    (fan_out, relu) sub-kernel per output channel group, repeated over the s*s sub-pixels."""
    out_ch, in_ch, kh, kw = tensor.shape
    groups = out_ch // (scale_factor ** 2)
    base = torch.empty(groups, in_ch, kh, kw)
    nn.init.kaiming_normal_(base, mode="fan_out", nonlinearity="relu")
    with torch.no_grad():
        tensor.copy_(base.repeat_interleave(scale_factor ** 2, dim=0))
    return tensor


def _need_hip(kernel_size: int):
    if kernel_size != 3:
        raise NotImplementedError("the gfx950 conv kernels implement 3x3 / pad 1 (the reference's only use)")


class ChannelAttention(nn.Module):
    """Squeeze-and-excitation gate (reference blocks.py:44-92)."""

    def __init__(self, num_channels: int, reduction_ratio: int = 4, precision: str = "fp32"):
        super().__init__()
        self.num_channels = num_channels
        self.reduction_ratio = reduction_ratio
        reduced = max(num_channels // reduction_ratio, 8)
        self.global_pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Sequential(
            nn.Linear(num_channels, reduced, bias=False),
            nn.ReLU(inplace=True),
            nn.Linear(reduced, num_channels, bias=False),
            nn.Sigmoid(),
        )
        self._rt = Runtime(self, None, compute_dtype(precision))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ChannelAttentionFn.apply(x, self.fc[0].weight, self.fc[2].weight, self._rt)


class RCAB(nn.Module):
    """Residual channel-attention block (reference blocks.py:95-153):
    conv3x3 -> PReLU -> conv3x3 -> SE gate -> out * res_scale + x."""

    def __init__(self, num_channels: int = 64, kernel_size: int = 3, reduction_ratio: int = 4,
                 bias: bool = True, res_scale: float = 0.2, precision: str = "fp32"):
        super().__init__()
        _need_hip(kernel_size)
        if not bias:
            raise NotImplementedError("RCAB(bias=False) is not used by the reference models")
        self.res_scale = res_scale
        self.conv1 = nn.Conv2d(num_channels, num_channels, kernel_size, padding=kernel_size // 2, bias=bias)
        self.prelu = nn.PReLU(num_channels)
        self.conv2 = nn.Conv2d(num_channels, num_channels, kernel_size, padding=kernel_size // 2, bias=bias)
        self.channel_attention = ChannelAttention(num_channels, reduction_ratio, precision)
        spec = NetSpec(C=num_channels, G=1, NB=1, Cr=max(num_channels // reduction_ratio, 8), res_scale=res_scale)
        self._rt = Runtime(self, spec, compute_dtype(precision))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        self._rt.grad_mode = torch.is_grad_enabled()
        return RCABFn.apply(x, self._rt, *[p for _, p in self.named_parameters()])


class ResidualGroup(nn.Module):
    """num_blocks RCABs + conv3x3 + group skip (reference blocks.py:156-189)."""

    def __init__(self, num_channels: int = 64, num_blocks: int = 4, kernel_size: int = 3,
                 reduction_ratio: int = 4, res_scale: float = 0.2, precision: str = "fp32"):
        super().__init__()
        _need_hip(kernel_size)
        self.blocks = nn.Sequential(*[
            RCAB(num_channels, kernel_size, reduction_ratio, res_scale=res_scale, precision=precision)
            for _ in range(num_blocks)
        ])
        self.conv = nn.Conv2d(num_channels, num_channels, kernel_size, padding=kernel_size // 2)
        spec = NetSpec(C=num_channels, G=1, NB=num_blocks, Cr=max(num_channels // reduction_ratio, 8),
                       res_scale=res_scale)
        self._rt = Runtime(self, spec, compute_dtype(precision))
        self._attn = None  # set by FaceEnhanceNet.get_attention_maps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        self._rt.grad_mode = torch.is_grad_enabled()
        return GroupFn.apply(x, self._rt, self._attn, *[p for _, p in self.named_parameters()])


class PixelShuffleUpsample(nn.Module):
    """conv C -> C*s^2, PixelShuffle(s), PReLU(C) (reference blocks.py:192-227)."""

    def __init__(self, in_channels: int, scale_factor: int = 2, precision: str = "fp32"):
        super().__init__()
        if scale_factor != 2:
            raise NotImplementedError("PixelShuffleUpsample stages are x2 (UpsampleModule builds log2(scale) of them)")
        self.scale_factor = scale_factor
        self.conv = nn.Conv2d(in_channels, in_channels * scale_factor ** 2, kernel_size=3, padding=1)
        self.pixel_shuffle = nn.PixelShuffle(scale_factor)
        self.prelu = nn.PReLU(in_channels)
        icnr_init(self.conv.weight, scale_factor)
        if self.conv.bias is not None:
            nn.init.zeros_(self.conv.bias)
        self._precision = precision

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # a single x2 stage is an UpsampleModule of scale 2 over this module's parameters
        rt = getattr(self, "_rt", None)
        if rt is None:
            rt = self._rt = _StageRuntime(self, compute_dtype(self._precision))
        return UpsampleFn.apply(x, rt, *[p for _, p in self.named_parameters()])


class _StageRuntime(Runtime):
    """Runtime exposing one PixelShuffleUpsample's parameters under UpsampleModule key names."""

    def __init__(self, stage: PixelShuffleUpsample, dtype):
        super().__init__(stage, NetSpec(C=stage.conv.in_channels, scale=2), dtype)

    def wt(self, device):
        from ..hip.autograd import LiveWeights
        if self.weights is None or self.weights.device != device:
            self.weights = LiveWeights({"stages.0." + k: v for k, v in self.module.named_parameters()},
                                       self.dtype, device)
        self.weights.refresh()
        return self.weights


class UpsampleModule(nn.Module):
    """log2(scale) PixelShuffleUpsample x2 stages (reference blocks.py:230-263)."""

    def __init__(self, num_channels: int = 64, scale_factor: int = 4, precision: str = "fp32"):
        super().__init__()
        self.scale_factor = scale_factor
        n, t = 0, scale_factor
        while t > 1:
            t //= 2
            n += 1
        self.stages = nn.Sequential(*[PixelShuffleUpsample(num_channels, 2, precision) for _ in range(n)])
        self._rt = Runtime(self, NetSpec(C=num_channels, scale=2 ** n), compute_dtype(precision))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return UpsampleFn.apply(x, self._rt, *[p for _, p in self.named_parameters()])


def initialize_weights(module: nn.Module, scale: float = 0.1) -> None:
    """Kaiming(fan_in) * scale for convs and linears, zero biases (reference blocks.py:266-286)."""
    for m in module.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            nn.init.kaiming_normal_(m.weight, a=0, mode="fan_in")
            if m.bias is not None:
                nn.init.zeros_(m.bias)
            m.weight.data *= scale
