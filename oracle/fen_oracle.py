"""CPU oracle for the FaceEnhanceNet hot path  --  TEST INFRASTRUCTURE ONLY.

This module is the *checker*.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it.  The product path (face-super-resolution_amd/src) never
imports or calls it and fails loudly when the HIP library is missing.

It is a functional restatement, in plain PyTorch-CPU ops, of the reference algorithm
(tomasz-pres/face-super-resolution @ /root/reference), written from SURVEY.md §8a and
the cited reference lines -- it shares no code with the reference.  Parity of this
oracle is PINNED against golden vectors produced by importing the reference itself
(tests/golden/make_golden.py -> tests/golden/*.npz; tests/test_oracle.py).

Parameters are passed as a flat dict keyed exactly like the reference state_dict
(SURVEY.md §8b), tensors in the reference OIHW fp32 layout.
"""
from __future__ import annotations

import math

import numpy as np
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


@dataclass
class NetShape:
    """Architecture knobs used by the oracle (reference custom.py:22-43)."""
    num_channels: int = 64
    num_groups: int = 3
    blocks_per_group: int = 4
    reduction_ratio: int = 4
    scale_factor: int = 4
    res_scale: float = 0.2


# ---------------------------------------------------------------------------------------
# bicubic resampling, align_corners=False, A = -0.75, border-clamped taps
# (used by custom.py:158-161 for the x4 skip and trainer.py:416-421 for the /4 LR synthesis)
# ---------------------------------------------------------------------------------------
def _cubic_weights(t: torch.Tensor, A: float = -0.75) -> torch.Tensor:
    """Keys cubic convolution weights for the 4 taps at offsets -1,0,1,2 around floor(src)."""
    def w_near(d):  # |d| <= 1
        return ((A + 2) * d - (A + 3)) * d * d + 1

    def w_far(d):  # 1 < |d| < 2
        return ((A * d - 5 * A) * d + 8 * A) * d - 4 * A

    return torch.stack([w_far(t + 1), w_near(t), w_near(1 - t), w_far(2 - t)], dim=-1)


def _resize_axis(x: torch.Tensor, out_len: int, scale: float, dim: int) -> torch.Tensor:
    in_len = x.shape[dim]
    d = torch.arange(out_len, dtype=torch.float64)
    src = (d + 0.5) / scale - 0.5
    i0 = torch.floor(src)
    t = src - i0
    w = _cubic_weights(t)                                    # [out, 4]
    idx = i0.long().unsqueeze(-1) + torch.arange(-1, 3)      # [out, 4]
    idx = idx.clamp(0, in_len - 1)
    xm = x.movedim(dim, -1)                                  # [..., in]
    g = xm[..., idx]                                         # [..., out, 4]
    y = (g * w.to(x.dtype)).sum(-1)
    return y.movedim(-1, dim)


def bicubic(x: torch.Tensor, scale: float) -> torch.Tensor:
    """F.interpolate(x, scale_factor=scale, mode='bicubic', align_corners=False) restated."""
    n, c, h, w = x.shape
    oh, ow = int(math.floor(h * scale)), int(math.floor(w * scale))
    y = _resize_axis(x, oh, scale, 2)
    return _resize_axis(y, ow, scale, 3)


def pixel_shuffle(x: torch.Tensor, r: int) -> torch.Tensor:
    """out[b, c, r*h+i, r*w+j] = in[b, c*r*r + i*r + j, h, w]  (blocks.py:215,225)."""
    b, c, h, w = x.shape
    co = c // (r * r)
    return x.reshape(b, co, r, r, h, w).permute(0, 1, 4, 2, 5, 3).reshape(b, co, h * r, w * r)


def prelu(x: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    return torch.where(x > 0, x, a.view(1, -1, 1, 1) * x)


def conv3x3(x, w, b):
    return F.conv2d(x, w, b, padding=1)


# ---------------------------------------------------------------------------------------
# network blocks (reference blocks.py / custom.py)
# ---------------------------------------------------------------------------------------
def channel_attention(t: torch.Tensor, p: Params, pre: str) -> torch.Tensor:
    """blocks.py:83-92 -> the sigmoid gate s[b, c]."""
    y = t.mean(dim=(2, 3))
    y = torch.relu(y @ p[pre + "fc.0.weight"].t())
    return torch.sigmoid(y @ p[pre + "fc.2.weight"].t())


def rcab(x: torch.Tensor, p: Params, pre: str, res_scale: float, attn: Optional[dict] = None,
         name: str = "") -> torch.Tensor:
    """blocks.py:135-153: conv -> PReLU -> conv -> SE gate -> out*res_scale + x."""
    t = conv3x3(x, p[pre + "conv1.weight"], p[pre + "conv1.bias"])
    t = prelu(t, p[pre + "prelu.weight"])
    t = conv3x3(t, p[pre + "conv2.weight"], p[pre + "conv2.bias"])
    s = channel_attention(t, p, pre + "channel_attention.")
    if attn is not None:
        attn[name] = s.detach()
    return t * s[:, :, None, None] * res_scale + x


def residual_group(x, p, pre, nb, res_scale, attn=None, gi=0):
    """blocks.py:185-189."""
    out = x
    for bi in range(nb):
        out = rcab(out, p, f"{pre}blocks.{bi}.", res_scale, attn, f"group{gi}_rcab{bi}")
    out = conv3x3(out, p[pre + "conv.weight"], p[pre + "conv.bias"])
    return out + x


def forward(p: Params, x: torch.Tensor, shape: NetShape, training: bool = True,
            attn: Optional[dict] = None) -> torch.Tensor:
    """FaceEnhanceNet.forward (custom.py:147-190)."""
    bic = bicubic(x, shape.scale_factor)
    feat = conv3x3(x, p["conv_first.weight"], p["conv_first.bias"])
    res = feat
    for g in range(shape.num_groups):
        feat = residual_group(feat, p, f"residual_groups.{g}.", shape.blocks_per_group,
                              shape.res_scale, attn, g)
    feat = conv3x3(feat, p["conv_after_body.weight"], p["conv_after_body.bias"]) + res
    n_stages = int(round(math.log2(shape.scale_factor)))
    for s in range(n_stages):
        pre = f"upsample.stages.{s}."
        feat = conv3x3(feat, p[pre + "conv.weight"], p[pre + "conv.bias"])
        feat = pixel_shuffle(feat, 2)
        feat = prelu(feat, p[pre + "prelu.weight"])
    out = conv3x3(feat, p["conv_last.weight"], p["conv_last.bias"]) + bic
    if not training:
        out = out.clamp(0.0, 1.0)
    return out


def lr_from_hr(hr: torch.Tensor) -> torch.Tensor:
    """trainer.py:416-421: F.interpolate(hr, 0.25, 'bicubic', align_corners=False)."""
    return bicubic(hr, 0.25)


def psnr(pred: torch.Tensor, target: torch.Tensor) -> float:
    """trainer.py:621-628 (batch-mean MSE), evaluated in fp64."""
    mse = torch.mean((pred.double() - target.double()) ** 2)
    return float(10.0 * torch.log10(1.0 / mse))


# ---------------------------------------------------------------------------------------
# one optimizer step: L1 loss, backward, clip_grad_norm_, AdamW (trainer.py:458-503)
# ---------------------------------------------------------------------------------------
def l1_grads(p: Params, hr: torch.Tensor, shape: NetShape) -> Tuple[float, Params]:
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    lr = lr_from_hr(hr)
    out = forward(leaves, lr, shape, training=True)
    loss = (out - hr).abs().mean()
    loss.backward()
    return float(loss), {k: v.grad.detach() for k, v in leaves.items()}


def clip_coef(grads: Params, max_norm: float) -> float:
    """torch.nn.utils.clip_grad_norm_ semantics: coef = max_norm/(||g||+1e-6), capped at 1."""
    norms = torch.stack([g.detach().float().norm(2) for g in grads.values()])
    total = norms.norm(2)
    return float(torch.clamp(max_norm / (total + 1e-6), max=1.0))


def adamw_step(p: Params, g: Params, m: Params, v: Params, step: int, lr: float,
               betas=(0.9, 0.999), eps=1e-8, wd=0.0) -> None:
    """torch.optim.AdamW single-tensor update restated (in place on p, m, v)."""
    b1, b2 = betas
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    for k in p:
        p[k].mul_(1 - lr * wd)
        m[k].lerp_(g[k], 1 - b1)
        v[k].mul_(b2).addcmul_(g[k], g[k], value=1 - b2)
        denom = (v[k].sqrt() / math.sqrt(bc2)).add_(eps)
        p[k].addcdiv_(m[k], denom, value=-lr / bc1)


def train_step(p: Params, hr: torch.Tensor, shape: NetShape, lr: float = 1e-4,
               clip: float = 0.5, wd: float = 0.0) -> Tuple[float, Params]:
    """One Trainer._train_epoch batch (fresh optimizer state): returns (loss, new params)."""
    loss, g = l1_grads(p, hr, shape)
    if clip > 0:
        c = clip_coef(g, clip)
        g = {k: t * c for k, t in g.items()}
    newp = {k: t.detach().clone() for k, t in p.items()}
    m = {k: torch.zeros_like(t) for k, t in newp.items()}
    v = {k: torch.zeros_like(t) for k, t in newp.items()}
    adamw_step(newp, g, m, v, 1, lr, wd=wd)
    return loss, newp


def rcab_with_grads(p: Params, x: torch.Tensor, r: torch.Tensor, res_scale: float = 0.2):
    """G2 helper: out and the gradients of sum(out*r) w.r.t. x and every RCAB parameter."""
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    xl = x.detach().clone().requires_grad_(True)
    out = rcab(xl, leaves, "", res_scale)
    (out * r).sum().backward()
    return out.detach(), xl.grad.detach(), {k: v.grad.detach() for k, v in leaves.items()}


# ---------------------------------------------------------------------------------------
# VGG19 perceptual loss (reference src/losses/perceptual.py:13-169).  PARITY UNPINNED: the
# reference builds torchvision.models.vgg19 with ImageNet weights (perceptual.py:48), and
# neither torchvision nor the weights exist offline.  This restates the
# torchvision vgg19.features layer list (config 'E': 16 convs 3x3 pad 1 + ReLU, max pools
# 2x2) and the loss as written in perceptual.py, for any weights given as a state dict
# keyed like torchvision ('features.{i}.weight' / '.bias').
VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
             512, 512, 512, 512, "M"]
VGG_MEAN = (0.485, 0.456, 0.406)     # perceptual.py:67-72
VGG_STD = (0.229, 0.224, 0.225)


def vgg19_layers():
    """[(index, kind, cin, cout)] of torchvision vgg19.features; kind in conv/relu/pool."""
    out, idx, cin = [], 0, 3
    for v in VGG19_CFG:
        if v == "M":
            out.append((idx, "pool", cin, cin))
            idx += 1
        else:
            out.append((idx, "conv", cin, v))
            out.append((idx + 1, "relu", v, v))
            idx += 2
            cin = v
    return out


def vgg19_init(seed: int = 0) -> Params:
    """Random weights in the torchvision layout (kaiming fan_out, zero bias), for tests."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for idx, kind, cin, cout in vgg19_layers():
        if kind == "conv":
            std = math.sqrt(2.0 / (cout * 9))
            p[f"features.{idx}.weight"] = torch.randn(cout, cin, 3, 3, generator=g) * std
            p[f"features.{idx}.bias"] = torch.randn(cout, generator=g) * 0.01
    return p


def vgg_features(p: Params, x: torch.Tensor, layer_indices, normalize: bool = True) -> Dict[int, torch.Tensor]:
    """perceptual.py:84-101: normalise, run features[:max+1], collect the listed indices."""
    if normalize:
        mean = torch.tensor(VGG_MEAN, dtype=x.dtype).view(1, 3, 1, 1)
        std = torch.tensor(VGG_STD, dtype=x.dtype).view(1, 3, 1, 1)
        x = (x - mean) / std
    feats = {}
    last = max(layer_indices)
    for idx, kind, _, _ in vgg19_layers():
        if idx > last:
            break
        if kind == "conv":
            x = F.conv2d(x, p[f"features.{idx}.weight"].to(x.dtype), p[f"features.{idx}.bias"].to(x.dtype), padding=1)
        elif kind == "relu":
            x = F.relu(x)
        else:
            x = F.max_pool2d(x, 2, 2)
        if idx in layer_indices:
            feats[idx] = x
    return feats


def perceptual_loss(p: Params, pred: torch.Tensor, target: torch.Tensor, layer_indices, weights=None,
                    criterion: str = "l1", normalize: bool = True) -> torch.Tensor:
    """perceptual.py:144-169: sum over layers of weight * criterion(f_pred, f_target)."""
    fp = vgg_features(p, pred, layer_indices, normalize)
    ft = vgg_features(p, target, layer_indices, normalize)
    loss = 0.0
    for i in layer_indices:
        w = 1.0 if weights is None else weights[i]
        d = F.l1_loss(fp[i], ft[i]) if criterion == "l1" else F.mse_loss(fp[i], ft[i])
        loss = loss + w * d
    return loss


# ---------------------------------------------------------------------------------------
# VGGStyleDiscriminator forward (reference src/models/discriminator.py:58-90 tree, 118-136
# forward), functional, train-mode BatchNorm (batch statistics, eps 1e-5), for gradient replays.
D_STRIDES = (1, 2, 1, 2, 1, 2, 1, 2, 1, 2)


def disc_forward(p: Params, x: torch.Tensor, masks=None, record=None, slope: float = 0.2) -> torch.Tensor:
    """Scores [B,1] of the discriminator with parameters p (its state_dict keys) on x, in x's
    dtype.  The 11 LeakyReLUs (10 feature blocks, the classifier's hidden layer) take their
    branch from `masks[i]` (bool, the activation's shape) when given -- the derivative of the
    piecewise-linear net on the linear piece another run (the HIP discriminator) took: an
    element whose pre-activation sits within rounding of 0 flips sides between precisions and
    moves every gradient below it by a finite step -- else from the sign of the pre-activation;
    `record` (a list) collects the masks this run took."""
    h = x
    for i, st in enumerate(D_STRIDES):
        b = p.get(f"features.{i}.0.bias")
        h = F.conv2d(h, p[f"features.{i}.0.weight"].to(h.dtype), None if b is None else b.to(h.dtype), stride=st,
                     padding=1)
        if i > 0:
            mu = h.mean((0, 2, 3), keepdim=True)
            var = h.var((0, 2, 3), unbiased=False, keepdim=True)
            h = ((h - mu) / torch.sqrt(var + 1e-5) * p[f"features.{i}.1.weight"].to(h.dtype).view(1, -1, 1, 1)
                 + p[f"features.{i}.1.bias"].to(h.dtype).view(1, -1, 1, 1))
        if record is not None:
            record.append((h > 0).detach())
        h = torch.where(h > 0 if masks is None else masks[i], h, slope * h)
    h = F.linear(h.flatten(1), p["classifier.1.weight"].to(h.dtype), p["classifier.1.bias"].to(h.dtype))
    if record is not None:
        record.append((h > 0).detach())
    h = torch.where(h > 0 if masks is None else masks[10], h, slope * h)
    return F.linear(h, p["classifier.3.weight"].to(h.dtype), p["classifier.3.bias"].to(h.dtype))


# ---------------------------------------------------------------------------------------
# SSIM (reference src/losses/ssim_loss.py:14-98,174-226); pinned by tests/golden/g7_ssim.npz
# (made by importing the reference module, tests/golden/make_golden_ssim.py)
def gaussian_window(window_size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    """ssim_loss.py:14-41: normalised 1-D Gaussian, 2-D window = outer product."""
    c = torch.arange(window_size, dtype=torch.float32) - window_size // 2
    g = torch.exp(-(c ** 2) / (2 * sigma ** 2))
    g = g / g.sum()
    return g[:, None] @ g[None, :]


def _ssim_terms(pred, target, window_size, sigma, data_range):
    C = pred.shape[1]
    w = gaussian_window(window_size, sigma).to(pred.dtype).expand(C, 1, window_size, window_size)
    pad = window_size // 2
    f = lambda x: F.conv2d(x, w, padding=pad, groups=C)   # noqa: E731
    mp, mt = f(pred), f(target)
    spp = f(pred * pred) - mp * mp
    stt = f(target * target) - mt * mt
    spt = f(pred * target) - mp * mt
    C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    lum = (2 * mp * mt + C1) / (mp * mp + mt * mt + C1)
    cs = (2 * spt + C2) / (spp + stt + C2)
    return lum, cs


def ssim(pred, target, window_size=11, sigma=1.5, data_range=1.0, size_average=True):
    """ssim_loss.py:44-98 (zero-padded depthwise Gaussian, K = (0.01, 0.03))."""
    lum, cs = _ssim_terms(pred, target, window_size, sigma, data_range)
    m = lum * cs
    return m.mean() if size_average else m.mean(dim=[1, 2, 3])


def ms_ssim(pred, target, window_size=11, sigma=1.5, data_range=1.0, weights=None):
    """ssim_loss.py:101-171: 5 scales, 2x2 average pooling between them."""
    if weights is None:
        weights = torch.tensor([0.0448, 0.2856, 0.3001, 0.2363, 0.1333], dtype=pred.dtype)
    mcs = []
    for i in range(len(weights)):
        lum, cs = _ssim_terms(pred, target, window_size, sigma, data_range)
        if i == len(weights) - 1:
            val = (lum * cs).mean()
        else:
            mcs.append(cs.mean())
        pred, target = F.avg_pool2d(pred, 2, 2), F.avg_pool2d(target, 2, 2)
    for i, m in enumerate(mcs):
        val = val * (m ** weights[i])
    return val


# ---------------------------------------------------------------------------------------
# train-mode HR transform (reference src/data/transforms.py:173-279, to_tensor 260-279), one
# sample with given parameters.  Flip / rot90 / brightness / contrast / uint8 quantisation
# follow the reference's numpy code; the HSV saturation round trip restates OpenCV's 8-bit
# RGB2HSV_b / HSV2RGB_b (cv2 is absent offline: that step is PARITY UNPINNED).
def _rgb2hsv8(img):
    r, g, b = (img[..., k].astype(np.int64) for k in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    sdiv = np.where(v > 0, np.rint((255 << 12) / np.maximum(v, 1)), 0).astype(np.int64)
    hdiv = np.where(diff > 0, np.rint((180 << 12) / (6.0 * np.maximum(diff, 1))), 0).astype(np.int64)
    s = (diff * sdiv + (1 << 11)) >> 12
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + (~vg & (r - g + 4 * diff))))
    h = (h * hdiv + (1 << 11)) >> 12
    h = h + np.where(h < 0, 180, 0)
    return np.stack([h, s, v], -1)


def _hsv2rgb8(hsv):
    h = hsv[..., 0].astype(np.float32)
    s = hsv[..., 1].astype(np.float32) * np.float32(1 / 255)
    v = hsv[..., 2].astype(np.float32) * np.float32(1 / 255)
    hh = h * np.float32(6 / 180)
    hh = np.where(hh >= 6, hh - 6, hh)
    sector = np.floor(hh).astype(np.int64)
    f = (hh - sector).astype(np.float32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    f = np.where(bad, np.float32(0), f)
    tab = np.stack([v, v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))], -1).astype(np.float32)
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    bgr = np.take_along_axis(tab, sd[sector], -1)
    bgr = np.where((s == 0)[..., None], v[..., None], bgr)
    out = np.clip(np.rint(bgr * np.float32(255)), 0, 255).astype(np.uint8)
    return out[..., ::-1]                       # b, g, r -> r, g, b


def transform_hr(img: np.ndarray, flip: int, rot: int, jitter: int, brightness: float, contrast: float,
                 saturation: float) -> np.ndarray:
    """uint8 HxWx3 crop -> float32 [3,H,W] in [0,1] (transforms.py:210-257 + to_tensor)."""
    if flip:
        img = np.fliplr(img).copy()
    if rot:
        img = np.rot90(img, rot).copy()
    if jitter:
        f = img.astype(np.float32) / np.float32(255.0)
        f = f * np.float32(brightness)
        mean = f.mean()
        f = (f - mean) * np.float32(contrast) + mean
        img = np.clip(f * np.float32(255), 0, 255).astype(np.uint8)
        hsv = _rgb2hsv8(img).astype(np.float32)
        hsv[..., 1] = hsv[..., 1] * np.float32(saturation)
        img = _hsv2rgb8(np.clip(hsv, 0, 255).astype(np.uint8))
    return img.transpose(2, 0, 1).astype(np.float32) / np.float32(255.0)
