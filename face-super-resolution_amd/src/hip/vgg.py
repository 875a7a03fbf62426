"""VGG19 perceptual loss on the HIP path (reference src/losses/perceptual.py:13-169).

The frozen feature extractor runs ONCE over [pred; target] stacked in one batch of 2B
(pred = the generator output, target = HR): conv1_1 on the K=27 input kernel with the
ImageNet normalisation fused (perceptual.py:67-72,84-95); every later conv on fen_conv3x3
with bias + ReLU fused (PReLU epilogue with zero slopes; a feature layer keeps its
pre-ReLU output through y_pre); the max pools from the store of the conv before them
(fen_conv_desc.y_pool, which also keeps that conv's ReLU output for the pred half only).  The loss
(weight x nn.L1Loss / nn.MSELoss of each requested layer, perceptual.py:155-167) and its
gradient come from fen_feat_loss, and the backward runs on the pred half only: mode-2
data gradients whose epilogue applies the ReLU mask (FEN_EPI_RELU_BWD, pre_in = the saved
ReLU output; no slope partials), fen_maxpool2_bwd_relu through the pools, and conv1_1's data
gradient (weights pre-divided by the ImageNet std, so it yields d(pred)) added straight into
the generator's dL/dsr buffer.  No weight gradients: the extractor is frozen
(perceptual.py:60-64).

Feature layers: conv outputs (the reference's LAYER_MAP 'convX_Y' names, e.g. the stage
configs' conv3_4 / conv4_4) except conv1_1.  relu / pool names raise NotImplementedError.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch

from . import lib as L
from .net import conv
from .program import Ctx, ptr

# perceptual.py:21-30 (torchvision vgg19.features indices)
LAYER_MAP = {
    'conv1_1': 0, 'relu1_1': 1, 'conv1_2': 2, 'relu1_2': 3, 'pool1': 4,
    'conv2_1': 5, 'relu2_1': 6, 'conv2_2': 7, 'relu2_2': 8, 'pool2': 9,
    'conv3_1': 10, 'relu3_1': 11, 'conv3_2': 12, 'relu3_2': 13,
    'conv3_3': 14, 'relu3_3': 15, 'conv3_4': 16, 'relu3_4': 17, 'pool3': 18,
    'conv4_1': 19, 'relu4_1': 20, 'conv4_2': 21, 'relu4_2': 22,
    'conv4_3': 23, 'relu4_3': 24, 'conv4_4': 25, 'relu4_4': 26, 'pool4': 27,
    'conv5_1': 28, 'relu5_1': 29, 'conv5_2': 30, 'relu5_2': 31,
    'conv5_3': 32, 'relu5_3': 33, 'conv5_4': 34, 'relu5_4': 35, 'pool5': 36,
}
VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
             512, 512, 512, 512, "M"]
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
# A/B switch only: FEN_VGG_LEGACY=1 records round 5's form (PReLU-backward epilogues with slope
# partials, k_maxpool2 passes) instead of FEN_EPI_RELU_BWD and the fused y_pool stores
_LEGACY = os.environ.get("FEN_VGG_LEGACY", "0") == "1"


def vgg19_convs() -> List[dict]:
    """The convs of vgg19.features in order: index, cin, cout, and whether a pool follows
    the conv's ReLU."""
    convs, idx, cin = [], 0, 3
    for v in VGG19_CFG:
        if v == "M":
            convs[-1]["pool_after"] = True
            idx += 1
        else:
            convs.append(dict(idx=idx, cin=cin, cout=v, pool_after=False))
            idx += 2
            cin = v
    return convs


def feature_indices(layers: Sequence[str]) -> List[int]:
    out = []
    for name in layers:
        if name not in LAYER_MAP:
            raise KeyError(f"unknown VGG19 layer {name!r}")
        i = LAYER_MAP[name]
        if not name.startswith("conv"):
            raise NotImplementedError(f"HIP perceptual loss: feature layer {name!r} (only conv outputs are wired)")
        if i == 0:
            raise NotImplementedError("HIP perceptual loss: conv1_1 as a feature layer")
        out.append(i)
    return out


class VGGPerceptual:
    """Records the perceptual loss (forward on [pred; target], loss, pred-half backward)
    into a Ctx program.  `params`: fp32 device tensors keyed like torchvision
    ('features.{i}.weight' / '.bias')."""

    def __init__(self, ctx: Ctx, params: Dict[str, torch.Tensor], layers: Sequence[str] = ("conv3_4",),
                 weights: Optional[Dict[str, float]] = None, criterion: str = "l1", normalize: bool = True):
        if criterion not in ("l1", "l2"):
            raise ValueError(f"Unknown criterion: {criterion}")
        self.ctx, self.p = ctx, params
        self.layers = list(layers)
        self.idx = feature_indices(self.layers)
        self.wts = {LAYER_MAP[n]: float((weights or {}).get(n, 1.0)) for n in self.layers}
        self.l2 = criterion == "l2"
        last = max(self.idx)
        self.convs = [c for c in vgg19_convs() if c["idx"] <= last]
        dev = next(iter(params.values())).device
        self.dev = dev
        if normalize:
            self.mean = torch.tensor(IMAGENET_MEAN, device=dev)
            self.istd = 1.0 / torch.tensor(IMAGENET_STD, device=dev)
        else:
            self.mean = torch.zeros(3, device=dev)
            self.istd = torch.ones(3, device=dev)
        self.zeros = {}
        self.packed = {}
        self.refresh_weights()

    def _zeros(self, n):
        if n not in self.zeros:
            self.zeros[n] = torch.zeros(n, device=self.dev)
        return self.zeros[n]

    def refresh_weights(self):
        """(Re)pack the frozen weights: forward layout for convs after conv1_1, data-gradient
        layout for every conv (conv1_1's divided by the normalisation std per input channel)."""
        ctx = self.ctx
        for c in self.convs:
            w = self.p[f"features.{c['idx']}.weight"].float().contiguous()
            if c["idx"] > 0:
                self.packed[(c["idx"], 0)] = self._pack(w, 0)
                wd = w
            else:
                wd = (w * self.istd.view(1, 3, 1, 1)).contiguous()
                self._keep = wd
            self.packed[(c["idx"], 2)] = self._pack(wd, 2)

    def _pack(self, w, mode):
        ctx = self.ctx
        cout, cin = w.shape[0], w.shape[1]
        n = ctx.lib.fen_packed_elems(mode, cout, cin)
        out = torch.empty(n, dtype=ctx.tdtype, device=self.dev)
        L.check(ctx.lib.fen_pack_conv_w(ctx.code, mode, cout, cin, ptr(w), ptr(out),
                                        torch.cuda.current_stream().cuda_stream), "vgg pack")
        return out

    # ------------------------------------------------------------------ program
    def forward(self, x: torch.Tensor, ctx: Optional[Ctx] = None, upto: Optional[int] = None,
                keep_images: int = 0):
        """Record the extractor over NCHW fp32 x [N,3,H,W] up to conv index `upto` (default:
        the deepest feature).  Returns (acts, feats): per conv its ReLU output and geometry,
        and {feature index: NHWC [N,h,w,C] pre-ReLU conv output}.  A conv followed by a max pool
        stores the pooled map from its epilogue (fen_conv_desc.y_pool, no k_maxpool2 pass) and
        its own ReLU output only for the first `keep_images` images (0: all) -- the pred half,
        whose pool masks the backward reads."""
        ctx = ctx or self.ctx
        N, _, H, W = x.shape
        last_idx = self.convs[-1]["idx"] if upto is None else upto
        convs = [c for c in self.convs if c["idx"] <= last_idx]
        acts, feats = [], {}
        h, hh, ww = None, H, W
        for c in convs:
            i, cin, cout = c["idx"], c["cin"], c["cout"]
            fuse = False
            is_feat, is_last = i in self.idx, i == last_idx
            if i == 0:
                a = ctx.alloc((N, hh, ww, cout))
                ctx.emit("vgg_conv1_1", ctx.lib.fen_conv_first_fwd_ex, ctx.code, N, 3, hh, ww, cout, ptr(x),
                         ptr(self.p["features.0.weight"]), ptr(self.p["features.0.bias"]), ptr(self.mean),
                         ptr(self.istd), 0.0, ptr(a))
                z = None
            elif is_last:
                z = ctx.alloc((N, hh, ww, cout))
                conv(ctx, h, self.packed[(i, 0)], N, hh, ww, cin, cout, bias=self.p[f"features.{i}.bias"], y=z)
                a = None
            else:
                # (fen_conv3x3 fuses the pool into the 16-bit persistent kernels' store and pools
                # in a k_maxpool2 pass everywhere else)
                pool = c["pool_after"] and not is_last and not (hh | ww) & 1
                fuse = pool and not _LEGACY
                a = ctx.alloc((N, hh, ww, cout))
                z = ctx.alloc((N, hh, ww, cout)) if is_feat else None
                pooled = ctx.alloc((N, hh // 2, ww // 2, cout)) if pool else None
                conv(ctx, h, self.packed[(i, 0)], N, hh, ww, cin, cout, bias=self.p[f"features.{i}.bias"],
                     epi=L.EPI_PRELU, alpha=self._zeros(cout), y=a, y_pre=z, y_pool=pooled if fuse else None,
                     y_images=keep_images if fuse and not is_feat else 0)
            if is_feat:
                feats[i] = z
            acts.append(dict(c=c, a=a, H=hh, W=ww))
            h = a
            if c["pool_after"] and not is_last:
                if not fuse:
                    pooled = ctx.alloc((N, hh // 2, ww // 2, cout))
                    ctx.emit("vgg_pool", ctx.lib.fen_maxpool2, ctx.code, N, hh, ww, cout, ptr(a), ptr(pooled))
                h, hh, ww = pooled, hh // 2, ww // 2
        return acts, feats

    def build(self, x2: torch.Tensor, loss: torch.Tensor, dpred: Optional[torch.Tensor], ctx: Optional[Ctx] = None,
              grad_scale: float = 1.0) -> Dict[int, torch.Tensor]:
        """x2: NCHW fp32 [2B,3,H,W] = [pred; target]; loss: fp32 [1], set to the weighted
        perceptual loss; dpred: NHWC [B,H,W,16] (dtype) dL/dpred, which grad_scale x the
        perceptual gradient is ADDED to (None: forward + loss only).  Returns the features."""
        ctx = ctx or self.ctx
        N = x2.shape[0]
        B = N // 2
        train = dpred is not None
        acts, feats = self.forward(x2, ctx, keep_images=B if train else 0)
        nparts = ctx.lib.fen_feat_loss_parts()
        order = sorted(self.idx, reverse=True)
        first = [True]

        def feat_loss(i, d, j):
            f = feats[i]
            n = f.numel() // 2
            g = d if d is not None else ctx.alloc((B,) + tuple(f.shape[1:]))
            part = ctx.scratch(f"vgg_lpart{j}", (nparts,), torch.float32)
            ctx.emit("vgg_feat_loss", ctx.lib.fen_feat_loss, ctx.code, n, ptr(f), int(self.l2),
                     self.wts[i] / n * grad_scale, ptr(g), int(d is not None), ptr(part))
            ctx.emit("vgg_loss_sum", ctx.lib.fen_colsum, nparts, 1, ptr(part), self.wts[i] / n, ptr(loss),
                     0 if first[0] else 1)
            first[0] = False
            return g

        if not train:
            for j, i in enumerate(order):
                feat_loss(i, None, j)
            return feats
        # backward on the pred half (first B images of every saved activation)
        d = None
        for k in range(len(acts) - 1, -1, -1):
            c = acts[k]["c"]
            i = c["idx"]
            if i in self.idx:
                d = feat_loss(i, d, order.index(i))
            hh, ww = acts[k]["H"], acts[k]["W"]
            if i == 0:
                # d(pred) (NHWC, 3 valid of 16 channels) += dgrad of conv1_1 / std
                conv(ctx, d, self.packed[(0, 2)], B, hh, ww, c["cout"], 16, y=dpred, res=(dpred,))
                break
            prev = acts[k - 1]
            pc = prev["c"]
            if pc["pool_after"]:
                # (the pool's backward in the dgrad's epilogue instead -- 2x2 scatter of 8-B stores
                # and window loads -- measured slower: 189 vs 82 + 45 us at conv3_1, 274 vs 93 + 92 at
                # conv2_1, r6)
                dp = ctx.alloc((B, hh, ww, c["cin"]))
                conv(ctx, d, self.packed[(i, 2)], B, hh, ww, c["cout"], c["cin"], y=dp)
                dz = ctx.alloc((B, prev["H"], prev["W"], pc["cout"]))
                ctx.emit("vgg_pool_bwd", ctx.lib.fen_maxpool2_bwd_relu, ctx.code, B, prev["H"], prev["W"],
                         pc["cout"], ptr(dp), ptr(prev["a"]), ptr(dz))
            else:
                dz = ctx.alloc((B, hh, ww, c["cin"]))
                if _LEGACY:
                    part = ctx.scratch("vgg_dal", (B * ((hh + 15) // 16) * ((ww + 15) // 16), c["cin"]), torch.float32)
                    conv(ctx, d, self.packed[(i, 2)], B, hh, ww, c["cout"], c["cin"], epi=L.EPI_PRELU_BWD,
                         alpha=self._zeros(c["cin"]), pre_in=prev["a"], y=dz, part=part)
                else:
                    conv(ctx, d, self.packed[(i, 2)], B, hh, ww, c["cout"], c["cin"], epi=L.EPI_RELU_BWD,
                         pre_in=prev["a"], y=dz)
            d = dz
        return feats
