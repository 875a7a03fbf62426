"""torch.autograd.Functions that put the HIP kernels behind the reference's nn.Module API.

Module boundary tensors are logical NCHW [B,C,H,W] with channels_last storage (a free
permute of the kernels' NHWC buffers), in the model's compute dtype; GradCAM-style hooks
(reference src/explainability/gradcam.py:63-71) therefore see ordinary 4-D activations.
Every Function forwards/backwards through net.py builders on an eager Ctx: the work is
done by libfen_hip.so, PyTorch only allocates and orders it on the current stream.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

from . import lib as L
from .net import Backward, Forward, NetSpec, Weights, colsum, tiles, wgrad
from .program import Ctx, ptr


def to_nhwc(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """[B,C,H,W] (any layout) -> contiguous NHWC [B,H,W,C] of dtype (a view when already channels_last)."""
    if t.dtype != dtype:
        t = t.to(dtype)
    v = t.permute(0, 2, 3, 1)
    return v if v.is_contiguous() else v.contiguous()


def as_nchw(t_nhwc: torch.Tensor) -> torch.Tensor:
    return t_nhwc.permute(0, 3, 1, 2)


class LiveWeights(Weights):
    """Weights over live nn.Parameters; a packed copy is refreshed whenever its source
    parameter was modified in place (optimizer step, load_state_dict) or re-homed."""

    def __init__(self, params: Dict[str, torch.nn.Parameter], dtype, device):
        super().__init__({}, dtype, device)
        self.params = params
        self._stamp: Dict[tuple, tuple] = {}

    def refresh(self):
        self.p = {k: v.detach() for k, v in self.params.items()}

    def packed(self, key: str, mode: int) -> torch.Tensor:
        w = self.params[key + ".weight"]
        stamp = (w.data_ptr(), w._version)
        k = (key, mode)
        old = self._stamp.get(k)
        if k in self.packs and old != stamp:
            if old[0] == stamp[0]:
                # updated in place (an optimizer step bumps every parameter's version): re-pack
                # every known copy in ONE fen_pack_multi launch, instead of one launch per use.
                # A copy whose parameter was re-homed since it was packed (flatten_params) packs
                # from the current storage: the job table is rebuilt from the live parameters
                for kk in self.packs:
                    ww = self.params[kk[0] + ".weight"]
                    if self._src[kk].data_ptr() != ww.data_ptr():
                        self._src[kk] = ww.detach()
                        self._dirty = True
                self.pack()
                for kk in self.packs:
                    ww = self.params[kk[0] + ".weight"]
                    self._stamp[kk] = (ww.data_ptr(), ww._version)
                return self.packs[k]
            del self.packs[k]   # re-homed: a new copy from the new storage (table rebuilt) below
        buf = super().packed(key, mode)
        self._stamp[k] = stamp
        return buf


class Runtime:
    """Per-module HIP state: spec, compute dtype, live packed weights."""

    def __init__(self, module: torch.nn.Module, spec: NetSpec, dtype: torch.dtype):
        self.spec = spec
        self.dtype = dtype
        self.module = module
        self.weights = None
        self.shared: dict = {}            # eager contexts' long-lived state (fused-RCAB workspace)
        # the caller's grad mode (set by the module's forward: inside Function.forward grad mode
        # is always off, and ctx.needs_input_grad stays True for parameters under no_grad)
        self.grad_mode = True

    def wt(self, device) -> LiveWeights:
        if self.weights is None or self.weights.device != device:
            self.weights = LiveWeights(dict(self.module.named_parameters()), self.dtype, device)
        self.weights.refresh()
        return self.weights

    def ctx(self, device) -> Ctx:
        return Ctx(self.dtype, device, shared=self.shared)


def _check_input(x: torch.Tensor):
    if not x.is_cuda:
        raise RuntimeError("the HIP backend runs on a ROCm GPU tensor (got a CPU tensor); there is no CPU path")


def _check_grad(rt: "Runtime"):
    """fp16 is an inference precision here: the reference trains fp16 only under a GradScaler
    (trainer.py:227,482-503), and unscaled fp16 activation gradients underflow (the L1
    gradient of a B=32 256x256 batch is 1.6e-7, a subnormal)."""
    if rt.dtype == torch.float16:
        raise NotImplementedError("precision='fp16' is inference-only on the HIP backend; train in 'bf16' or 'fp32'")


# ---------------------------------------------------------------- FaceEnhanceNet pieces
class HeadFn(torch.autograd.Function):
    """conv_first (custom.py:164)."""

    @staticmethod
    def forward(ctx, x, w, b, rt: Runtime):
        _check_input(x)
        if x.requires_grad:
            raise NotImplementedError("gradient w.r.t. the LR input image is not provided by the HIP backend")
        x = x.contiguous().float()
        W = rt.wt(x.device)
        c = rt.ctx(x.device)
        feat = Forward(rt.spec, c, W, save=False).head(x)
        ctx.rt = rt
        ctx.save_for_backward(x)
        return as_nchw(feat)

    @staticmethod
    def backward(ctx, d):
        _check_grad(ctx.rt)
        (x,) = ctx.saved_tensors
        rt = ctx.rt
        c = rt.ctx(x.device)
        G = {"conv_first.weight": torch.empty_like(rt.module.conv_first.weight),
             "conv_first.bias": torch.empty_like(rt.module.conv_first.bias)}
        Backward(rt.spec, c, rt.wt(x.device), G).head(x, to_nhwc(d, rt.dtype))
        return None, G["conv_first.weight"], G["conv_first.bias"], None


class GroupFn(torch.autograd.Function):
    """ResidualGroup (blocks.py:185-189) over its own parameters (keys relative to the group)."""

    @staticmethod
    def forward(ctx, x, rt: Runtime, attn, *params):
        _check_input(x)
        L.check_strip_status()      # an earlier strip launch's timed-out wait raises here
        xh = to_nhwc(x, rt.dtype)
        W = rt.wt(x.device)
        c = rt.ctx(x.device)
        fw = Forward(rt.spec, c, W, save=rt.grad_mode and any(ctx.needs_input_grad), attn=attn)
        y, sv = fw.group(xh, 0, pre="")
        ctx.rt, ctx.sv = rt, sv
        return as_nchw(y)

    @staticmethod
    def backward(ctx, dy):
        _check_grad(ctx.rt)
        L.check_strip_status()
        rt, sv = ctx.rt, ctx.sv
        dyh = to_nhwc(dy, rt.dtype)
        c = rt.ctx(dy.device)
        named = list(rt.module.named_parameters())
        G = {k: torch.empty_like(p) for k, p in named}
        dx = Backward(rt.spec, c, rt.wt(dy.device), G).group(sv, dyh, 0, pre="")
        ctx.sv = None
        return (as_nchw(dx), None, None) + tuple(G[k] for k, _ in named)


class TailFn(torch.autograd.Function):
    """conv_after_body + skip, upsampler, conv_last + bicubic skip (+ eval clamp)
    (custom.py:158-161, 172-188)."""

    @staticmethod
    def forward(ctx, feat, feat0, x, rt: Runtime, clamp: bool, *params):
        fh = to_nhwc(feat, rt.dtype)
        f0 = to_nhwc(feat0, rt.dtype)
        W = rt.wt(feat.device)
        c = rt.ctx(feat.device)
        out, sv = Forward(rt.spec, c, W, save=rt.grad_mode).tail(fh, f0, x, training=not clamp)
        ctx.rt, ctx.sv = rt, sv
        return out

    @staticmethod
    def backward(ctx, dout):
        _check_grad(ctx.rt)
        rt, sv = ctx.rt, ctx.sv
        s = rt.spec
        B, Co, Ho, Wo = dout.shape
        c = rt.ctx(dout.device)
        d16 = torch.empty(B, Ho, Wo, 16, dtype=rt.dtype, device=dout.device)
        dd = dout.contiguous().float()
        c.emit("nchw_to_nhwc", c.lib.fen_nchw_to_nhwc, c.code, B, Co, Ho, Wo, 16, ptr(dd), ptr(d16))
        sv["dout"] = d16
        names = [k for k, _ in rt.module.named_parameters()
                 if k.startswith(("conv_after_body.", "upsample.", "conv_last."))]
        params = dict(rt.module.named_parameters())
        G = {k: torch.empty_like(params[k]) for k in names}
        d_body = Backward(s, c, rt.wt(dout.device), G).tail(sv)
        d_fb = sv["d_fb"]
        ctx.sv = None
        return (as_nchw(d_body), as_nchw(d_fb), None, None, None) + tuple(G[k] for k in names)


# ---------------------------------------------------------------- standalone blocks
class RCABFn(torch.autograd.Function):
    """RCAB (blocks.py:135-153) used on its own."""

    @staticmethod
    def forward(ctx, x, rt: Runtime, *params):
        _check_input(x)
        xh = to_nhwc(x, rt.dtype)
        c = rt.ctx(x.device)
        y, sv = Forward(rt.spec, c, rt.wt(x.device), save=rt.grad_mode).rcab(xh, "")
        ctx.rt, ctx.sv = rt, sv
        return as_nchw(y)

    @staticmethod
    def backward(ctx, dy):
        _check_grad(ctx.rt)
        rt, sv = ctx.rt, ctx.sv
        c = rt.ctx(dy.device)
        named = list(rt.module.named_parameters())
        G = {k: torch.empty_like(p) for k, p in named}
        dx = Backward(rt.spec, c, rt.wt(dy.device), G).rcab(sv, to_nhwc(dy, rt.dtype), "")
        ctx.sv = None
        return (as_nchw(dx), None) + tuple(G[k] for k, _ in named)


class ChannelAttentionFn(torch.autograd.Function):
    """ChannelAttention (blocks.py:75-92): y = t * sigmoid(W2 relu(W1 mean_hw(t)))."""

    @staticmethod
    def forward(ctx, t, w1, w2, rt: Runtime):
        _check_input(t)
        th = to_nhwc(t, rt.dtype)
        B, H, W, C = th.shape
        Cr = w1.shape[0]
        c = rt.ctx(t.device)
        npart = c.lib.fen_pool_parts(H * W)
        part = c.alloc((B * npart, C), torch.float32)
        c.emit("pool_dot", c.lib.fen_pool_dot, c.code, B, H * W, C, ptr(th), 0, ptr(part))
        mean = c.alloc((B, C), torch.float32)
        hid = c.alloc((B, Cr), torch.float32)
        s = c.alloc((B, C), torch.float32)
        w1c, w2c = w1.detach().contiguous(), w2.detach().contiguous()
        c.emit("se_fwd", c.lib.fen_se_fwd, B, C, Cr, npart, 1.0 / (H * W), ptr(part), ptr(w1c), ptr(w2c), ptr(mean),
               ptr(hid), ptr(s))
        zero = c.zeros(th.shape)
        y = c.alloc(th.shape)
        c.emit("se_apply", c.lib.fen_se_apply, c.code, B, H * W, C, ptr(th), ptr(s), 1.0, ptr(zero), ptr(y))
        ctx.rt = rt
        ctx.save_for_backward(th, mean, hid, s, w1c, w2c)
        ctx.s = s
        return as_nchw(y)

    @staticmethod
    def backward(ctx, dy):
        _check_grad(ctx.rt)
        th, mean, hid, s, w1, w2 = ctx.saved_tensors
        rt = ctx.rt
        B, H, W, C = th.shape
        Cr = w1.shape[0]
        c = rt.ctx(dy.device)
        dyh = to_nhwc(dy, rt.dtype)
        npart = c.lib.fen_pool_parts(H * W)
        part = c.alloc((B * npart, C), torch.float32)
        c.emit("pool_dot", c.lib.fen_pool_dot, c.code, B, H * W, C, ptr(dyh), ptr(th), ptr(part))
        g = c.alloc((B, C), torch.float32)
        dw1p = c.alloc((B, Cr * C), torch.float32)
        dw2p = c.alloc((B, Cr * C), torch.float32)
        c.emit("se_bwd", c.lib.fen_se_bwd, B, C, Cr, npart, 1.0 / (H * W), 1.0, ptr(part), ptr(mean), ptr(hid), ptr(s),
               ptr(w1), ptr(w2), ptr(g), ptr(dw1p), ptr(dw2p))
        dw1 = torch.empty_like(w1)
        dw2 = torch.empty_like(w2)
        colsum(c, dw1p, B, Cr * C, dw1)
        colsum(c, dw2p, B, Cr * C, dw2)
        dt = c.alloc(th.shape)
        c.emit("se_bwd_apply", c.lib.fen_se_bwd_apply, c.code, B, H * W, C, ptr(dyh), ptr(s), 1.0, ptr(g), ptr(dt))
        return as_nchw(dt), dw1, dw2, None


class UpsampleFn(torch.autograd.Function):
    """UpsampleModule (blocks.py:230-263): log2(scale) x [conv C->4C, PixelShuffle(2), PReLU]."""

    @staticmethod
    def forward(ctx, x, rt: Runtime, *params):
        _check_input(x)
        h = to_nhwc(x, rt.dtype)
        c = rt.ctx(x.device)
        W = rt.wt(x.device)
        p = W.p
        B, hh, ww, C = h.shape
        stages = []
        for st in range(rt.spec.n_stages):
            key = f"stages.{st}."
            a = c.alloc((B, 2 * hh, 2 * ww, C))
            v = c.alloc((B, 2 * hh, 2 * ww, C))
            from .net import conv
            conv(c, h, W.packed(key + "conv", 1), B, hh, ww, C, 4 * C, bias=p[key + "conv.bias"],
                 epi=L.EPI_PRELU | L.EPI_SHUFFLE, alpha=p[key + "prelu.weight"], y=a, y_pre=v)
            stages.append(dict(x=h, v=v, H=hh, W=ww))
            h, hh, ww = a, 2 * hh, 2 * ww
        ctx.rt, ctx.stages = rt, stages
        return as_nchw(h)

    @staticmethod
    def backward(ctx, dy):
        _check_grad(ctx.rt)
        from .net import conv
        rt, stages = ctx.rt, ctx.stages
        c = rt.ctx(dy.device)
        W = rt.wt(dy.device)
        p = W.p
        named = list(rt.module.named_parameters())
        G = {k: torch.empty_like(q) for k, q in named}
        d = to_nhwc(dy, rt.dtype)
        B, Ho, Wo, C = d.shape
        n = len(stages)
        last = stages[-1]
        du = c.alloc((B, last["H"], last["W"], 4 * C))
        dal = c.alloc((B * tiles(Ho, Wo), C), torch.float32)
        c.emit("prelu_bwd_unshuffle", c.lib.fen_prelu_bwd_unshuffle, c.code, B, Ho, Wo, C, ptr(d), ptr(last["v"]),
               ptr(p[f"stages.{n - 1}.prelu.weight"]), ptr(du), ptr(dal))
        colsum(c, dal, B * tiles(Ho, Wo), C, G[f"stages.{n - 1}.prelu.weight"])
        for st in reversed(range(n)):
            info = stages[st]
            key = f"stages.{st}."
            hh, ww = info["H"], info["W"]
            wgrad(c, info["x"], du, B, hh, ww, C, 4 * C, G[key + "conv.weight"], G[key + "conv.bias"])
            if st > 0:
                prev = stages[st - 1]
                du_prev = c.alloc((B, prev["H"], prev["W"], 4 * C))
                dal = c.alloc((B * tiles(hh, ww), C), torch.float32)
                conv(c, du, W.packed(key + "conv", 2), B, hh, ww, 4 * C, C, epi=L.EPI_PRELU_BWD | L.EPI_UNSHUFFLE,
                     alpha=p[f"stages.{st - 1}.prelu.weight"], pre_in=prev["v"], y=du_prev, part=dal)
                colsum(c, dal, B * tiles(hh, ww), C, G[f"stages.{st - 1}.prelu.weight"])
                du = du_prev
            else:
                dx = c.alloc((B, hh, ww, C))
                conv(c, du, W.packed(key + "conv", 2), B, hh, ww, 4 * C, C, y=dx)
        ctx.stages = None
        return (as_nchw(dx), None) + tuple(G[k] for k, _ in named)
