"""FaceEnhanceNet forward / backward as sequences of C-ABI launches.

One builder, used two ways (program.Ctx): eagerly by the nn.Module autograd Functions
(src/models) and recorded once into static programs by the training/inference engine
(engine.py).  Activations are NHWC tensors of the compute dtype; parameters and their
gradients are the reference's fp32 OIHW tensors, addressed by state_dict key.

Reference structure followed (tomasz-pres/face-super-resolution):
  FaceEnhanceNet.forward   src/models/custom.py:147-190
  ResidualGroup.forward    src/models/blocks.py:185-189
  RCAB.forward             src/models/blocks.py:135-153
  ChannelAttention.forward src/models/blocks.py:75-92
  PixelShuffleUpsample     src/models/blocks.py:223-227
and their autograd backward (trainer.py:482-485).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import torch

from . import lib as L
from .program import Ctx, byref, ptr


@dataclass(frozen=True)
class NetSpec:
    C: int = 64
    G: int = 3
    NB: int = 4
    Cr: int = 16
    scale: int = 4
    res_scale: float = 0.2
    in_ch: int = 3
    out_ch: int = 3

    @property
    def n_stages(self) -> int:
        return int(round(math.log2(self.scale)))

    @staticmethod
    def from_config(cfg) -> "NetSpec":
        # reduced channels rule of blocks.py:62
        return NetSpec(C=cfg.num_channels, G=cfg.num_groups, NB=cfg.blocks_per_group,
                       Cr=max(cfg.num_channels // cfg.reduction_ratio, 8), scale=cfg.scale_factor,
                       res_scale=float(cfg.res_scale), in_ch=cfg.in_channels, out_ch=cfg.out_channels)


# RCAB chain implementation (FEN_RCAB): 'deferred' (default) -- fen_rcab_deferred, one launch
# per RCAB whose SE gate is applied by the next launch (the chain end by fen_se_fused), no
# in-launch synchronisation between blocks; 'perop' -- conv1(+PReLU) / conv2(+pool) / SE
# launches (shapes outside the deferred kernel's envelope always take this path).
RCAB_MODE = os.environ.get("FEN_RCAB", "deferred")
# a ResidualGroup's end on the deferred path: the last RCAB's gate + residual and the group conv
# in one fen_rcab_group_end launch ('fused', default) or fen_se_fused + fen_conv3x3 ('split')
GROUP_END_FUSED = os.environ.get("FEN_GROUP_END", "fused") != "split"
# inference: a whole ResidualGroup as ONE persistent strip-resident launch (fen_group_strip,
# group_strip.hip) where its envelope holds (16-bit, 64 ch, W = 64, H % 8 == 0); FEN_GROUP_STRIP=0
# selects the per-RCAB deferred launches
GROUP_STRIP = os.environ.get("FEN_GROUP_STRIP", "1") != "0"
# ... and the training forward too (the kernel then writes the backward's saved tensors);
# FEN_GROUP_STRIP_TRAIN=0 keeps training on the per-RCAB launches
GROUP_STRIP_TRAIN = os.environ.get("FEN_GROUP_STRIP_TRAIN", "1") != "0"
# inference: the body's G groups as ONE fen_group_strip_chain launch (strips stay on their CUs
# across groups); FEN_GROUP_CHAIN=0 keeps a fen_group_strip launch per group
GROUP_CHAIN = os.environ.get("FEN_GROUP_CHAIN", "1") != "0"
# ... and the training forward too (the launch writes every group's saved set);
# FEN_GROUP_CHAIN_TRAIN=0 keeps a training launch per group
GROUP_CHAIN_TRAIN = os.environ.get("FEN_GROUP_CHAIN_TRAIN", "1") != "0"
# ... with conv_after_body as the chain's last step (a group of no RCABs); FEN_CHAIN_AFTER_BODY=0
# keeps it a conv launch of its own
CHAIN_AFTER_BODY = os.environ.get("FEN_CHAIN_AFTER_BODY", "1") != "0"
# inference at 128 channels (BASELINE configs[4]): a ResidualGroup as 2 * nb + 1 fen_rcab_c128
# launches (rcab128.hip: each RCAB's gate deferred into the next conv's input, its pool sums in
# conv2's epilogue) where the envelope holds (16-bit, H % 4 == 0, W % 64 == 0, Cr <= 32);
# FEN_RCAB_C128=0 selects the per-op launches
RCAB_C128 = os.environ.get("FEN_RCAB_C128", "1") != "0"
# RCAB backward: the SE backward and its apply as one fen_se_bwd_fused launch (default) or
# the fen_se_bwd + fen_se_bwd_apply pair (FEN_SE_BWD=pair; shapes outside the fused
# kernel's envelope always take the pair)
SE_BWD_FUSED = os.environ.get("FEN_SE_BWD", "fused") != "pair"
# inference: the upsampler and conv_last run over the batch in chunks of this many images, so a
# chunk's x2 / x4 activations (16.8 + 67 MB per 8 images at 64 -> 256) are written and re-read
# while they sit in the 256-MB Infinity Cache instead of making a round trip through HBM
# (0 = the whole batch in one pass)
TAIL_CHUNK = int(os.environ.get("FEN_TAIL_CHUNK", "0"))
# training: the upsampler stages' pre-activations are not saved where the PReLU slopes are > 0
# (their 4-channel groups); the backward recovers v = a > 0 ? a : a / alpha from the stage
# output a (fen_conv_desc.pre_elide / post_in) -- 268 + 67 MB fewer writes and reads per step
# at B=32; FEN_PRE_ELIDE=0 saves and reads v as before
PRE_ELIDE = os.environ.get("FEN_PRE_ELIDE", "1") != "0"


def tiles(H: int, W: int) -> int:
    return ((H + 15) // 16) * ((W + 15) // 16)


class Weights:
    """fp32 parameters (by state_dict key) + their packed kernel-layout copies.  `pack()`
    refreshes every packed copy in ONE launch (fen_pack_multi over a device job table)."""

    def __init__(self, params: Dict[str, torch.Tensor], dtype: torch.dtype, device):
        self.p = params
        self.dtype = dtype
        self.device = device
        self.packs: Dict[tuple, torch.Tensor] = {}
        self.pack_ctx = Ctx(dtype, device, record=True)
        self._src: Dict[tuple, torch.Tensor] = {}
        self._table = None        # (device job table, njobs, total elements)
        self._dirty = True

    def packed(self, key: str, mode: int) -> torch.Tensor:
        k = (key, mode)
        if k not in self.packs:
            w = self.p[key + ".weight"]
            cout, cin = int(w.shape[0]), int(w.shape[1])
            lib = self.pack_ctx.lib
            n = lib.fen_packed_elems(mode, cout, cin)
            buf = torch.empty(n, dtype=self.dtype, device=self.device)
            args = (L.dtype_code(self.dtype), mode, cout, cin, ptr(w), ptr(buf))
            # pack now, so a buffer is valid from the moment a builder sees it
            L.check(lib.fen_pack_conv_w(*args, torch.cuda.current_stream().cuda_stream), "pack_conv_w")
            self.packs[k] = buf
            self._src[k] = w
            self._dirty = True
        return self.packs[k]

    def _build_table(self) -> None:
        lib = self.pack_ctx.lib
        keys = list(self.packs)
        jobs = (L.PackJob * len(keys))()
        for i, k in enumerate(keys):
            w = self._src[k]
            jobs[i].w, jobs[i].out = ptr(w), ptr(self.packs[k])
            jobs[i].mode, jobs[i].Cout, jobs[i].Cin = k[1], int(w.shape[0]), int(w.shape[1])
        nbytes = lib.fen_pack_table_bytes(len(keys))
        host = (ctypes.c_uint8 * nbytes)()
        total = ctypes.c_size_t(0)
        L.check(lib.fen_pack_table(L.dtype_code(self.dtype), len(keys), ctypes.cast(jobs, ctypes.c_void_p),
                                   ctypes.cast(host, ctypes.c_void_p), ctypes.byref(total)), "pack_table")
        dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(self.device)
        self._table = (dev, len(keys), int(total.value))
        self._dirty = False

    def pack(self) -> None:
        if not self.packs:
            return
        if self._dirty:
            self._build_table()
        dev, nj, total = self._table
        L.check(self.pack_ctx.lib.fen_pack_multi(L.dtype_code(self.dtype), nj, dev.data_ptr(), total,
                                                 torch.cuda.current_stream().cuda_stream), "pack_multi")


# --------------------------------------------------------------------------------------
# primitive emitters
# --------------------------------------------------------------------------------------
def conv(ctx: Ctx, x, wpk, B, H, W, Cin, Cout, *, bias=None, epi=0, alpha=None, y=None, y_pre=None,
         res: Sequence = (), pre_in=None, part=None, lr=None, scale=0, clamp=0, hr=None, dout=None,
         l1_scale=0.0, loss_part=None, debug=0, s2d_in=0, s2d_out=0, pre_elide=0, post_in=None,
         y_pool=None, y_images=0) -> None:
    d = L.ConvDesc()
    d.dtype, d.B, d.H, d.W, d.Cin, d.Cout = ctx.code, B, H, W, Cin, Cout
    d.x, d.w, d.bias = ptr(x), ptr(wpk), ptr(bias)
    d.epi = epi | (L.EPI_BIAS if bias is not None else 0)
    d.alpha, d.y, d.y_pre = ptr(alpha), ptr(y), ptr(y_pre)
    for i, r in enumerate(res):
        d.res[i] = ptr(r)
    d.pre_in, d.part = ptr(pre_in), ptr(part)
    d.lr, d.scale, d.clamp, d.hr, d.dout = ptr(lr), scale, clamp, ptr(hr), ptr(dout)
    d.l1_scale, d.loss_part = float(l1_scale), ptr(loss_part)
    d.debug = debug
    d.s2d_in, d.s2d_out = s2d_in, s2d_out
    d.pre_elide, d.post_in = int(pre_elide), ptr(post_in)
    d.y_pool, d.y_images = ptr(y_pool), int(y_images)
    ctx.emit("conv3x3", ctx.lib.fen_conv3x3, byref(d))


# stride-2 3x3 conv as a stride-1 conv over the space-to-depth input (fen_s2d2): filter tap
# (kh, kw) -> (input phase (a, b), tap (kh', kw')) of the phase-major filter
#   kh = 0 -> a = 1, kh' = 0;  kh = 1 -> a = 0, kh' = 1;  kh = 2 -> a = 1, kh' = 1  (kw likewise)
def s2d_filter(w: torch.Tensor) -> torch.Tensor:
    """OIHW fp32 [Cout, C, 3, 3] (GPU) -> the phase-major [Cout, 4C, 3, 3] filter (fen_s2d_filter,
    zeros where no tap lands), on the current stream."""
    w = w.contiguous()
    co, c = int(w.shape[0]), int(w.shape[1])
    out = torch.empty(co, 4 * c, 3, 3, dtype=torch.float32, device=w.device)
    L.check(L.load().fen_s2d_filter(co, c, w.data_ptr(), out.data_ptr(), 0, torch.cuda.current_stream().cuda_stream),
            "s2d_filter")
    return out


def s2d_filter_grad(g4: torch.Tensor, out: torch.Tensor) -> None:
    """The phase-major filter's gradient [Cout, 4C, 3, 3] -> the OIHW gradient (into out)."""
    co, c = int(out.shape[0]), int(out.shape[1])
    L.check(L.load().fen_s2d_filter(co, c, g4.contiguous().data_ptr(), out.data_ptr(), 1,
                                    torch.cuda.current_stream().cuda_stream), "s2d_filter_grad")


def wgrad(ctx: Ctx, x, dy, B, H, W, Cin, Cout, dw, db, cout_valid=None) -> None:
    d = L.WgradDesc()
    d.dtype, d.B, d.H, d.W, d.Cin, d.Cout = ctx.code, B, H, W, Cin, Cout
    d.cout_valid = Cout if cout_valid is None else cout_valid
    d.x, d.dy, d.dw, d.db, d.accumulate = ptr(x), ptr(dy), ptr(dw), ptr(db), 0
    nwork = ctx.lib.fen_wgrad_work_floats(byref(d))
    work = ctx.scratch("wgrad_work", (nwork,), torch.float32)
    d.work = ptr(work)
    ctx.emit("wgrad3x3", ctx.lib.fen_wgrad3x3, byref(d))


# weight gradients of the RCAB convs issued per launch (fen_wgrad3x3_multi jobs, <= 8): the
# jobs share the CUs, so the per-block fp32 slabs shrink by that factor (FEN_WGRAD_BATCH=1:
# one launch per conv)
# RCAB backward data gradients: both convs (+ PReLU backward, + dy, + the next DOT partials) in
# one fen_rcab_bwd launch where the deferred kernel's envelope holds ('fused', default), or the
# conv2 dgrad (PReLU-backward epilogue) + conv1 dgrad (residual epilogue) pair (FEN_RCAB_BWD=pair)
RCAB_BWD_FUSED = os.environ.get("FEN_RCAB_BWD", "fused") != "pair"
# sum(dy * t) of the SE backward from the producing dgrad's epilogue (FEN_EPI_DOT) instead of
# a fen_pool_dot pass over dy and t (FEN_SE_DOT=pass: the separate pass)
DOT_FUSED = os.environ.get("FEN_SE_DOT", "fused") != "pass"
# the SE backward folded into the fused RCAB backward launch where its envelope holds (the DOT
# partials from dy's producer, <= 6 tiles per CU): 'fold' (default) or a separate
# fen_se_bwd_fused launch (FEN_SE_IN_BWD=launch)
SE_IN_BWD = os.environ.get("FEN_SE_IN_BWD", "fold") != "launch"
# a group's first RCAB (dx also carries the group's output gradient) on the fused backward too,
# the second residual in the DOT operand's slot (FEN_RCAB_BWD_RES=1).  Measured 8.838 vs
# 8.826 ms per training step against the two-launch pair (3 same-box reps): off by default
BWD_RES_FUSED = os.environ.get("FEN_RCAB_BWD_RES", "0") == "1"
WGRAD_BATCH = max(1, min(8, int(os.environ.get("FEN_WGRAD_BATCH", "8"))))
# ... on the strip backward: the group's 21 weight gradients in batches of FEN_WGRAD_STRIP_BATCH
# (the group conv's first), by default all 21 in one launch (252 blocks of 43 tiles, 3x fewer
# fp32 slabs than batches of 8): 6.67-6.68 vs 6.87-6.90 ms per stage-1 step at 8 and 6.81 at 11
# (same box, 3 reps each), once the launch geometry stopped spilling past 256 blocks
WGRAD_STRIP_BATCH = max(1, min(32, int(os.environ.get("FEN_WGRAD_STRIP_BATCH", "21"))))
# a ResidualGroup's whole backward (group conv^T, every RCAB's SE backward, conv2^T, PReLU',
# conv1^T) as ONE strip-resident fen_group_strip_bwd launch where its envelope holds (16-bit,
# 64 ch, W = 64, H % 8 == 0); FEN_GROUP_STRIP_BWD=0 selects the per-RCAB launches
GROUP_STRIP_BWD = os.environ.get("FEN_GROUP_STRIP_BWD", "1") != "0"
# conv_last's data, slope, weight and bias gradients as ONE fen_conv_last_bwd pass over the last
# stage's output (16-bit, 64 ch, whole 16x16 tiles, PRE_ELIDE); FEN_CL_BWD=0: the separate
# weight-gradient pass + fen_conv_last_dgrad
CL_BWD_FUSED = os.environ.get("FEN_CL_BWD", "1") != "0"
# FEN_CS_SIDE=1 (A/B only): a recorded strip-backward group issues its PReLU / SE column sums on a
# side stream, forked after the strip launch and joined before the group's end (its DP bucket
# mark, the next group's strip launch), beside the group's batched weight gradients instead of
# after them.  Measured slower: stage-1 step 5.603-5.623 vs 5.579-5.590 ms in line (the sums'
# blocks slow the weight gradients they share the CUs with by more than the 10 us they hide)
CS_SIDE = os.environ.get("FEN_CS_SIDE", "0") == "1"
# test-only fault injection for the strip kernels' bounded waits (fen_group_strip_desc.fault):
# bit 0 = the forward launches, bit 1 = the backward launches skip one hand-off flag in one
# strip, so its neighbour's wait times out and the launch reports through the status word
# (lib.check_strip_status).  Read when a launch is built; 0 in production.
GS_FAULT = 0


class WgradBatch:
    """Weight gradients of one shape queued by the backward builder and issued as ONE
    fen_wgrad3x3_multi launch pair once `size` jobs are queued, on a shape change or at
    flush().  The caller keeps each job's x / dy alive (unwritten) until the flush."""

    def __init__(self, ctx: Ctx, size: int = WGRAD_BATCH):
        self.ctx, self.size = ctx, size
        self.jobs: List[L.WgradDesc] = []
        self.hold: List[torch.Tensor] = []   # eager mode: x / dy must outlive the launch

    def add(self, x, dy, B, H, W, Cin, Cout, dw, db) -> None:
        d = L.WgradDesc()
        d.dtype, d.B, d.H, d.W, d.Cin, d.Cout = self.ctx.code, B, H, W, Cin, Cout
        d.cout_valid = Cout
        d.x, d.dy, d.dw, d.db, d.accumulate = ptr(x), ptr(dy), ptr(dw), ptr(db), 0
        if self.jobs and (B, H, W, Cin, Cout) != (self.jobs[0].B, self.jobs[0].H, self.jobs[0].W,
                                                   self.jobs[0].Cin, self.jobs[0].Cout):
            self.flush()
        self.jobs.append(d)
        self.hold += [x, dy]
        if len(self.jobs) >= self.size:
            self.flush()

    def flush(self) -> None:
        if not self.jobs:
            return
        n = len(self.jobs)
        arr = (L.WgradDesc * n)(*self.jobs)
        nwork = self.ctx.lib.fen_wgrad_multi_work_floats(n, ctypes.cast(arr, ctypes.c_void_p))
        work = self.ctx.scratch("wgrad_work", (nwork,), torch.float32)
        arr[0].work = ptr(work)
        self.ctx.emit("wgrad3x3_multi", self.ctx.lib.fen_wgrad3x3_multi, n, ctypes.cast(arr, ctypes.c_void_p))
        self.ctx.keep(arr)
        self.jobs, self.hold = [], []


def colsum(ctx: Ctx, part, rows, cols, out, scale=1.0) -> None:
    ctx.emit("colsum", ctx.lib.fen_colsum, rows, cols, ptr(part), float(scale), ptr(out), 0)


class ColsumBatch:
    """Column sums queued by a backward builder and issued as ONE fen_colsum_multi launch
    (each job keeps its own partial buffer until the flush)."""

    MAX = 40

    def __init__(self, ctx: Ctx):
        self.ctx = ctx
        self.jobs: List[tuple] = []

    def add(self, part, rows, cols, out, scale=1.0) -> None:
        self.jobs.append((part, int(rows), int(cols), out, float(scale)))
        if len(self.jobs) == self.MAX:
            self.flush()

    def flush(self, stream=None) -> None:
        """stream: a torch stream to launch on instead of the program's (recorded programs)."""
        if not self.jobs:
            return
        arr = (L.ColsumJob * len(self.jobs))()
        for i, (part, rows, cols, out, scale) in enumerate(self.jobs):
            arr[i].part, arr[i].out, arr[i].rows, arr[i].cols = ptr(part), ptr(out), rows, cols
            arr[i].scale, arr[i].accumulate = scale, 0
        fn = self.ctx.lib.fen_colsum_multi
        if stream is not None:
            h, lib_fn = stream.cuda_stream, fn
            fn = lambda n, a, _s: lib_fn(n, a, h)      # noqa: E731  (the op's stream argument ignored)
        self.ctx.emit("colsum_multi", fn, len(self.jobs), ctypes.cast(arr, ctypes.c_void_p))
        self.ctx.keep(arr)
        self.jobs = []


# --------------------------------------------------------------------------------------
# forward
# --------------------------------------------------------------------------------------
class Forward:
    """Builds the forward of FaceEnhanceNet; with `save=True` keeps what backward needs."""

    def __init__(self, spec: NetSpec, ctx: Ctx, Wt: Weights, save: bool, attn: Optional[dict] = None):
        self.s, self.ctx, self.Wt, self.save = spec, ctx, Wt, save
        self.attn = attn  # optional {name: s[B,C]} capture (get_attention_maps, custom.py:192-230)

    def head(self, x: torch.Tensor) -> torch.Tensor:
        """conv_first on the NCHW fp32 LR input (custom.py:164)."""
        B, _, H, W = x.shape
        s, ctx, p = self.s, self.ctx, self.Wt.p
        feat = ctx.alloc((B, H, W, s.C))
        ctx.emit("conv_first_fwd", ctx.lib.fen_conv_first_fwd, ctx.code, B, s.in_ch, H, W, s.C, ptr(x),
                 ptr(p["conv_first.weight"]), ptr(p["conv_first.bias"]), ptr(feat))
        return feat

    def rcab(self, x: torch.Tensor, pre: str, out: Optional[torch.Tensor] = None, name: Optional[str] = None):
        """RCAB (blocks.py:135-153) -> (y, saved).  A one-RCAB chain on fen_rcab_deferred + the
        fen_se_fused gate/residual where the shape allows it, else conv1(+PReLU) / conv2(+pool) /
        SE gate+apply launches."""
        s, ctx, Wt, p = self.s, self.ctx, self.Wt, self.Wt.p
        B, H, W, C = x.shape
        if self._deferred_ok(x):
            y, saved = self._chain(x, [pre], [name], out)
            return y, saved[0]
        a1 = ctx.alloc(x.shape) if self.save else ctx.scratch("rcab_a1", x.shape)
        z1 = ctx.alloc(x.shape) if self.save else None
        conv(ctx, x, Wt.packed(pre + "conv1", 0), B, H, W, C, C, bias=p[pre + "conv1.bias"],
             epi=L.EPI_PRELU, alpha=p[pre + "prelu.weight"], y=a1, y_pre=z1)
        t = ctx.alloc(x.shape) if self.save else ctx.scratch("rcab_t", x.shape)
        T = tiles(H, W)
        part = ctx.scratch("pool_part", (B * T, C), torch.float32)
        conv(ctx, a1, Wt.packed(pre + "conv2", 0), B, H, W, C, C, bias=p[pre + "conv2.bias"],
             epi=L.EPI_POOL, y=t, part=part)
        if self.save:
            mean = ctx.alloc((B, C), torch.float32)
            hid = ctx.alloc((B, s.Cr), torch.float32)
            sg = ctx.alloc((B, C), torch.float32)
        else:
            mean = hid = None
            sg = ctx.scratch("se_s", (B, C), torch.float32)
        ca = pre + "channel_attention.fc."
        if self.attn is not None and name is not None:
            self.attn[name] = sg
        y = out if out is not None else ctx.alloc(x.shape)
        ctx.emit("se_fused", ctx.lib.fen_se_fused, ctx.code, B, H * W, C, s.Cr, T, 1.0 / (H * W), ptr(part),
                 ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"]), ptr(mean), ptr(hid), ptr(sg), ptr(t), s.res_scale,
                 ptr(x), ptr(y))
        saved = dict(x=x, z1=z1, a1=a1, t=t, mean=mean, hid=hid, s=sg) if self.save else dict(s=sg)
        return y, saved

    def _deferred_ok(self, x) -> bool:
        B, H, W, C = x.shape
        return RCAB_MODE == "deferred" and bool(self.ctx.lib.fen_rcab_deferred_supported(self.ctx.code, B, H, W, C,
                                                                                           self.s.Cr))

    def _chain(self, x: torch.Tensor, pres: Sequence[str], names: Sequence[Optional[str]],
               out: Optional[torch.Tensor] = None, gconv: Optional[dict] = None):
        """A chain of RCABs (blocks.py:135-153; a ResidualGroup's blocks, blocks.py:185-188) on
        fen_rcab_deferred: launch j computes t_j and its tile sums and applies RCAB j-1's gate to
        build x_j; the chain end's gate and residual are fen_se_fused -- or, with gconv = {w, b,
        res, y}, fen_rcab_group_end, which also runs the group conv (y = conv(chain out) + res;
        `out`, the chain's output, is then written only when given).  -> (y, [saved per RCAB])."""
        s, ctx, Wt, p = self.s, self.ctx, self.Wt, self.Wt.p
        B, H, W, C = x.shape
        T = tiles(H, W)
        n = len(pres)
        want_s = self.save or self.attn is not None
        saved: List[dict] = []
        prev = None
        for j, (pre, name) in enumerate(zip(pres, names)):
            d = L.RcabDeferredDesc()
            d.dtype, d.B, d.H, d.W, d.C, d.Cr = ctx.code, B, H, W, C, s.Cr
            d.res_scale, d.inv_hw = float(s.res_scale), 1.0 / (H * W)
            d.w1, d.b1 = ptr(Wt.packed(pre + "conv1", 0)), ptr(p[pre + "conv1.bias"])
            d.alpha = ptr(p[pre + "prelu.weight"])
            d.w2, d.b2 = ptr(Wt.packed(pre + "conv2", 0)), ptr(p[pre + "conv2.bias"])
            if prev is None:
                xin = x
                d.x = ptr(x)
            else:
                xin = ctx.alloc(x.shape) if self.save else ctx.scratch(f"rd_x{j & 1}", x.shape)
                ca = prev["pre"] + "channel_attention.fc."
                d.x, d.tp, d.pp = ptr(prev["x"]), ptr(prev["t"]), ptr(prev["part"])
                d.pfc1, d.pfc2 = ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"])
                d.ps, d.pmean, d.phid = ptr(prev["s"]), ptr(prev["mean"]), ptr(prev["hid"])
                d.xo = ptr(xin)
            t = ctx.alloc(x.shape) if self.save else ctx.scratch(f"rd_t{j & 1}", x.shape)
            part = (ctx.alloc((B * T, C), torch.float32) if self.save
                    else ctx.scratch(f"rd_p{j & 1}", (B * T, C), torch.float32))
            d.t, d.part = ptr(t), ptr(part)
            z1 = a1 = None
            if self.save:
                z1, a1 = ctx.alloc(x.shape), ctx.alloc(x.shape)
                d.z1, d.a1 = ptr(z1), ptr(a1)
            sg = ctx.alloc((B, C), torch.float32) if want_s else None
            mean = ctx.alloc((B, C), torch.float32) if self.save else None
            hid = ctx.alloc((B, s.Cr), torch.float32) if self.save else None
            ctx.emit("rcab_deferred", ctx.lib.fen_rcab_deferred, byref(d))
            if self.attn is not None and name is not None:
                self.attn[name] = sg
            prev = dict(pre=pre, x=xin, t=t, part=part, s=sg, mean=mean, hid=hid)
            saved.append(dict(x=xin, z1=z1, a1=a1, t=t, mean=mean, hid=hid, s=sg) if self.save else dict(s=sg))
        ca = prev["pre"] + "channel_attention.fc."
        if gconv is not None:
            d = L.RcabDeferredDesc()
            d.dtype, d.B, d.H, d.W, d.C, d.Cr = ctx.code, B, H, W, C, s.Cr
            d.res_scale, d.inv_hw = float(s.res_scale), 1.0 / (H * W)
            d.x, d.tp, d.pp = ptr(prev["x"]), ptr(prev["t"]), ptr(prev["part"])
            d.pfc1, d.pfc2 = ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"])
            d.ps, d.pmean, d.phid = ptr(prev["s"]), ptr(prev["mean"]), ptr(prev["hid"])
            d.xo = ptr(out)
            ctx.emit("rcab_group_end", ctx.lib.fen_rcab_group_end, byref(d), ptr(gconv["w"]), ptr(gconv["b"]),
                     ptr(gconv["res"]), ptr(gconv["y"]))
            return gconv["y"], saved
        # chain end: the last RCAB's gate + residual
        y = out if out is not None else ctx.alloc(x.shape)
        ctx.emit("se_fused", ctx.lib.fen_se_fused, ctx.code, B, H * W, C, s.Cr, T, 1.0 / (H * W), ptr(prev["part"]),
                 ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"]), ptr(prev["mean"]), ptr(prev["hid"]),
                 ptr(prev["s"]), ptr(prev["t"]), s.res_scale, ptr(prev["x"]), ptr(y))
        return y, saved

    def _strip_ok(self, x) -> bool:
        B, H, W, C = x.shape
        return (GROUP_STRIP and (not self.save or GROUP_STRIP_TRAIN) and self.s.NB > 0 and
                bool(self.ctx.lib.fen_group_strip_supported(self.ctx.code, B, H, W, C, self.s.Cr, self.s.NB)))

    def _group_strip(self, x: torch.Tensor, pre: str, names: Sequence[str], y: torch.Tensor) -> dict:
        """The whole group in one fen_group_strip launch: y = conv(chain(x)) + b + x; in training
        (self.save) the launch also writes every RCAB's x_j, z1, a1, t_j, s, mean, hid and the
        chain's output (the backward's operands, the per-RCAB launches' saved set)."""
        ctx = self.ctx
        B, H = x.shape[0], x.shape[1]
        d = L.GroupStripDesc()
        sv = self._group_strip_desc(d, x, pre, names, y)
        nbytes = int(ctx.lib.fen_group_strip_work_bytes(B, H))
        work = ctx.persistent_zeros(f"group_strip/{B}x{H}", nbytes)
        d.work, d.work_bytes = ptr(work), nbytes
        d.status, d.fault = L.strip_status_ptr(ctx.device), GS_FAULT & 1
        ctx.emit("group_strip", ctx.lib.fen_group_strip, byref(d))
        ctx.keep(d)
        return sv

    def fb_buffer(self, shape) -> torch.Tensor:
        """conv_after_body's output buffer (kept for backward in training)."""
        return self.ctx.alloc(shape) if self.save else self.ctx.scratch("tail_fb", shape)

    def fb_for_chain(self, x: torch.Tensor) -> Optional[torch.Tensor]:
        """conv_after_body's output buffer for body(fb=...) when the chained launch will compute
        it; None otherwise (tail() then allocates its own: nothing is held unused)."""
        return self.fb_buffer(x.shape) if (CHAIN_AFTER_BODY and self._chain_ok(x)) else None

    def _chain_ok(self, x) -> bool:
        return (GROUP_CHAIN and (not self.save or GROUP_CHAIN_TRAIN) and self.s.G > 1 and self._strip_ok(x) and
                not self._c128_ok(x))

    def body(self, x: torch.Tensor, outs: Sequence[torch.Tensor], fb: Optional[torch.Tensor] = None):
        """The body's ResidualGroups (custom.py:168-169, blocks.py:185-189 each) -> (h, saved per
        group); outs[g] is group g's output (consecutive outputs distinct, outs[0] not x; in
        training all distinct: each is the next group's saved input).  On the strip kernels: ONE
        fen_group_strip_chain launch (GROUP_CHAIN; training: GROUP_CHAIN_TRAIN, the launch also
        writes every group's saved set), each strip resident on its CU through all G groups;
        otherwise a launch (or chain) per group.  With `fb` given and the chain taken, the same
        launch also computes conv_after_body (custom.py:172-175: fb = conv(h) + b + x) into fb and
        self.fb_done is set (tail() then skips that conv)."""
        s, ctx = self.s, self.ctx
        self.fb_done = False
        if not self._chain_ok(x):
            saved, h = [], x
            for g in range(s.G):
                h, sv = self.group(h, g, out=outs[g])
                saved.append(sv)
            return h, saved
        B, H = x.shape[0], x.shape[1]
        G = s.G
        ds = (L.GroupStripDesc * G)()
        saved, h = [], x
        for g in range(G):
            names = [f"group{g}_rcab{b}" for b in range(s.NB)]
            saved.append(self._group_strip_desc(ds[g], h, f"residual_groups.{g}.", names, outs[g]))
            h = outs[g]
        nbytes = int(ctx.lib.fen_group_strip_chain_work_bytes(B, H, G))
        # the chain's own workspace (its parameter table is this program's)
        work = torch.zeros(nbytes, dtype=torch.uint8, device=ctx.device)
        ctx.keep(work)
        for g in range(G):
            ds[g].work, ds[g].work_bytes = ptr(work), nbytes
            ds[g].status, ds[g].fault = L.strip_status_ptr(ctx.device), GS_FAULT & 1
        tail = None
        if fb is not None and CHAIN_AFTER_BODY:
            tail = L.GroupStripChainTail()
            tail.w, tail.bias = ptr(self.Wt.packed("conv_after_body", 0)), ptr(self.Wt.p["conv_after_body.bias"])
            tail.skip, tail.y = ptr(x), ptr(fb)
            ctx.keep(tail)
        tp = byref(tail) if tail is not None else None
        L.check(ctx.lib.fen_group_strip_chain_prepare(ds, G, tp, torch.cuda.current_stream(ctx.device).cuda_stream),
                "group_strip_chain_prepare")
        ctx.emit("group_strip_chain", ctx.lib.fen_group_strip_chain, ds, G, tp)
        ctx.keep(ds)
        self.fb_done = tail is not None
        return h, saved

    def _group_strip_desc(self, d, x: torch.Tensor, pre: str, names: Sequence[str], y: torch.Tensor) -> dict:
        """Fill a fen_group_strip descriptor (all but the workspace) -> the group's saved set."""
        s, ctx, Wt, p = self.s, self.ctx, self.Wt, self.Wt.p
        B, H, W, C = x.shape
        d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.nb = ctx.code, B, H, W, C, s.Cr, s.NB
        d.res_scale = float(s.res_scale)
        d.x, d.y = ptr(x), ptr(y)
        blocks = []
        for b in range(s.NB):
            q = f"{pre}blocks.{b}."
            ca = q + "channel_attention.fc."
            d.w1[b], d.b1[b] = ptr(Wt.packed(q + "conv1", 0)), ptr(p[q + "conv1.bias"])
            d.alpha[b] = ptr(p[q + "prelu.weight"])
            d.w2[b], d.b2[b] = ptr(Wt.packed(q + "conv2", 0)), ptr(p[q + "conv2.bias"])
            d.fc1[b], d.fc2[b] = ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"])
            sg = None
            if self.attn is not None or self.save:
                sg = ctx.alloc((B, C), torch.float32)
                d.s_out[b] = ptr(sg)
                if self.attn is not None:
                    self.attn[names[b]] = sg
            if self.save:
                xb = x if b == 0 else ctx.alloc(x.shape)
                z1, a1, t = ctx.alloc(x.shape), ctx.alloc(x.shape), ctx.alloc(x.shape)
                mean, hid = ctx.alloc((B, C), torch.float32), ctx.alloc((B, s.Cr), torch.float32)
                d.sv_x[b], d.sv_z1[b], d.sv_a1[b], d.sv_t[b] = ptr(xb), ptr(z1), ptr(a1), ptr(t)
                d.sv_mean[b], d.sv_hid[b] = ptr(mean), ptr(hid)
                blocks.append(dict(x=xb, z1=z1, a1=a1, t=t, mean=mean, hid=hid, s=sg))
            else:
                blocks.append(dict(s=sg))
        x_last = None
        z1_elided = False
        if self.save:
            x_last = ctx.alloc(x.shape)
            d.save, d.x_last = 1, ptr(x_last)
            # z1 of an RCAB whose slopes are all > 0 is left unwritten when the backward will be
            # the strip backward, which recovers it from a1 (PRE_ELIDE)
            z1_elided = PRE_ELIDE and GROUP_STRIP_BWD and bool(
                ctx.lib.fen_group_strip_bwd_supported(ctx.code, B, H, W, C, s.Cr, s.NB))
            d.pre_elide = int(z1_elided)
        d.wg, d.bg = ptr(Wt.packed(pre + "conv", 0)), ptr(p[pre + "conv.bias"])
        return dict(blocks=blocks, x=x, x_last=x_last, z1_elided=z1_elided)

    def _c128_ok(self, x) -> bool:
        B, H, W, C = x.shape
        return (RCAB_C128 and not self.save and self.s.NB > 0 and
                bool(self.ctx.lib.fen_rcab_c128_supported(self.ctx.code, B, H, W, C, self.s.Cr)))

    def _group_c128(self, x: torch.Tensor, pre: str, names: Sequence[str], y: torch.Tensor) -> dict:
        """The group on fen_rcab_c128 (inference): per RCAB j a conv1 launch that builds x_j from
        x_{j-1} + rs * s_{j-1} * t_{j-1} while staging its input (writing x_j for the next
        combine) and a conv2 launch (t_j + its tile sums); the group conv applies the last
        gate the same way and adds the group's input."""
        s, ctx, Wt, p = self.s, self.ctx, self.Wt, self.Wt.p
        B, H, W, C = x.shape
        T = int(ctx.lib.fen_rcab_c128_tiles(H, W))
        blocks = []
        prev = None

        def desc(mode, xin, w, bias, yout):
            d = L.RcabC128Desc()
            d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.mode = ctx.code, B, H, W, C, s.Cr, mode
            d.res_scale = float(s.res_scale)
            d.x, d.w, d.bias, d.y = ptr(xin), ptr(w), ptr(bias), ptr(yout)
            return d

        def gate_from(d, pv):
            ca = pv["pre"] + "channel_attention.fc."
            d.tp, d.pp = ptr(pv["t"]), ptr(pv["part"])
            d.pfc1, d.pfc2 = ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"])
            if self.attn is not None:
                sg = ctx.alloc((B, C), torch.float32)
                self.attn[pv["name"]] = sg
                d.ps = ptr(sg)
                pv["blk"]["s"] = sg

        for j in range(s.NB):
            q = f"{pre}blocks.{j}."
            a1 = ctx.scratch("c128_a1", x.shape)
            if prev is None:
                d = desc(1, x, Wt.packed(q + "conv1", 0), p[q + "conv1.bias"], a1)
                xj = x
            else:
                xj = ctx.scratch(f"c128_x{j & 1}", x.shape)
                d = desc(1, prev["x"], Wt.packed(q + "conv1", 0), p[q + "conv1.bias"], a1)
                gate_from(d, prev)
                d.xo = ptr(xj)
            d.alpha = ptr(p[q + "prelu.weight"])
            ctx.emit("rcab_c128_conv1", ctx.lib.fen_rcab_c128, byref(d))
            ctx.keep(d)
            t = ctx.scratch(f"c128_t{j & 1}", x.shape)
            part = ctx.scratch(f"c128_p{j & 1}", (B * T, C), torch.float32)
            d = desc(2, a1, Wt.packed(q + "conv2", 0), p[q + "conv2.bias"], t)
            d.part = ptr(part)
            ctx.emit("rcab_c128_conv2", ctx.lib.fen_rcab_c128, byref(d))
            ctx.keep(d)
            blk = dict(s=None)
            blocks.append(blk)
            prev = dict(pre=q, x=xj, t=t, part=part, name=names[j], blk=blk)
        d = desc(3, prev["x"], Wt.packed(pre + "conv", 0), p[pre + "conv.bias"], y)
        gate_from(d, prev)
        d.res = ptr(x)
        ctx.emit("rcab_c128_group_conv", ctx.lib.fen_rcab_c128, byref(d))
        ctx.keep(d)
        return dict(blocks=blocks, x=x, x_last=None)

    def group(self, x: torch.Tensor, g: int, out: Optional[torch.Tensor] = None, pre: Optional[str] = None):
        """ResidualGroup (blocks.py:185-189) -> (y, saved)."""
        s, ctx, Wt, p = self.s, self.ctx, self.Wt, self.Wt.p
        B, H, W, C = x.shape
        pre = f"residual_groups.{g}." if pre is None else pre
        if self._c128_ok(x):
            y = out if out is not None and out.data_ptr() != x.data_ptr() else ctx.alloc(x.shape)
            names = [f"group{g}_rcab{b}" for b in range(s.NB)]
            return y, self._group_c128(x, pre, names, y)
        if self._strip_ok(x):
            y = out if out is not None and out.data_ptr() != x.data_ptr() else ctx.alloc(x.shape)
            names = [f"group{g}_rcab{b}" for b in range(s.NB)]
            return y, self._group_strip(x, pre, names, y)
        if self._deferred_ok(x) and s.NB > 0:
            pres = [f"{pre}blocks.{b}." for b in range(s.NB)]
            names = [f"group{g}_rcab{b}" for b in range(s.NB)]
            y = out if out is not None else ctx.alloc(x.shape)
            if GROUP_END_FUSED:
                # the chain's output (the group conv's input) is materialised only for backward
                y_last = ctx.alloc(x.shape) if self.save else None
                _, blocks = self._chain(x, pres, names, out=y_last,
                                        gconv=dict(w=Wt.packed(pre + "conv", 0), b=p[pre + "conv.bias"], res=x, y=y))
                return y, dict(blocks=blocks, x=x, x_last=y_last)
            y_last = ctx.alloc(x.shape) if self.save else ctx.scratch("rd_y", x.shape)
            h, blocks = self._chain(x, pres, names, out=y_last)
            conv(ctx, h, Wt.packed(pre + "conv", 0), B, H, W, C, C, bias=p[pre + "conv.bias"], y=y, res=(x,))
            return y, dict(blocks=blocks, x=x, x_last=h)
        blocks = []
        h = x
        for b in range(s.NB):
            nm = f"group{g}_rcab{b}"
            if self.save:
                h, sv = self.rcab(h, f"{pre}blocks.{b}.", name=nm)
            else:  # ping-pong two scratch buffers between blocks
                h, sv = self.rcab(h, f"{pre}blocks.{b}.", out=ctx.scratch(f"rg_pp{b & 1}", x.shape), name=nm)
            blocks.append(sv)
        y = out if out is not None else ctx.alloc(x.shape)
        conv(ctx, h, Wt.packed(pre + "conv", 0), B, H, W, C, C, bias=p[pre + "conv.bias"], y=y, res=(x,))
        return y, dict(blocks=blocks, x=x, x_last=h)

    def tail(self, feat: torch.Tensor, feat0: torch.Tensor, x_lr: torch.Tensor, training: bool,
             out: Optional[torch.Tensor] = None, hr: Optional[torch.Tensor] = None, l1_scale: float = 0.0,
             fb: Optional[torch.Tensor] = None):
        """conv_after_body + skip, upsampler, conv_last + bicubic skip (+ clamp / + L1 grad).
        fb given: conv_after_body's output, already computed (the chained body launch)."""
        s, ctx, Wt, p = self.s, self.ctx, self.Wt, self.Wt.p
        B, H, W, C = feat.shape
        fb_given = fb is not None
        if fb is None:
            fb = self.fb_buffer(feat.shape)

        def c128(hh_, ww_) -> bool:   # the 128-channel kernels (inference)
            return (RCAB_C128 and not self.save and
                    bool(ctx.lib.fen_rcab_c128_supported(ctx.code, B, hh_, ww_, C, max(s.Cr, 1))))

        def c128_launch(name, mode, x_, w_, bias_, y_, alpha_=None, res_=None, b_=None):
            d = L.RcabC128Desc()
            d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.mode = ctx.code, b_ or B, x_.shape[1], x_.shape[2], C, max(s.Cr, 1), mode
            d.res_scale = float(s.res_scale)
            d.x, d.w, d.bias, d.y = ptr(x_), ptr(w_), ptr(bias_), ptr(y_)
            d.alpha, d.res = ptr(alpha_), ptr(res_)
            ctx.emit(name, ctx.lib.fen_rcab_c128, byref(d))
            ctx.keep(d)

        if fb_given:
            pass
        elif c128(H, W):
            c128_launch("c128_after_body", 3, feat, Wt.packed("conv_after_body", 0), p["conv_after_body.bias"], fb,
                        res_=feat0)
        else:
            conv(ctx, feat, Wt.packed("conv_after_body", 0), B, H, W, C, C, bias=p["conv_after_body.bias"], y=fb,
                 res=(feat0,))
        if out is None:
            out = ctx.alloc((B, s.out_ch, H << s.n_stages, W << s.n_stages), torch.float32)
        bc = B
        if TAIL_CHUNK > 0 and not self.save and hr is None and B % TAIL_CHUNK == 0:
            bc = TAIL_CHUNK
        dout = loss_part = None
        for b0 in range(0, B, bc):
            h, hh, ww = fb[b0:b0 + bc], H, W
            stages = []
            for st in range(s.n_stages):
                key = f"upsample.stages.{st}."
                shp = (bc, 2 * hh, 2 * ww, C)
                a = ctx.alloc(shp) if self.save else ctx.scratch(f"up_a{st & 1}", shp)
                v = ctx.alloc(shp) if self.save else None
                if c128(hh, ww):
                    c128_launch("c128_upsample", 4, h, Wt.packed(key + "conv", 1), p[key + "conv.bias"], a,
                                alpha_=p[key + "prelu.weight"], b_=bc)
                else:
                    conv(ctx, h, Wt.packed(key + "conv", 1), bc, hh, ww, C, 4 * C, bias=p[key + "conv.bias"],
                         epi=L.EPI_PRELU | L.EPI_SHUFFLE, alpha=p[key + "prelu.weight"], y=a, y_pre=v,
                         pre_elide=PRE_ELIDE)
                stages.append(dict(x=h, v=v, a=a, H=hh, W=ww))
                h, hh, ww = a, 2 * hh, 2 * ww
            if hr is not None:
                dout = ctx.alloc((B, hh, ww, 16)) if self.save else ctx.scratch("dout", (B, hh, ww, 16))
                loss_part = ctx.scratch("loss_part", (B * tiles(hh, ww), 1), torch.float32)
            conv(ctx, h, Wt.packed("conv_last", 0), bc, hh, ww, C, s.out_ch, bias=p["conv_last.bias"],
                 epi=L.EPI_LAST, y=out[b0:b0 + bc], lr=x_lr[b0:b0 + bc], scale=s.scale, clamp=0 if training else 1,
                 hr=hr, dout=dout, l1_scale=l1_scale, loss_part=loss_part)
        saved = dict(feat=feat, fb=fb, stages=stages, a_last=h, dout=dout, loss_part=loss_part, Ho=hh, Wo=ww)
        return out, saved


# --------------------------------------------------------------------------------------
# backward
# --------------------------------------------------------------------------------------
class Backward:
    """Builds the backward; writes fp32 parameter gradients into G[state_dict key]."""

    def __init__(self, spec: NetSpec, ctx: Ctx, Wt: Weights, G: Dict[str, torch.Tensor]):
        self.s, self.ctx, self.Wt, self.G = spec, ctx, Wt, G
        self.cs = ColsumBatch(ctx)   # flushed at the end of every group / the tail
        # the side stream of the strip-backward groups' column sums (recorded programs only)
        self.side = (torch.cuda.Stream(device=ctx.device) if (CS_SIDE and ctx.record and torch.cuda.is_available())
                     else None)
        self.wb = WgradBatch(ctx)    # RCAB conv weight gradients; flushed with self.cs
        self._rc = 0                 # RCAB backward counter: rotates the dt / dz1 buffers
        # (partials, parts per image) of sum dy*t for the next rcab(), computed by the epilogue
        # of the dgrad that produced its dy (FEN_EPI_DOT) instead of a fen_pool_dot pass
        self._dot = None

    def _wg(self, key, x, dy, B, H, W, Cin, Cout, cout_valid=None):
        wgrad(self.ctx, x, dy, B, H, W, Cin, Cout, self.G[key + ".weight"], self.G.get(key + ".bias"), cout_valid)

    def _dot_conv(self, t_next, B, H, W, C) -> dict:
        """conv() kwargs that make a dgrad also emit sum(output * t_next) per tile and channel
        (the next rcab()'s SE-backward operand); {} without t_next."""
        if t_next is None or not DOT_FUSED:
            return {}
        T = tiles(H, W)
        part = self.ctx.scratch(f"bw_dot{self._rc & 1}", (B * T, C), torch.float32)
        self._dot = (part, T)
        return dict(epi=L.EPI_DOT, pre_in=t_next, part=part)

    def rcab(self, sv: dict, dy: torch.Tensor, pre: str, extra_res: Sequence = (), dx_out=None,
             flush: bool = True, t_next=None) -> torch.Tensor:
        """RCAB backward; its PReLU / SE weight-gradient column sums are queued on self.cs and
        issued at the end (flush=True) or by the caller (group() batches a whole group).
        t_next: the SE input t of the RCAB whose backward follows (its dy is this one's dx),
        dotted with dx in the conv1 dgrad's epilogue."""
        s, ctx, Wt, p, G = self.s, self.ctx, self.Wt, self.Wt.p, self.G
        B, H, W, C = dy.shape
        HW = H * W
        dot_part = self._dot is not None
        if dot_part:
            part, npart = self._dot          # sum dy*t per tile, from dy's producer
            self._dot = None
        else:
            npart = ctx.lib.fen_pool_parts(HW)
            part = ctx.scratch("bw_pool", (B * npart, C), torch.float32)
            ctx.emit("pool_dot", ctx.lib.fen_pool_dot, ctx.code, B, HW, C, ptr(dy), ptr(sv["t"]), ptr(part))
        dw1p = ctx.scratch("bw_dw1p" + pre, (B, s.Cr * C), torch.float32)
        dw2p = ctx.scratch("bw_dw2p" + pre, (B, s.Cr * C), torch.float32)
        ca = pre + "channel_attention.fc."
        # dt / dz1 stay untouched until the queued weight gradients that read them are issued:
        # a batch of n jobs spans at most n // 2 + 1 RCABs, so n rotating buffers suffice
        rot = self._rc % self.wb.size
        self._rc += 1
        dt = ctx.scratch(f"bw_dt{rot}", dy.shape)
        se_args = (npart, 1.0 / HW, s.res_scale, ptr(part), ptr(sv["mean"]), ptr(sv["hid"]), ptr(sv["s"]),
                   ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"]))
        # (one extra residual -- a group's first RCAB -- rides in the DOT operand's slot)
        fused = (RCAB_BWD_FUSED and len(extra_res) <= (1 if BWD_RES_FUSED else 0)
                 and not (extra_res and t_next is not None)
                 and ctx.code != L.F32
                 and ctx.lib.fen_rcab_deferred_supported(ctx.code, B, H, W, C, s.Cr))
        # the SE backward folded into the fused launch (dt built on its dy halo in LDS)
        seb = fused and SE_IN_BWD and dot_part and ctx.lib.fen_rcab_bwd_se_supported(ctx.code, B, H, W, C, s.Cr)
        if seb:
            pass                             # fen_rcab_bwd below writes dt, dw1p, dw2p
        elif SE_BWD_FUSED and C <= 64 and npart <= 64 and C * s.Cr <= 4096:
            # SE backward + dt in one launch (same arithmetic as the pair below)
            ctx.emit("se_bwd_fused", ctx.lib.fen_se_bwd_fused, ctx.code, B, HW, C, s.Cr, *se_args, ptr(dy), None,
                     ptr(dw1p), ptr(dw2p), ptr(dt))
        else:
            g = ctx.scratch("bw_g", (B, C), torch.float32)
            ctx.emit("se_bwd", ctx.lib.fen_se_bwd, B, C, s.Cr, *se_args, ptr(g), ptr(dw1p), ptr(dw2p))
            ctx.emit("se_bwd_apply", ctx.lib.fen_se_bwd_apply, ctx.code, B, HW, C, ptr(dy), ptr(sv["s"]), s.res_scale,
                     ptr(g), ptr(dt))
        self.cs.add(dw1p, B, s.Cr * C, G[ca + "0.weight"])
        self.cs.add(dw2p, B, s.Cr * C, G[ca + "2.weight"])
        # conv2's weight gradient reads dt: queued only once dt's producer is emitted (with the
        # SE fold that is fen_rcab_bwd below -- an add may flush the batch at once)
        if not seb:
            self.wb.add(sv["a1"], dt, B, H, W, C, C, G[pre + "conv2.weight"], G[pre + "conv2.bias"])
        dz1 = ctx.scratch(f"bw_dz1{rot}", dy.shape)
        T = tiles(H, W)
        dal = ctx.scratch("bw_dal" + pre, (B * T, C), torch.float32)
        dx = dx_out if dx_out is not None else ctx.alloc(dy.shape)
        if fused:
            d = L.RcabBwdDesc()
            d.dtype, d.B, d.H, d.W, d.C = ctx.code, B, H, W, C
            d.dt, d.w2t, d.z1 = ptr(dt), ptr(Wt.packed(pre + "conv2", 2)), ptr(sv["z1"])
            d.alpha, d.w1t, d.dy = ptr(p[pre + "prelu.weight"]), ptr(Wt.packed(pre + "conv1", 2)), ptr(dy)
            d.dz1, d.dalpha_part, d.dx = ptr(dz1), ptr(dal), ptr(dx)
            if extra_res:
                d.dres = ptr(extra_res[0])
            if seb:
                d.se_part, d.se_s, d.se_mean, d.se_hid = ptr(part), ptr(sv["s"]), ptr(sv["mean"]), ptr(sv["hid"])
                d.se_w1, d.se_w2 = ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"])
                d.se_dw1p, d.se_dw2p, d.se_res_scale, d.se_Cr = ptr(dw1p), ptr(dw2p), s.res_scale, s.Cr
            dk = self._dot_conv(t_next, B, H, W, C)
            if dk:
                d.dot_t, d.dot_part = ptr(dk["pre_in"]), ptr(dk["part"])
            ctx.emit("rcab_bwd", ctx.lib.fen_rcab_bwd, byref(d))
            if seb:
                self.wb.add(sv["a1"], dt, B, H, W, C, C, G[pre + "conv2.weight"], G[pre + "conv2.bias"])
            self.cs.add(dal, B * T, C, G[pre + "prelu.weight"])
            self.wb.add(sv["x"], dz1, B, H, W, C, C, G[pre + "conv1.weight"], G[pre + "conv1.bias"])
            if flush:
                self.flush()
            return dx
        conv(ctx, dt, Wt.packed(pre + "conv2", 2), B, H, W, C, C, epi=L.EPI_PRELU_BWD, alpha=p[pre + "prelu.weight"],
             pre_in=sv["z1"], y=dz1, part=dal)
        self.cs.add(dal, B * T, C, G[pre + "prelu.weight"])
        self.wb.add(sv["x"], dz1, B, H, W, C, C, G[pre + "conv1.weight"], G[pre + "conv1.bias"])
        conv(ctx, dz1, Wt.packed(pre + "conv1", 2), B, H, W, C, C, y=dx, res=(dy,) + tuple(extra_res),
             **self._dot_conv(t_next, B, H, W, C))
        if flush:
            self.flush()
        return dx

    def flush(self) -> None:
        self.wb.flush()
        self.cs.flush()

    def _strip_bwd_ok(self, sv: dict, dy: torch.Tensor, extra_res: Sequence) -> bool:
        B, H, W, C = dy.shape
        blocks = sv.get("blocks") or []
        ok = (GROUP_STRIP_BWD and self.s.NB > 0 and len(extra_res) <= 1 and self.ctx.code != L.F32
              and len(blocks) == self.s.NB and all(b.get("z1") is not None for b in blocks)
              and bool(self.ctx.lib.fen_group_strip_bwd_supported(self.ctx.code, B, H, W, C, self.s.Cr, self.s.NB)))
        if sv.get("z1_elided") and not ok:   # only the strip backward recovers an unwritten z1
            raise L.FenError("group backward: the forward elided z1 but the strip backward does not apply")
        return ok

    def _group_strip_bwd(self, sv: dict, dy: torch.Tensor, pre: str, extra_res: Sequence, dx_out) -> torch.Tensor:
        """The group's backward in one fen_group_strip_bwd launch (data gradients, SE backward,
        dt / dz1 for the weight gradients), then its weight gradients (8 per fen_wgrad3x3_multi
        launch) and the PReLU / SE column sums."""
        s, ctx, Wt, p, G = self.s, self.ctx, self.Wt, self.Wt.p, self.G
        B, H, W, C = dy.shape
        d = L.GroupStripBwdDesc()
        d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.nb = ctx.code, B, H, W, C, s.Cr, s.NB
        d.res_scale = float(s.res_scale)
        dx = dx_out if dx_out is not None else ctx.alloc(dy.shape)
        d.dy, d.dx = ptr(dy), ptr(dx)
        if extra_res:
            d.dres = ptr(extra_res[0])
        d.wgt = ptr(Wt.packed(pre + "conv", 2))
        outs = []
        drows = int(ctx.lib.fen_group_strip_bwd_dal_rows(B, H))    # one dalpha partial row per strip
        for b in range(s.NB):
            q = f"{pre}blocks.{b}."
            ca = q + "channel_attention.fc."
            blk = sv["blocks"][b]
            d.w1t[b], d.w2t[b] = ptr(Wt.packed(q + "conv1", 2)), ptr(Wt.packed(q + "conv2", 2))
            d.alpha[b] = ptr(p[q + "prelu.weight"])
            d.fc1[b], d.fc2[b] = ptr(p[ca + "0.weight"]), ptr(p[ca + "2.weight"])
            d.z1[b], d.t[b] = ptr(blk["z1"]), ptr(blk["t"])
            if PRE_ELIDE:
                d.a1[b] = ptr(blk["a1"])
            d.s[b], d.mean[b], d.hid[b] = ptr(blk["s"]), ptr(blk["mean"]), ptr(blk["hid"])
            o = dict(dt=ctx.scratch(f"gsb_dt{b}", dy.shape), dz1=ctx.scratch(f"gsb_dz1{b}", dy.shape),
                     dal=ctx.scratch(f"gsb_dal{b}", (drows, C), torch.float32),
                     dw1p=ctx.scratch(f"gsb_dw1p{b}", (B, s.Cr * C), torch.float32),
                     dw2p=ctx.scratch(f"gsb_dw2p{b}", (B, s.Cr * C), torch.float32))
            d.dt[b], d.dz1[b], d.dalpha_part[b] = ptr(o["dt"]), ptr(o["dz1"]), ptr(o["dal"])
            d.dw1p[b], d.dw2p[b] = ptr(o["dw1p"]), ptr(o["dw2p"])
            outs.append(o)
        nbytes = int(ctx.lib.fen_group_strip_bwd_work_bytes(B, H))
        work = ctx.persistent_zeros(f"group_strip_bwd/{B}x{H}", nbytes)
        d.work, d.work_bytes = ptr(work), nbytes
        d.status, d.fault = L.strip_status_ptr(ctx.device), (GS_FAULT >> 1) & 1
        ctx.emit("group_strip_bwd", ctx.lib.fen_group_strip_bwd, byref(d))
        ctx.keep(d)
        wb = self.wb
        size = getattr(wb, "size", None)
        if size is not None:   # this group's weight gradients in one batch
            wb.flush()
            wb.size = WGRAD_STRIP_BATCH
        # the column sums read only the strip launch's partials: on the side stream (when
        # recording, nothing else queued on self.cs) beside the weight gradients below
        side = self.side if (self.side is not None and not self.cs.jobs) else None
        for b in reversed(range(s.NB)):
            q = f"{pre}blocks.{b}."
            ca = q + "channel_attention.fc."
            o = outs[b]
            self.cs.add(o["dal"], drows, C, G[q + "prelu.weight"])
            self.cs.add(o["dw1p"], B, s.Cr * C, G[ca + "0.weight"])
            self.cs.add(o["dw2p"], B, s.Cr * C, G[ca + "2.weight"])
        if side is not None:
            ctx.mark("cs_fork", lambda: side.wait_stream(torch.cuda.current_stream(ctx.device)))
            self.cs.flush(stream=side)
        wb.add(sv["x_last"], dy, B, H, W, C, C, G[pre + "conv.weight"], G[pre + "conv.bias"])
        for b in reversed(range(s.NB)):
            q = f"{pre}blocks.{b}."
            blk, o = sv["blocks"][b], outs[b]
            wb.add(blk["a1"], o["dt"], B, H, W, C, C, G[q + "conv2.weight"], G[q + "conv2.bias"])
            wb.add(blk["x"], o["dz1"], B, H, W, C, C, G[q + "conv1.weight"], G[q + "conv1.bias"])
        wb.flush()
        if size is not None:
            wb.size = size
        self.flush()
        if side is not None:   # the group's gradients complete on the compute stream from here
            ctx.mark("cs_join", lambda: torch.cuda.current_stream(ctx.device).wait_stream(side))
        return dx

    def group(self, sv: dict, dy: torch.Tensor, g: int, extra_res: Sequence = (), dx_out=None,
              pre: Optional[str] = None) -> torch.Tensor:
        s, ctx, Wt = self.s, self.ctx, self.Wt
        B, H, W, C = dy.shape
        pre = f"residual_groups.{g}." if pre is None else pre
        if self._strip_bwd_ok(sv, dy, extra_res):
            return self._group_strip_bwd(sv, dy, pre, extra_res, dx_out)
        self._wg(pre + "conv", sv["x_last"], dy, B, H, W, C, C)
        d = ctx.scratch("bw_rg_in", dy.shape)
        blocks = sv["blocks"]
        conv(ctx, dy, Wt.packed(pre + "conv", 2), B, H, W, C, C, y=d,
             **(self._dot_conv(blocks[-1].get("t"), B, H, W, C) if s.NB > 0 else {}))
        for b in reversed(range(s.NB)):
            if b == 0:
                d = self.rcab(blocks[b], d, f"{pre}blocks.{b}.", extra_res=(dy,) + tuple(extra_res),
                              dx_out=dx_out, flush=False)
            else:
                d = self.rcab(blocks[b], d, f"{pre}blocks.{b}.",
                              dx_out=ctx.scratch(f"bw_rg_pp{b & 1}", dy.shape), flush=False,
                              t_next=blocks[b - 1].get("t"))
        self.flush()
        return d

    def tail(self, sv: dict) -> torch.Tensor:
        """Backward of conv_last, the upsampler and conv_after_body; returns d(body output).
        sv['dout'] holds dL/dsr (written by the conv_last epilogue); stores d(fb) in sv['d_fb']."""
        s, ctx, Wt, p, G = self.s, self.ctx, self.Wt, self.Wt.p, self.G
        C = s.C
        B, Ho, Wo = sv["dout"].shape[0], sv["Ho"], sv["Wo"]
        stages = sv["stages"]
        last = stages[-1]
        rows = ctx.lib.fen_conv_last_dgrad_part_rows(B, Ho, Wo)
        dal = ctx.scratch(f"bw_dal_up{len(stages) - 1}", (rows, C), torch.float32)
        du = ctx.scratch(f"bw_du{(len(stages) - 1) & 1}", (B, last["H"], last["W"], 4 * C))
        alpha_last = p[f"upsample.stages.{len(stages) - 1}.prelu.weight"]
        if CL_BWD_FUSED and PRE_ELIDE and ctx.lib.fen_conv_last_bwd_supported(ctx.code, B, Ho, Wo, C, s.out_ch):
            # conv_last's data gradient (+ the last stage's PReLU backward and PixelShuffle
            # inverse) and its weight / bias gradients in one pass over the stage output
            co = s.out_ch
            dwp = ctx.scratch("bw_cl_dw", (rows, co * C * 9), torch.float32)
            dbp = ctx.scratch("bw_cl_db", (rows, co), torch.float32)
            ctx.emit("conv_last_bwd", ctx.lib.fen_conv_last_bwd, ctx.code, B, Ho, Wo, C, co, ptr(sv["dout"]),
                     ptr(p["conv_last.weight"]), ptr(last["v"]), ptr(last["a"]), ptr(alpha_last), ptr(du), ptr(dal),
                     ptr(dwp), ptr(dbp))
            self.cs.add(dwp, rows, co * C * 9, G["conv_last.weight"])
            self.cs.add(dbp, rows, co, G["conv_last.bias"])
        else:
            # conv_last: weight grad (dy = zero-padded 16-channel dout), data grad fused with the
            # last stage's PReLU backward and PixelShuffle inverse
            self._wg("conv_last", sv["a_last"], sv["dout"], B, Ho, Wo, C, 16, cout_valid=s.out_ch)
            ctx.emit("conv_last_dgrad", ctx.lib.fen_conv_last_dgrad, ctx.code, B, Ho, Wo, C, s.out_ch,
                     ptr(sv["dout"]), ptr(p["conv_last.weight"]), ptr(last["v"]),
                     ptr(last["a"]) if PRE_ELIDE else None, ptr(alpha_last), ptr(du), ptr(dal))
        self.cs.add(dal, rows, C, G[f"upsample.stages.{len(stages) - 1}.prelu.weight"])
        for st in reversed(range(len(stages))):
            info = stages[st]
            key = f"upsample.stages.{st}."
            hh, ww = info["H"], info["W"]
            self._wg(key + "conv", info["x"], du, B, hh, ww, C, 4 * C)
            if st > 0:
                prev = stages[st - 1]
                du_prev = ctx.scratch(f"bw_du{(st - 1) & 1}", (B, prev["H"], prev["W"], 4 * C))
                T = tiles(hh, ww)
                dal = ctx.scratch(f"bw_dal_up{st - 1}", (B * T, C), torch.float32)
                conv(ctx, du, Wt.packed(key + "conv", 2), B, hh, ww, 4 * C, C, epi=L.EPI_PRELU_BWD | L.EPI_UNSHUFFLE,
                     alpha=p[f"upsample.stages.{st - 1}.prelu.weight"], pre_in=prev["v"], y=du_prev, part=dal,
                     post_in=prev["a"] if PRE_ELIDE else None)
                self.cs.add(dal, B * T, C, G[f"upsample.stages.{st - 1}.prelu.weight"])
                du = du_prev
            else:
                d_fb = ctx.scratch("bw_d_fb", (B, hh, ww, C))
                conv(ctx, du, Wt.packed(key + "conv", 2), B, hh, ww, 4 * C, C, y=d_fb)
        H, W = stages[0]["H"], stages[0]["W"]
        self._wg("conv_after_body", sv["feat"], d_fb, B, H, W, C, C)
        d_body = ctx.scratch("bw_d_body", (B, H, W, C))
        conv(ctx, d_fb, Wt.packed("conv_after_body", 2), B, H, W, C, C, y=d_body)
        sv["d_fb"] = d_fb
        self.cs.flush()
        return d_body

    def head(self, x_lr: torch.Tensor, d_feat0: torch.Tensor) -> None:
        s, ctx, G = self.s, self.ctx, self.G
        B, _, H, W = x_lr.shape
        nwork = ctx.lib.fen_conv_first_work_floats(B, s.in_ch, H, W, s.C)
        work = ctx.scratch("cf_work", (nwork,), torch.float32)
        ctx.emit("conv_first_wgrad", ctx.lib.fen_conv_first_wgrad, ctx.code, B, s.in_ch, H, W, s.C, ptr(x_lr),
                 ptr(d_feat0), ptr(G["conv_first.weight"]), ptr(G["conv_first.bias"]), 0, ptr(work))
