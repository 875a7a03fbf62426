"""VGG-style discriminator and GAN loss (reference src/models/discriminator.py:12-219) on the
HIP path -- SURVEY.md §8f row 2 (stage-3 GAN step, trainer.py:424-455,468-475).

Same classes, constructor arguments, module tree, state_dict keys and initialisation calls
as the reference, so its checkpoints and trainer code work unchanged.  The feature stack
(10 conv blocks) runs as one autograd Function over C-ABI launches, NHWC in the compute
dtype:
  block 1    conv 3->64 + bias + LeakyReLU(0.2): the K=27 input kernel (fen_conv_first_fwd_ex)
  blocks 2-10 conv (stride 1; stride 2 = a stride-1 conv over the space-to-depth input,
             fen_s2d2, with the phase-major filter -- only the filled taps run, a quarter of
             the full-resolution conv's work; FEN_D_S2D=0: the full-resolution conv +
             fen_subsample2),
             train-mode BatchNorm statistics (+ running-stat update) and BN + LeakyReLU
             (fen_bn_stats / fen_bn_apply; eval mode uses the running statistics)
  backward   fen_bn_bwd (BN + LeakyReLU); stride-2 layers: the weight gradient of the
             phase-major filter on the space-to-depth input (gathered back to OIHW) and the
             data gradient through the same masked conv + the inverse fen_s2d2 (or, with
             FEN_D_S2D=0, fen_zero_insert2 + the full-resolution gradients); weight
             gradients on fen_wgrad3x3 / fen_conv_first_wgrad, data gradients on mode-2 convs
             (block 2's epilogue applies block 1's LeakyReLU mask), and d(input) -- needed by
             the generator's adversarial step -- through a 64->16 conv (3 valid channels).
The classifier head (Flatten -> Linear(32768,1024) -> LeakyReLU -> Linear(1024,1), and the
optional sigmoid) is one autograd Function over fen_dhead_fwd / fen_dhead_bwd (disc.hip): the
first layer on fp32 MFMAs in k-splits summed in fixed order, its backward one pass over the
weight (d(input) and the weight gradient together).  use_bn=False is not wired on the HIP path
(the reference's factory always builds use_bn=True).
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.nn as nn

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32}
_SLOPE = 0.2
_S2D = os.environ.get("FEN_D_S2D", "1") != "0"
# (the 64-channel stride-2 layer stays on the full-resolution persistent kernels)
_S2D_MIN_CIN = int(os.environ.get("FEN_D_S2D_MIN_CIN", "128"))
_S2D_MAX_CIN = int(os.environ.get("FEN_D_S2D_MAX_CIN", "256"))
# FEN_GAN_LOSS=0: GANLoss on the torch criteria (A/B; CPU tensors always take them)
_HIP_GAN_LOSS = os.environ.get("FEN_GAN_LOSS", "1") != "0"
# A/B switch: FEN_D_PACK_MULTI=0 re-packs each stale filter copy in a launch of its own
_PACK_MULTI = os.environ.get("FEN_D_PACK_MULTI", "1") != "0"
# A/B switch: FEN_D_BN_MULTI=0 runs the pair pass's BatchNorm launches once per batch
_BN_MULTI = os.environ.get("FEN_D_BN_MULTI", "1") != "0"


class _DFeatures(torch.autograd.Function):
    """x [ng * Bg, 3, H, W]: ng independent batches of Bg images (forward_pair: ng = 2, the D
    step's real and fake).  The convs, the LeakyReLUs and the head are per image, so the groups
    run as one batch; train-mode BatchNorm takes each group's own statistics (and updates the
    running ones group by group, in order), as separate calls would; the weight gradients come
    out summed over the groups in one launch each."""

    @staticmethod
    def forward(fctx, x, mod, ng, *params):
        from ..hip import lib as L
        from ..hip.net import conv, wgrad  # noqa: F401
        from ..hip.program import Ctx, ptr
        dt = mod.compute_dtype
        ctx = Ctx(dt, x.device)
        lib = ctx.lib
        B, _, H, W = x.shape
        xin = x.detach().float().contiguous()
        blocks = mod._hip_blocks()
        saved = []
        # block 1: conv 3->64 + bias + LeakyReLU
        c0 = blocks[0]
        a = ctx.alloc((B, H, W, c0["cout"]))
        ctx.emit("d_conv1", lib.fen_conv_first_fwd_ex, ctx.code, B, 3, H, W, c0["cout"], ptr(xin),
                 ptr(c0["conv"].weight.detach().float().contiguous()), ptr(c0["conv"].bias.detach().float()), 0, 0,
                 _SLOPE, ptr(a))
        hh, ww = H, W
        tracked = []                                  # BN counters to advance (one launch at the end)
        for blk in blocks[1:]:
            cin, cout, st = blk["cin"], blk["cout"], blk["stride"]
            xs = None
            if st == 2 and _S2D and _S2D_MIN_CIN <= cin <= _S2D_MAX_CIN:
                ho, wo = hh // 2, ww // 2
                xs = ctx.alloc((B, ho, wo, 4 * cin))
                ctx.emit("d_s2d", lib.fen_s2d2, ctx.code, B, hh, ww, cin, ptr(a), ptr(xs), 0)
                z = ctx.alloc((B, ho, wo, cout))
                conv(ctx, xs, mod._packed(ctx, blk, 0, s2d=True), B, ho, wo, 4 * cin, cout, y=z, s2d_in=cin)
            else:
                wpk = mod._packed(ctx, blk, 0)
                z = ctx.alloc((B, hh, ww, cout))
                conv(ctx, a, wpk, B, hh, ww, cin, cout, y=z)
                ho, wo = (hh // 2, ww // 2) if st == 2 else (hh, ww)
                if st == 2:
                    zs = ctx.alloc((B, ho, wo, cout))
                    ctx.emit("d_sub", lib.fen_subsample2, ctx.code, B, hh, ww, cout, ptr(z), ptr(zs))
                    z = zs
            bn = blk["bn"]
            out = ctx.alloc((B, ho, wo, cout))
            gs = ng if mod.training else 1
            npx = (B // gs) * ho * wo                     # one BN group's pixels
            stat = ctx.alloc((gs, 2 * cout), torch.float32)
            if gs > 1 and _BN_MULTI:
                # the groups' statistics (running stats moved group by group) and BN + LeakyReLU
                # in the launches of one group (fen_bn_stats_n / fen_bn_apply_n: bit-identical)
                work = ctx.alloc((gs * lib.fen_bn_work_floats(cout),), torch.float32)
                ctx.emit("d_bn_stats", lib.fen_bn_stats_n, ctx.code, gs, npx, cout, ptr(z), float(bn.eps),
                         float(bn.momentum), ptr(stat), ptr(bn.running_mean), ptr(bn.running_var), ptr(work))
                tracked += [bn.num_batches_tracked] * gs
                ctx.emit("d_bn_apply", lib.fen_bn_apply_n, ctx.code, gs, npx, cout, ptr(z), ptr(stat), ptr(stat[0, cout:]),
                         2 * cout, ptr(bn.weight.detach()), ptr(bn.bias.detach()), _SLOPE, ptr(out))
            for gi in range(gs if not (gs > 1 and _BN_MULTI) else 0):
                zg, sg, og = z[gi * (B // gs):], stat[gi], out[gi * (B // gs):]
                if mod.training:
                    work = ctx.alloc((lib.fen_bn_work_floats(cout),), torch.float32)
                    ctx.emit("d_bn_stats", lib.fen_bn_stats, ctx.code, npx, cout, ptr(zg), float(bn.eps),
                             float(bn.momentum), ptr(sg), ptr(bn.running_mean), ptr(bn.running_var), ptr(work))
                    tracked.append(bn.num_batches_tracked)
                else:
                    with torch.no_grad():
                        sg[:cout] = bn.running_mean
                        sg[cout:] = (bn.running_var + bn.eps).rsqrt()
                ctx.emit("d_bn_apply", lib.fen_bn_apply, ctx.code, npx, cout, ptr(zg), ptr(sg), ptr(sg[cout:]),
                         ptr(bn.weight.detach()), ptr(bn.bias.detach()), _SLOPE, ptr(og))
            saved.append(dict(blk=blk, a_in=a, xs=xs, z=z, stat=stat, H=hh, W=ww, Ho=ho, Wo=wo))
            a, hh, ww = out, ho, wo
        if tracked:
            # num_batches_tracked += its BN calls (ng per layer), every layer in one launch (a
            # tensor once in the list: repeated entries would race inside the launch)
            cnt = {}
            for t in tracked:
                cnt[id(t)] = (t, cnt.get(id(t), (t, 0))[1] + 1)
            with torch.no_grad():
                torch._foreach_add_([t for t, _ in cnt.values()], [n for _, n in cnt.values()])
        fctx.saved_blocks, fctx.a1, fctx.xin, fctx.mod = saved, saved[0]["a_in"], xin, mod
        fctx.shape = (B, H, W)
        fctx.ng = ng if mod.training else 1
        fctx.x_needs_grad = x.requires_grad
        return a.float().permute(0, 3, 1, 2).contiguous()        # NCHW for the Flatten

    @staticmethod
    def backward(fctx, g):
        from ..hip import lib as L
        from ..hip.net import conv, s2d_filter_grad, tiles, wgrad
        from ..hip.program import Ctx, ptr
        mod = fctx.mod
        dt = mod.compute_dtype
        ctx = Ctx(dt, g.device)
        lib = ctx.lib
        B, H, W = fctx.shape
        d = g.permute(0, 2, 3, 1).contiguous().to(dt)            # NHWC
        blocks = mod._hip_blocks()
        grads = {}
        # the parameters' gradients only when autograd wants them (the trainer's generator step
        # passes D frozen: its data gradient alone, TrainerConfig.freeze_d_in_g_step)
        pgrad = any(fctx.needs_input_grad[3:])
        ng = fctx.ng
        for k in range(len(fctx.saved_blocks) - 1, -1, -1):
            sv = fctx.saved_blocks[k]
            blk, bn = sv["blk"], sv["blk"]["bn"]
            cin, cout = blk["cin"], blk["cout"]
            npx = (B // ng) * sv["Ho"] * sv["Wo"]
            dz = ctx.alloc((B, sv["Ho"], sv["Wo"], cout))
            # (every gradient buffer below is written whole by its kernel: no zero fill; the BN
            # groups' dgamma / dbeta accumulate)
            dgam = torch.empty(cout, device=g.device)
            dbet = torch.empty(cout, device=g.device)
            if ng > 1 and _BN_MULTI:
                # every group in the launches of one (fen_bn_bwd_n; dgamma / dbeta summed in group
                # order, as the per-group calls below accumulate them)
                work = ctx.alloc((ng * lib.fen_bn_work_floats(cout),), torch.float32)
                ctx.emit("d_bn_bwd", lib.fen_bn_bwd_n, ctx.code, ng, npx, cout, ptr(d), ptr(sv["z"]), ptr(sv["stat"]),
                         ptr(bn.weight.detach()), ptr(bn.bias.detach()), _SLOPE, ptr(dz), ptr(dgam), ptr(dbet), 0,
                         ptr(work))
            else:
                work = ctx.alloc((lib.fen_bn_work_floats(cout),), torch.float32)
            for gi in range(ng if not (ng > 1 and _BN_MULTI) else 0):
                o = gi * (B // ng)
                ctx.emit("d_bn_bwd", lib.fen_bn_bwd, ctx.code, npx, cout, ptr(d[o:]), ptr(sv["z"][o:]), ptr(sv["stat"][gi]),
                         ptr(bn.weight.detach()), ptr(bn.bias.detach()), _SLOPE, ptr(dz[o:]), ptr(dgam), ptr(dbet),
                         int(gi > 0), ptr(work))
            grads[bn.weight] = dgam
            grads[bn.bias] = dbet
            if sv["xs"] is not None:
                # stride 2 over the space-to-depth input: the phase-major filter's gradients
                ho, wo, c4 = sv["Ho"], sv["Wo"], 4 * cin
                if pgrad:
                    dw4 = torch.empty(cout, c4, 3, 3, device=g.device)
                    wgrad(ctx, sv["xs"], dz, B, ho, wo, c4, cout, dw4, None)
                    dw = torch.empty_like(blk["conv"].weight)
                    s2d_filter_grad(dw4, dw)
                    grads[blk["conv"].weight] = dw
                dxs = ctx.alloc((B, ho, wo, c4))
                if k == 0:
                    part = ctx.alloc((B * tiles(ho, wo), c4), torch.float32)
                    conv(ctx, dz, mod._packed(ctx, blk, 2, s2d=True), B, ho, wo, cout, c4, epi=L.EPI_PRELU_BWD,
                         alpha=mod._slopes(c4, g.device), pre_in=sv["xs"], y=dxs, part=part, s2d_out=cin)
                else:
                    conv(ctx, dz, mod._packed(ctx, blk, 2, s2d=True), B, ho, wo, cout, c4, y=dxs, s2d_out=cin)
                da = ctx.alloc((B, sv["H"], sv["W"], cin))
                ctx.emit("d_s2d_inv", lib.fen_s2d2, ctx.code, B, sv["H"], sv["W"], cin, ptr(dxs), ptr(da), 1)
                d = da
                continue
            if blk["stride"] == 2:
                dzf = ctx.alloc((B, sv["H"], sv["W"], cout))
                ctx.emit("d_zins", lib.fen_zero_insert2, ctx.code, B, sv["Ho"], sv["Wo"], cout, ptr(dz), ptr(dzf))
                dz = dzf
            if pgrad:
                dw = torch.empty_like(blk["conv"].weight)
                wgrad(ctx, sv["a_in"], dz, B, sv["H"], sv["W"], cin, cout, dw, None)
                grads[blk["conv"].weight] = dw
            da = ctx.alloc((B, sv["H"], sv["W"], cin))
            if k == 0:
                # block 1's LeakyReLU mask on the way down: a1 > 0 <=> its pre-activation > 0
                part = ctx.alloc((B * ((sv["H"] + 15) // 16) * ((sv["W"] + 15) // 16), cin), torch.float32)
                conv(ctx, dz, mod._packed(ctx, blk, 2), B, sv["H"], sv["W"], cout, cin, epi=L.EPI_PRELU_BWD,
                     alpha=mod._slopes(cin, g.device), pre_in=fctx.a1, y=da, part=part)
            else:
                conv(ctx, dz, mod._packed(ctx, blk, 2), B, sv["H"], sv["W"], cout, cin, y=da)
            d = da
        # block 1: conv 3->64 weight / bias gradient, and d(input) when asked for
        c0 = blocks[0]
        if pgrad:
            dw0 = torch.empty_like(c0["conv"].weight)
            db0 = torch.empty_like(c0["conv"].bias)
            work = ctx.alloc((lib.fen_conv_first_work_floats(B, 3, H, W, c0["cout"]),), torch.float32)
            ctx.emit("d_conv1_wgrad", lib.fen_conv_first_wgrad, ctx.code, B, 3, H, W, c0["cout"], ptr(fctx.xin), ptr(d),
                     ptr(dw0), ptr(db0), 0, ptr(work))
            grads[c0["conv"].weight] = dw0
            grads[c0["conv"].bias] = db0
        dx = None
        if fctx.x_needs_grad:
            d16 = ctx.alloc((B, H, W, 16))
            conv(ctx, d, mod._packed(ctx, c0, 2), B, H, W, c0["cout"], 16, y=d16)
            dx = d16[..., :3].float().permute(0, 3, 1, 2).contiguous()
        out = [grads.get(p) if pgrad else None for p in mod._feature_params()]
        return (dx, None, None, *out)


def _dhead_forward(h, w1, b1, w2, b2, sigmoid):
    """fen_dhead_fwd: (pre-activation [B, N], score [B, 1]) of the classifier head."""
    from ..hip import lib as L
    from ..hip.program import ptr
    B, K = h.shape
    N = w1.shape[0]
    pre = torch.empty(B, N, device=h.device)
    y = torch.empty(B, 1, device=h.device)
    work = torch.empty(L.load().fen_dhead_work_floats(B, K, N), device=h.device)
    L.check(L.load().fen_dhead_fwd(B, K, N, ptr(h), ptr(w1.detach()), ptr(b1.detach()), ptr(w2.detach()),
                                   ptr(b2.detach()), _SLOPE, int(sigmoid), ptr(pre), ptr(y), ptr(work),
                                   torch.cuda.current_stream().cuda_stream), "dhead_fwd")
    return pre, y


class _DHead(torch.autograd.Function):
    """The classifier head on the C-ABI's fen_dhead_fwd / fen_dhead_bwd (discriminator.py:85-90,
    131-132): Linear(K, N) -> LeakyReLU(0.2) -> Linear(N, 1) (-> sigmoid), fp32."""

    @staticmethod
    def forward(fctx, h, w1, b1, w2, b2, sigmoid):
        h = h.detach().contiguous()
        pre, y = _dhead_forward(h, w1, b1, w2, b2, sigmoid)
        fctx.save_for_backward(h, w1, w2, pre, y)
        fctx.sigmoid = bool(sigmoid)
        return y

    @staticmethod
    def backward(fctx, gy):
        from ..hip import lib as L
        from ..hip.program import ptr
        h, w1, w2, pre, y = fctx.saved_tensors
        B, K = h.shape
        N = w1.shape[0]
        gy = gy.detach().float().contiguous()
        dx = torch.empty_like(h) if fctx.needs_input_grad[0] else None
        dw1 = torch.empty_like(w1)
        db1 = torch.empty(N, device=h.device)
        dw2 = torch.empty_like(w2)
        db2 = torch.empty(1, device=h.device)
        work = torch.empty(L.load().fen_dhead_work_floats(B, K, N), device=h.device)
        L.check(L.load().fen_dhead_bwd(B, K, N, ptr(h), ptr(w1.detach()), ptr(pre), ptr(w2.detach()), ptr(y), ptr(gy),
                                       _SLOPE, int(fctx.sigmoid), ptr(dx), ptr(dw1), ptr(db1), ptr(dw2), ptr(db2),
                                       ptr(work), torch.cuda.current_stream().cuda_stream), "dhead_bwd")
        return dx, dw1, db1, dw2, db2, None


class VGGStyleDiscriminator(nn.Module):
    """VGG-style discriminator for 256x256 images (discriminator.py:12-151)."""

    def __init__(self, in_channels: int = 3, base_channels: int = 64, input_size: int = 256, use_bn: bool = True,
                 use_sigmoid: bool = False, precision: str = "bf16"):
        super().__init__()
        self.use_sigmoid = use_sigmoid
        self.use_bn = use_bn

        def conv_block(in_ch, out_ch, kernel_size=3, stride=1, use_bn=True):
            layers = [nn.Conv2d(in_ch, out_ch, kernel_size, stride, padding=kernel_size // 2, bias=not use_bn)]
            if use_bn:
                layers.append(nn.BatchNorm2d(out_ch))
            layers.append(nn.LeakyReLU(0.2, inplace=True))
            return nn.Sequential(*layers)

        bc = base_channels
        self.features = nn.Sequential(
            conv_block(in_channels, bc, use_bn=False),
            conv_block(bc, bc, stride=2, use_bn=use_bn),
            conv_block(bc, bc * 2, use_bn=use_bn),
            conv_block(bc * 2, bc * 2, stride=2, use_bn=use_bn),
            conv_block(bc * 2, bc * 4, use_bn=use_bn),
            conv_block(bc * 4, bc * 4, stride=2, use_bn=use_bn),
            conv_block(bc * 4, bc * 8, use_bn=use_bn),
            conv_block(bc * 8, bc * 8, stride=2, use_bn=use_bn),
            conv_block(bc * 8, bc * 8, use_bn=use_bn),
            conv_block(bc * 8, bc * 8, stride=2, use_bn=use_bn),
        )
        feature_size = input_size // 32
        self.classifier = nn.Sequential(
            nn.Flatten(),
            nn.Linear(bc * 8 * feature_size * feature_size, 1024),
            nn.LeakyReLU(0.2, inplace=True),
            nn.Linear(1024, 1),
        )
        self._initialize_weights()
        self.compute_dtype = _DTYPES[precision]
        self._packs = {}
        self._pack_tab = {}                            # dtype code -> (device job table, njobs, total)

    def _initialize_weights(self):
        """discriminator.py:104-116."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, a=0.2, mode='fan_in', nonlinearity='leaky_relu')
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.kaiming_normal_(m.weight, a=0.2, mode='fan_in', nonlinearity='leaky_relu')
                nn.init.zeros_(m.bias)

    # ---- HIP plumbing ----
    def _hip_blocks(self) -> List[dict]:
        out = []
        for i, seq in enumerate(self.features):
            cv = seq[0]
            bn = seq[1] if isinstance(seq[1], nn.BatchNorm2d) else None
            out.append(dict(i=i, conv=cv, bn=bn, cin=cv.in_channels, cout=cv.out_channels, stride=cv.stride[0]))
        return out

    def _feature_params(self):
        return [p for p in self.features.parameters()]

    def _packed(self, ctx, blk, mode, s2d=False):
        """The packed copy of block blk's filter for fen_conv3x3 mode `mode` (phase-major for the
        space-to-depth form).  A new copy is packed on its own; when the weights move (an
        optimizer step bumps every version at once) the first stale lookup re-packs every known
        copy in ONE fen_pack_multi launch (+ the space-to-depth scatters), not one launch per
        (layer, mode).  (A captured GAN iteration records the re-packs its Python saw: the
        optimizer steps bump the versions at capture time exactly as in every eager iteration.)"""
        from ..hip.net import s2d_filter
        from ..hip.program import ptr
        w = blk["conv"].weight
        key = (blk["i"], mode, ctx.code, s2d)
        ent = self._packs.get(key)
        if ent is None or ent[1] != w.data_ptr():
            cout, cin = w.shape[0], w.shape[1] * (4 if s2d else 1)
            n = ctx.lib.fen_packed_elems(mode, cout, cin)
            buf = torch.empty(n, dtype=ctx.tdtype, device=w.device)
            src = self._s2d_src(blk, w) if s2d else w.detach()
            if s2d:
                self._s2d_scatter(blk, w)
            ctx.emit("d_pack", ctx.lib.fen_pack_conv_w, ctx.code, mode, cout, cin, ptr(src.contiguous()), ptr(buf))
            ent = (w._version, w.data_ptr(), buf, w, mode, cout, cin, src, blk, s2d)
            self._packs[key] = ent
            self._pack_tab.pop(ctx.code, None)
        elif ent[0] != w._version:
            if _PACK_MULTI:
                self._repack_all(ctx)
            else:                                      # (A/B: one launch per stale copy)
                if s2d:
                    self._s2d_scatter(blk, w)
                ctx.emit("d_pack", ctx.lib.fen_pack_conv_w, ctx.code, mode, ent[5], ent[6], ptr(ent[7]), ptr(ent[2]))
                self._packs[key] = (w._version,) + ent[1:]
            ent = self._packs[key]
        return ent[2]

    def _s2d_src(self, blk, w):
        """The persistent fp32 phase-major filter of a space-to-depth block (re-scattered from the
        weights on every re-pack)."""
        k = ("s2d_src", blk["i"])
        if k not in self._packs:
            self._packs[k] = torch.empty(w.shape[0], 4 * w.shape[1], 3, 3, device=w.device)
        return self._packs[k]

    def _s2d_scatter(self, blk, w):
        from ..hip import lib as L
        src = self._s2d_src(blk, w)
        L.check(L.load().fen_s2d_filter(int(w.shape[0]), int(w.shape[1]), w.detach().contiguous().data_ptr(),
                                        src.data_ptr(), 0, torch.cuda.current_stream().cuda_stream), "s2d_filter")

    def _repack_all(self, ctx):
        """Every packed copy of dtype ctx.code whose weights moved: the space-to-depth scatters,
        then one fen_pack_multi over all of them (its job table built once per entry set)."""
        import ctypes
        from ..hip import lib as L
        ents = [(k, e) for k, e in self._packs.items() if isinstance(k[0], int) and k[2] == ctx.code]
        done = set()
        for k, e in ents:
            if e[9] and e[8]["i"] not in done:
                self._s2d_scatter(e[8], e[3])
                done.add(e[8]["i"])
        tab = self._pack_tab.get(ctx.code)
        if tab is None:
            lib = ctx.lib
            jobs = (L.PackJob * len(ents))()
            for i, (k, e) in enumerate(ents):
                jobs[i].w, jobs[i].out = e[7].data_ptr(), e[2].data_ptr()
                jobs[i].mode, jobs[i].Cout, jobs[i].Cin = e[4], e[5], e[6]
            nbytes = lib.fen_pack_table_bytes(len(ents))
            host = (ctypes.c_uint8 * nbytes)()
            total = ctypes.c_size_t(0)
            L.check(lib.fen_pack_table(ctx.code, len(ents), ctypes.cast(jobs, ctypes.c_void_p),
                                       ctypes.cast(host, ctypes.c_void_p), ctypes.byref(total)), "d_pack_table")
            dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(ents[0][1][2].device)
            tab = self._pack_tab[ctx.code] = (dev, len(ents), int(total.value))
        dev, nj, total = tab
        L.check(ctx.lib.fen_pack_multi(ctx.code, nj, dev.data_ptr(), total, torch.cuda.current_stream().cuda_stream),
                "d_pack_multi")
        for k, e in ents:
            self._packs[k] = (e[3]._version,) + e[1:]

    def _slopes(self, n, dev):
        key = ("slopes", n, dev)
        if key not in self._packs:
            self._packs[key] = torch.full((n,), _SLOPE, device=dev)
        return self._packs[key]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B, 3, H, W) -> (B, 1) score (discriminator.py:118-136)."""
        if not x.is_cuda:
            raise RuntimeError("the HIP discriminator runs on a ROCm GPU tensor (got CPU); there is no CPU path")
        if not self.use_bn:
            raise NotImplementedError("use_bn=False is not wired on the HIP path")
        if x.shape[1] != 3 or x.shape[2] % 32 or x.shape[3] % 32:
            raise ValueError("input must be (B, 3, H, W) with H, W multiples of 32")
        feats = _DFeatures.apply(x, self, 1, *self._feature_params())
        lin1, lin2 = self.classifier[1], self.classifier[3]
        return _DHead.apply(feats.flatten(1), lin1.weight, lin1.bias, lin2.weight, lin2.bias, self.use_sigmoid)

    def forward_pair(self, x1: torch.Tensor, x2: torch.Tensor):
        """(self(x1), self(x2)) -- the D step's real and fake batches (trainer.py:433-434) -- as
        one pass: the two batches' convs, LeakyReLUs and head run as one batch, train-mode
        BatchNorm takes each batch's own statistics and updates the running ones x1 then x2,
        exactly as the two calls do; the parameter gradients come out summed in one launch each
        (no per-parameter accumulation of two gradients).  Same scores; gradients equal to the two
        calls' up to fp32 summation order."""
        if x1.shape != x2.shape or os.environ.get("FEN_D_PAIR", "1") == "0":
            return self(x1), self(x2)
        x = torch.cat([x1, x2])
        if not x.is_cuda:
            raise RuntimeError("the HIP discriminator runs on a ROCm GPU tensor (got CPU); there is no CPU path")
        if not self.use_bn:
            raise NotImplementedError("use_bn=False is not wired on the HIP path")
        if x.shape[1] != 3 or x.shape[2] % 32 or x.shape[3] % 32:
            raise ValueError("input must be (B, 3, H, W) with H, W multiples of 32")
        feats = _DFeatures.apply(x, self, 2, *self._feature_params())
        lin1, lin2 = self.classifier[1], self.classifier[3]
        y = _DHead.apply(feats.flatten(1), lin1.weight, lin1.bias, lin2.weight, lin2.bias, self.use_sigmoid)
        return y[:x1.shape[0]], y[x1.shape[0]:]

    def head_preactivation(self, h: torch.Tensor) -> torch.Tensor:
        """The classifier's hidden layer before its LeakyReLU, Linear(32768, 1024) of the
        flattened features, exactly as forward computes it (the same fen_dhead_fwd launch;
        tests read its branches)."""
        lin1, lin2 = self.classifier[1], self.classifier[3]
        return _dhead_forward(h.detach().float().contiguous(), lin1.weight, lin1.bias, lin2.weight, lin2.bias,
                              self.use_sigmoid)[0]

    def get_model_info(self) -> dict:
        total_params = sum(p.numel() for p in self.parameters())
        trainable_params = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return {'name': 'VGGStyleDiscriminator', 'total_params': total_params, 'trainable_params': trainable_params,
                'size_mb': total_params * 4 / (1024 ** 2)}


_GAN_MODES = {'vanilla': 0, 'lsgan': 1, 'wgan': 2}


class _GanLossFn(torch.autograd.Function):
    """GANLoss's criterion on fen_gan_loss / fen_gan_loss_bwd: one launch each way (the module
    losses take ~10 small aten kernels per call)."""

    @staticmethod
    def forward(fctx, x, mode, target):
        from ..hip import lib as L
        x = x.detach().float().contiguous()
        loss = torch.empty((), device=x.device)
        L.check(L.load().fen_gan_loss(mode, x.numel(), x.data_ptr(), float(target), loss.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream), "gan_loss")
        fctx.save_for_backward(x)
        fctx.mode, fctx.target = mode, float(target)
        return loss

    @staticmethod
    def backward(fctx, gy):
        from ..hip import lib as L
        (x,) = fctx.saved_tensors
        gy = gy.detach().float().contiguous()
        gx = torch.empty_like(x)
        L.check(L.load().fen_gan_loss_bwd(fctx.mode, x.numel(), x.data_ptr(), fctx.target, gy.data_ptr(),
                                          gx.data_ptr(), torch.cuda.current_stream().cuda_stream), "gan_loss_bwd")
        return gx, None, None


class GANLoss(nn.Module):
    """'vanilla' (BCE with logits), 'lsgan' (MSE), 'wgan' (raw scores) -- discriminator.py:154-206."""

    def __init__(self, gan_type: str = 'vanilla', real_label: float = 1.0, fake_label: float = 0.0):
        super().__init__()
        self.gan_type = gan_type
        self.real_label = real_label
        self.fake_label = fake_label
        if gan_type == 'vanilla':
            self.loss = nn.BCEWithLogitsLoss()
        elif gan_type == 'lsgan':
            self.loss = nn.MSELoss()
        elif gan_type == 'wgan':
            self.loss = None
        else:
            raise ValueError(f"Unknown GAN type: {gan_type}")

    def get_target_tensor(self, prediction: torch.Tensor, is_real: bool) -> torch.Tensor:
        return torch.full_like(prediction, self.real_label if is_real else self.fake_label)

    def forward(self, prediction: torch.Tensor, is_real: bool) -> torch.Tensor:
        if prediction.is_cuda and prediction.dtype == torch.float32 and _HIP_GAN_LOSS:
            t = (-1.0 if is_real else 1.0) if self.gan_type == 'wgan' else (self.real_label if is_real else self.fake_label)
            return _GanLossFn.apply(prediction, _GAN_MODES[self.gan_type], t)
        if self.gan_type == 'wgan':
            return -prediction.mean() if is_real else prediction.mean()
        return self.loss(prediction, self.get_target_tensor(prediction, is_real))


def create_discriminator(input_size: int = 256, base_channels: int = 64, use_bn: bool = True,
                         **kwargs) -> VGGStyleDiscriminator:
    """discriminator.py:209-219."""
    return VGGStyleDiscriminator(in_channels=3, base_channels=base_channels, input_size=input_size, use_bn=use_bn,
                                 use_sigmoid=False, **{k: v for k, v in kwargs.items() if k == "precision"})


__all__ = ["VGGStyleDiscriminator", "GANLoss", "create_discriminator"]
