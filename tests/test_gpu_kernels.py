"""Per-kernel GPU parity: each C-ABI entry point against the CPU oracle's restatement of
the same op (fp32 exact-ish, bf16 within bf16 rounding)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ctx(dtype):
    from src.hip.program import Ctx
    return Ctx(dtype, DEV)


def nhwc(x_nchw, dtype):
    return x_nchw.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)


def nchw(x_nhwc):
    return x_nhwc.float().cpu().permute(0, 3, 1, 2).contiguous()


def _tol(dtype, ref):
    return (2e-5 if dtype == torch.float32 else 3e-2) * max(1.0, float(ref.abs().max()))


def _pack(ctx, w, mode):
    from src.hip.program import ptr
    n = ctx.lib.fen_packed_elems(mode, w.shape[0], w.shape[1])
    buf = torch.empty(n, dtype=ctx.tdtype, device=DEV)
    wd = w.to(DEV).contiguous()
    ctx.emit("pack", ctx.lib.fen_pack_conv_w, ctx.code, mode, w.shape[0], w.shape[1], ptr(wd), ptr(buf))
    return buf


DT = [torch.float32, torch.bfloat16]
DT_FWD = DT + [torch.float16]     # the forward kernels also run fp16 (inference precision)


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 16, 64, 64), (1, 20, 36, 64, 64), (2, 32, 16, 128, 64),
                                             (1, 16, 32, 64, 256), (1, 8, 8, 64, 16), (2, 16, 16, 32, 32),
                                             (1, 20, 24, 32, 128), (2, 16, 16, 96, 32), (1, 16, 16, 32, 16)])
def test_conv3x3_plain(dtype, B, H, W, Cin, Cout):
    from src.hip import net
    torch.manual_seed(0)
    x = torch.randn(B, Cin, H, W)
    w = torch.randn(Cout, Cin, 3, 3) * 0.05
    b = torch.randn(Cout) * 0.1
    ref = F.conv2d(x, w, b, padding=1)
    ctx = _ctx(dtype)
    wp = _pack(ctx, w, 0)
    y = ctx.alloc((B, H, W, Cout))
    net.conv(ctx, nhwc(x, dtype), wp, B, H, W, Cin, Cout, bias=b.to(DEV), y=y)
    torch.cuda.synchronize()
    err = (nchw(y) - ref).abs().max()
    assert err <= _tol(dtype, ref), float(err)


@pytest.mark.parametrize("dtype", DT_FWD)
def test_conv3x3_prelu_pool_res(dtype):
    from src.hip import lib as L, net
    torch.manual_seed(1)
    B, H, W, C = 2, 24, 40, 64
    x = torch.randn(B, C, H, W)
    r = torch.randn(B, C, H, W)
    w = torch.randn(C, C, 3, 3) * 0.05
    b = torch.randn(C) * 0.1
    a = torch.rand(C) * 0.5
    z = F.conv2d(x, w, b, padding=1) + r
    act = O.prelu(z, a)
    ctx = _ctx(dtype)
    wp = _pack(ctx, w, 0)
    y = ctx.alloc((B, H, W, C))
    ypre = ctx.alloc((B, H, W, C))
    T = net.tiles(H, W)
    net.conv(ctx, nhwc(x, dtype), wp, B, H, W, C, C, bias=b.to(DEV), epi=L.EPI_PRELU, alpha=a.to(DEV), y=y,
             y_pre=ypre, res=(nhwc(r, dtype),))
    part = ctx.alloc((B * T, C), torch.float32)
    y2 = ctx.alloc((B, H, W, C))
    net.conv(ctx, nhwc(x, dtype), wp, B, H, W, C, C, bias=b.to(DEV), epi=L.EPI_POOL, y=y2, part=part)
    torch.cuda.synchronize()
    assert (nchw(ypre) - z).abs().max() <= _tol(dtype, z)
    assert (nchw(y) - act).abs().max() <= _tol(dtype, act)
    pool = part.view(B, T, C).sum(1).cpu() / (H * W)
    ref_pool = F.conv2d(x, w, b, padding=1).mean(dim=(2, 3))
    assert (pool - ref_pool).abs().max() <= (1e-5 if dtype == torch.float32 else 2e-3)


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("B,H,W,nres", [(2, 64, 64, 0), (2, 64, 64, 1), (3, 40, 56, 1), (1, 16, 16, 2),
                                         (32, 64, 64, 1)])
def test_conv_dot_epilogue(dtype, B, H, W, nres):
    """FEN_EPI_DOT: the conv's output (after residual adds) as stored, dotted with pre_in per
    16x16 tile and channel (the SE backward's sum dy*t for the next RCAB).  The output must
    equal the plain conv's bit for bit, and the partials the tile sums of y_stored * t
    (rel 1e-5; a wrong tile / channel mapping is O(1)).  (2, 64, 64) with 0 / 1 residual are
    the ping-pong kernel's DOT instantiations, 2 residuals the generic one-group kernel,
    40x56 ragged tiles, B=32 the training batch."""
    from src.hip import lib as L, net
    torch.manual_seed(5)
    C = 64
    x = torch.randn(B, C, H, W)
    w = torch.randn(C, C, 3, 3) * 0.05
    t = torch.randn(B, C, H, W)
    res = [torch.randn(B, C, H, W) for _ in range(nres)]
    ctx = _ctx(dtype)
    wp = _pack(ctx, w, 0)
    xd, td = nhwc(x, dtype), nhwc(t, dtype)
    rd = [nhwc(r, dtype) for r in res]
    y0 = ctx.alloc((B, H, W, C))
    net.conv(ctx, xd, wp, B, H, W, C, C, y=y0, res=rd)
    T = net.tiles(H, W)
    part = ctx.alloc((B * T, C), torch.float32)
    y1 = ctx.alloc((B, H, W, C))
    net.conv(ctx, xd, wp, B, H, W, C, C, y=y1, res=rd, epi=L.EPI_DOT, pre_in=td, part=part)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    prod = (y1.float() * td.float()).cpu()                            # [B, H, W, C]
    th, tw = (H + 15) // 16, (W + 15) // 16
    pad = torch.zeros(B, th * 16, tw * 16, C)
    pad[:, :H, :W] = prod
    ref = pad.view(B, th, 16, tw, 16, C).sum((2, 4)).reshape(B * T, C)
    rel = float((part.cpu() - ref).norm() / ref.norm())
    assert rel <= 1e-5, rel


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("B,H,W", [(2, 16, 32), (2, 16, 64), (1, 24, 128)])
def test_upsample_conv_shuffle_prelu(dtype, B, H, W):
    """The upsampler stage conv (64 -> 256 + bias + PixelShuffle + PReLU, y_pre kept), partial
    and full tile rows, several tiles per block."""
    from src.hip import lib as L, net
    torch.manual_seed(2)
    C = 64
    x = torch.randn(B, C, H, W)
    w = torch.randn(4 * C, C, 3, 3) * 0.05
    b = torch.randn(4 * C) * 0.1
    a = torch.rand(C) * 0.5
    v = O.pixel_shuffle(F.conv2d(x, w, b, padding=1), 2)
    ref = O.prelu(v, a)
    ctx = _ctx(dtype)
    wp = _pack(ctx, w, 1)
    y = ctx.alloc((B, 2 * H, 2 * W, C))
    ypre = ctx.alloc((B, 2 * H, 2 * W, C))
    net.conv(ctx, nhwc(x, dtype), wp, B, H, W, C, 4 * C, bias=b.to(DEV), epi=L.EPI_PRELU | L.EPI_SHUFFLE,
             alpha=a.to(DEV), y=y, y_pre=ypre)
    torch.cuda.synchronize()
    assert (nchw(ypre) - v).abs().max() <= _tol(dtype, v)
    assert (nchw(y) - ref).abs().max() <= _tol(dtype, ref)


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("B,H,W", [(2, 20, 24), (3, 17, 19), (40, 64, 64)])
def test_conv_first(dtype, B, H, W):
    """4-pixel runs (W % 4 == 0, grid-stride over several runs at B = 40) and the one-pixel form."""
    torch.manual_seed(3)
    C = 64
    x = torch.rand(B, 3, H, W)
    w = torch.randn(C, 3, 3, 3) * 0.2
    b = torch.randn(C) * 0.1
    ref = F.conv2d(x, w, b, padding=1)
    ctx = _ctx(dtype)
    from src.hip.program import ptr
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    y = ctx.alloc((B, H, W, C))
    ctx.emit("cf", ctx.lib.fen_conv_first_fwd, ctx.code, B, 3, H, W, C, ptr(xd), ptr(wd), ptr(bd), ptr(y))
    torch.cuda.synchronize()
    assert (nchw(y) - ref).abs().max() <= _tol(dtype, ref)


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("B,H,W,C", [(2, 20, 24, 16), (3, 17, 19, 48), (2, 33, 40, 64), (1, 16, 32, 128),
                                     (70, 64, 64, 64)])
def test_conv_first_ex(dtype, B, H, W, C):
    """fen_conv_first_fwd_ex with the VGG input normalisation and LeakyReLU(0.2): the split-f16
    matrix-core form for 16-bit outputs (C % 16 == 0, ragged tiles, grid-stride at B = 70)."""
    torch.manual_seed(4)
    x = torch.rand(B, 3, H, W)
    w = torch.randn(C, 3, 3, 3) * 0.2
    b = torch.randn(C) * 0.1
    mean, std = torch.tensor([0.485, 0.456, 0.406]), torch.tensor([0.229, 0.224, 0.225])
    ref = F.leaky_relu(F.conv2d((x - mean.view(1, 3, 1, 1)) / std.view(1, 3, 1, 1), w, b, padding=1), 0.2)
    ctx = _ctx(dtype)
    from src.hip.program import ptr
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    md, isd = mean.to(DEV), (1.0 / std).to(DEV)
    y = ctx.alloc((B, H, W, C))
    ctx.emit("cf", ctx.lib.fen_conv_first_fwd_ex, ctx.code, B, 3, H, W, C, ptr(xd), ptr(wd), ptr(bd), ptr(md),
             ptr(isd), 0.2, ptr(y))
    torch.cuda.synchronize()
    assert (nchw(y) - ref).abs().max() <= _tol(dtype, ref)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,H,W,C", [(2, 20, 24, 64), (1, 16, 16, 64), (3, 37, 19, 64), (4, 64, 64, 64),
                                     (1, 16, 32, 128)])
def test_conv_first_wgrad(dtype, B, H, W, C):
    """fen_conv_first_wgrad (3 -> C, fp32 NCHW input, NHWC dy) vs float64 autograd on the
    same dy rounded to the compute dtype; ragged tiles (37 x 19), C = 128 (two lane sets)."""
    torch.manual_seed(11)
    x = torch.rand(B, 3, H, W)
    dy = torch.randn(B, C, H, W).to(dtype).float()
    w = torch.zeros(C, 3, 3, 3, dtype=torch.float64, requires_grad=True)
    bb = torch.zeros(C, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double(), w, bb, padding=1).mul(dy.double()).sum().backward()
    ctx = _ctx(dtype)
    from src.hip.program import ptr
    xd = x.to(DEV)
    dyd = nhwc(dy, dtype)
    dw = ctx.alloc((C, 3, 3, 3), torch.float32)
    db = ctx.alloc((C,), torch.float32)
    work = ctx.alloc((ctx.lib.fen_conv_first_work_floats(B, 3, H, W, C),), torch.float32)
    ctx.emit("cfw", ctx.lib.fen_conv_first_wgrad, ctx.code, B, 3, H, W, C, ptr(xd), ptr(dyd), ptr(dw), ptr(db), 0,
             ptr(work))
    torch.cuda.synchronize()
    rel = float((dw.cpu().double() - w.grad).norm() / w.grad.norm())
    relb = float((db.cpu().double() - bb.grad).norm() / bb.grad.norm())
    assert rel <= 1e-5 and relb <= 1e-5, (rel, relb)


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("clamp", [0, 1])
def test_conv_last_bicubic_l1(dtype, clamp):
    from src.hip import lib as L, net
    torch.manual_seed(4)
    B, C, h, w_ = 2, 64, 8, 12
    H, W = 4 * h, 4 * w_
    feat = torch.randn(B, C, H, W)
    lr = torch.rand(B, 3, h, w_)
    hr = torch.rand(B, 3, H, W)
    wl = torch.randn(3, C, 3, 3) * 0.01
    bl = torch.randn(3) * 0.01
    out_ref = F.conv2d(feat, wl, bl, padding=1) + O.bicubic(lr.double(), 4).float()
    if clamp:
        out_ref = out_ref.clamp(0, 1)
    n = out_ref.numel()
    ctx = _ctx(dtype)
    wp = _pack(ctx, wl, 0)
    out = ctx.alloc((B, 3, H, W), torch.float32)
    dout = ctx.alloc((B, H, W, 16))
    lp = ctx.alloc((B * net.tiles(H, W), 1), torch.float32)
    net.conv(ctx, nhwc(feat, dtype), wp, B, H, W, C, 3, bias=bl.to(DEV), epi=L.EPI_LAST, y=out, lr=lr.to(DEV),
             scale=4, clamp=clamp, hr=hr.to(DEV), dout=dout, l1_scale=1.0 / n, loss_part=lp)
    torch.cuda.synchronize()
    assert (out.cpu() - out_ref).abs().max() <= (1e-4 if dtype == torch.float32 else 3e-2)
    loss = float(lp.sum()) / n
    assert abs(loss - float((out.cpu() - hr).abs().mean())) < 1e-5
    g = dout.float().cpu()
    assert torch.all(g[..., 3:] == 0)
    sgn = torch.sign(out.cpu() - hr).permute(0, 2, 3, 1) / n
    assert torch.allclose(g[..., :3], sgn.to(g.dtype).float(), rtol=1e-2, atol=0)


def test_conv_last_persistent_ring():
    """The persistent conv_last kernel (csrc/conv_last.hip) over many tiles per CU, with an
    uneven tile count per block (816 tiles): halo ring, deferred loss writes, border tiles.
    Reference on the same bf16-rounded feature map and weights, fp32 on the CPU."""
    from src.hip import lib as L, net
    torch.manual_seed(41)
    B, C, H, W = 3, 64, 256, 272
    feat = torch.randn(B, C, H, W).bfloat16().float()
    lr = torch.rand(B, 3, H // 4, W // 4)
    hr = torch.rand(B, 3, H, W)
    wl = (torch.randn(3, C, 3, 3) * 0.02).bfloat16().float()
    bl = torch.randn(3) * 0.01
    out_ref = (F.conv2d(feat.double(), wl.double(), bl.double(), padding=1) + O.bicubic(lr.double(), 4)).float()
    n = out_ref.numel()
    ctx = _ctx(torch.bfloat16)
    wp = _pack(ctx, wl, 0)
    out = ctx.alloc((B, 3, H, W), torch.float32)
    dout = ctx.alloc((B, H, W, 16))
    lp = ctx.alloc((B * net.tiles(H, W), 1), torch.float32)
    lp.fill_(float("nan"))
    net.conv(ctx, nhwc(feat, torch.bfloat16), wp, B, H, W, C, 3, bias=bl.to(DEV), epi=L.EPI_LAST, y=out,
             lr=lr.to(DEV), scale=4, clamp=0, hr=hr.to(DEV), dout=dout, l1_scale=1.0 / n, loss_part=lp)
    torch.cuda.synchronize()
    o = out.cpu()
    assert (o - out_ref).abs().max() <= 1e-4
    # every tile's partial written, each equal to its tile's |sr - hr| sum
    d = (o - hr).abs().double()
    tile_ref = d.view(B, 3, H // 16, 16, W // 16, 16).sum(dim=(1, 3, 5)).reshape(-1)
    got = lp.cpu().double().view(-1)
    assert torch.isfinite(got).all()
    assert torch.allclose(got, tile_ref, rtol=1e-5, atol=1e-4)
    g = dout.float().cpu()
    assert torch.all(g[..., 3:] == 0)
    diff = (o - hr).permute(0, 2, 3, 1)
    far = diff.abs() > 1e-5
    assert torch.equal(torch.sign(g[..., :3])[far], torch.sign(diff)[far])


def test_bicubic_down4_and_layouts():
    torch.manual_seed(5)
    from src.hip.program import ptr
    ctx = _ctx(torch.float32)
    hr = torch.rand(2, 3, 64, 48)
    lr = ctx.alloc((2, 3, 16, 12), torch.float32)
    hd = hr.to(DEV)
    ctx.emit("down", ctx.lib.fen_bicubic_down4, 2, 3, 64, 48, ptr(hd), ptr(lr))
    torch.cuda.synchronize()
    ref = O.lr_from_hr(hr.double()).float()
    assert (lr.cpu() - ref).abs().max() < 2e-6


@pytest.mark.parametrize("dtype", DT)
def test_se_fwd_apply(dtype):
    from src.hip.program import ptr
    torch.manual_seed(6)
    B, C, Cr, H, W = 3, 64, 16, 16, 16
    t = torch.randn(B, C, H, W)
    x = torch.randn(B, C, H, W)
    w1 = torch.randn(Cr, C) * 0.2
    w2 = torch.randn(C, Cr) * 0.2
    p = {"fc.0.weight": w1, "fc.2.weight": w2}
    s_ref = O.channel_attention(t, p, "")
    y_ref = t * s_ref[:, :, None, None] * 0.2 + x
    ctx = _ctx(dtype)
    td, xd = nhwc(t, dtype), nhwc(x, dtype)
    npart = ctx.lib.fen_pool_parts(H * W)
    part = ctx.alloc((B * npart, C), torch.float32)
    ctx.emit("pool", ctx.lib.fen_pool_dot, ctx.code, B, H * W, C, ptr(td), 0, ptr(part))
    mean = ctx.alloc((B, C), torch.float32)
    hid = ctx.alloc((B, Cr), torch.float32)
    s = ctx.alloc((B, C), torch.float32)
    w1d, w2d = w1.to(DEV), w2.to(DEV)
    ctx.emit("se", ctx.lib.fen_se_fwd, B, C, Cr, npart, 1.0 / (H * W), ptr(part), ptr(w1d), ptr(w2d), ptr(mean),
             ptr(hid), ptr(s))
    y = ctx.alloc((B, H, W, C))
    ctx.emit("apply", ctx.lib.fen_se_apply, ctx.code, B, H * W, C, ptr(td), ptr(s), 0.2, ptr(xd), ptr(y))
    torch.cuda.synchronize()
    tol_s = 1e-5 if dtype == torch.float32 else 3e-3
    assert (s.cpu() - s_ref).abs().max() <= tol_s
    assert (nchw(y) - y_ref).abs().max() <= _tol(dtype, y_ref)


@pytest.mark.parametrize("dtype", DT_FWD)
@pytest.mark.parametrize("B,C,Cr,H,W", [(3, 64, 16, 16, 16), (2, 64, 16, 64, 72), (2, 128, 32, 40, 24),
                                        (2, 32, 16, 16, 16)])
def test_se_fused(dtype, B, C, Cr, H, W):
    """fen_se_fused (gate + apply, several blocks per image) == fen_se_fwd's gate and the
    oracle's channel attention; block 0 of each image writes mean/hid/s."""
    from src.hip.program import ptr
    torch.manual_seed(7)
    t = torch.randn(B, C, H, W)
    x = torch.randn(B, C, H, W)
    w1 = torch.randn(Cr, C) * 0.2
    w2 = torch.randn(C, Cr) * 0.2
    s_ref = O.channel_attention(t, {"fc.0.weight": w1, "fc.2.weight": w2}, "")
    y_ref = t * s_ref[:, :, None, None] * 0.2 + x
    ctx = _ctx(dtype)
    td, xd = nhwc(t, dtype), nhwc(x, dtype)
    npart = ctx.lib.fen_pool_parts(H * W)
    part = ctx.alloc((B * npart, C), torch.float32)
    ctx.emit("pool", ctx.lib.fen_pool_dot, ctx.code, B, H * W, C, ptr(td), 0, ptr(part))
    mean = ctx.alloc((B, C), torch.float32)
    hid = ctx.alloc((B, Cr), torch.float32)
    s = ctx.alloc((B, C), torch.float32)
    w1d, w2d = w1.to(DEV), w2.to(DEV)
    y = ctx.alloc((B, H, W, C))
    ctx.emit("fused", ctx.lib.fen_se_fused, ctx.code, B, H * W, C, Cr, npart, 1.0 / (H * W), ptr(part), ptr(w1d),
             ptr(w2d), ptr(mean), ptr(hid), ptr(s), ptr(td), 0.2, ptr(xd), ptr(y))
    torch.cuda.synchronize()
    tol_s = 1e-5 if dtype == torch.float32 else 3e-3
    assert (s.cpu() - s_ref).abs().max() <= tol_s
    tm = t.to(dtype).float() if dtype != torch.float32 else t
    assert (mean.cpu() - tm.mean((2, 3))).abs().max() <= 1e-5
    assert (nchw(y) - y_ref).abs().max() <= _tol(dtype, y_ref)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 16, 64, 64), (1, 24, 40, 64, 64), (1, 16, 16, 64, 256),
                                             (1, 32, 32, 64, 16), (17, 64, 64, 64, 64), (2, 20, 36, 128, 64),
                                             (3, 32, 48, 64, 256), (2, 64, 64, 64, 64), (3, 40, 56, 64, 64),
                                             (2, 16, 16, 32, 32), (1, 24, 40, 32, 128), (2, 32, 32, 32, 16),
                                             (1, 16, 16, 96, 64), (3, 64, 48, 64, 16)])
def test_wgrad(dtype, B, H, W, Cin, Cout):
    """fen_wgrad3x3 vs autograd of conv2d.  The reference runs in float64 on the operands
    rounded to the compute dtype, so bf16 is held to fp32-accumulation accuracy (rel 1e-5):
    a wrong fragment mapping or a dropped tile shows as O(1).  (17, 64, 64) puts 2 tiles per
    block; Cout 256 / Cin 128 exercise the co-group / ci-group grid; Cout 16 (conv_last's
    padded dL/dsr, 3 valid rows) the persistent kernel's 4-wave 16-channel form at bf16.
    Several jobs per launch: test_wgrad_multi."""
    from src.hip import net
    torch.manual_seed(7)
    x = torch.randn(B, Cin, H, W).to(dtype).float()
    dy = torch.randn(B, Cout, H, W).to(dtype).float()
    w = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    bb = torch.zeros(Cout, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double(), w, bb, padding=1).mul(dy.double()).sum().backward()
    ctx = _ctx(dtype)
    cv = Cout if Cout != 16 else 3
    dw = ctx.alloc((cv, Cin, 3, 3), torch.float32)
    db = ctx.alloc((cv,), torch.float32)
    net.wgrad(ctx, nhwc(x, dtype), nhwc(dy, dtype), B, H, W, Cin, Cout, dw, db, cout_valid=cv)
    torch.cuda.synchronize()
    gw, gb = w.grad[:cv], bb.grad[:cv]
    rel = float((dw.cpu().double() - gw).norm() / gw.norm())
    relb = float((db.cpu().double() - gb).norm() / gb.norm())
    assert rel <= 1e-5 and relb <= 1e-5, (rel, relb)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,B,H,W,Cin,Cout", [(2, 2, 64, 64, 64, 64), (4, 32, 64, 64, 64, 64),
                                               (3, 3, 40, 56, 64, 64), (8, 1, 16, 16, 64, 64),
                                               (4, 17, 64, 64, 64, 64), (2, 2, 32, 32, 64, 256),
                                               (3, 2, 16, 16, 32, 32), (2, 2, 48, 64, 64, 16)])
def test_wgrad_multi(dtype, n, B, H, W, Cin, Cout):
    """fen_wgrad3x3_multi (n jobs of one shape in one launch pair, the CUs split between them)
    vs float64 autograd per job, rel 1e-5 as test_wgrad.  Covers the bench's B=32 64x64 batch
    of 4, ragged tiles, a one-tile job set (8 jobs x 1 tile), the co-group grid (Cout 256), a
    job with accumulate=1 and, for fp32 / 32 channels, the generic kernel run job by job."""
    from src.hip import lib as L
    from src.hip.program import ptr
    torch.manual_seed(11)
    ctx = _ctx(dtype)
    arr = (L.WgradDesc * n)()
    refs, outs, keep = [], [], []
    for i in range(n):
        x = torch.randn(B, Cin, H, W).to(dtype).float()
        dy = torch.randn(B, Cout, H, W).to(dtype).float()
        w = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
        bb = torch.zeros(Cout, dtype=torch.float64, requires_grad=True)
        F.conv2d(x.double(), w, bb, padding=1).mul(dy.double()).sum().backward()
        acc = 1 if i == 1 else 0
        dw0 = torch.randn(Cout, Cin, 3, 3) if acc else torch.zeros(Cout, Cin, 3, 3)
        db0 = torch.randn(Cout) if acc else torch.zeros(Cout)
        refs.append((w.grad + dw0.double() * acc, bb.grad + db0.double() * acc))
        xd, dyd = nhwc(x, dtype), nhwc(dy, dtype)
        dw, db = dw0.to(DEV), db0.to(DEV)
        keep += [xd, dyd]
        outs.append((dw, db))
        d = arr[i]
        d.dtype, d.B, d.H, d.W, d.Cin, d.Cout, d.cout_valid = ctx.code, B, H, W, Cin, Cout, Cout
        d.x, d.dy, d.dw, d.db, d.accumulate = ptr(xd), ptr(dyd), ptr(dw), ptr(db), acc
    import ctypes
    nwork = ctx.lib.fen_wgrad_multi_work_floats(n, ctypes.cast(arr, ctypes.c_void_p))
    assert nwork >= ctx.lib.fen_wgrad_work_floats(ctypes.byref(arr[0]))
    work = ctx.alloc((nwork,), torch.float32)
    arr[0].work = ptr(work)
    L.check(ctx.lib.fen_wgrad3x3_multi(n, ctypes.cast(arr, ctypes.c_void_p), torch.cuda.current_stream().cuda_stream),
            "wgrad_multi")
    torch.cuda.synchronize()
    for (gw, gb), (dw, db) in zip(refs, outs):
        rel = float((dw.cpu().double() - gw).norm() / gw.norm())
        relb = float((db.cpu().double() - gb).norm() / gb.norm())
        assert rel <= 1e-5 and relb <= 1e-5, (rel, relb)


@pytest.mark.parametrize("dtype", DT)
def test_dgrad_prelu_bwd(dtype):
    """dgrad (mode-2 weights) with the fused PReLU backward epilogue."""
    from src.hip import lib as L, net
    torch.manual_seed(8)
    B, H, W, C = 2, 16, 24, 64
    z = torch.randn(B, C, H, W)
    dy = torch.randn(B, C, H, W)
    w = torch.randn(C, C, 3, 3) * 0.05
    a = (torch.rand(C) * 0.5).requires_grad_(True)
    a1 = torch.randn(B, C, H, W, requires_grad=True)
    zz = z.clone().requires_grad_(True)
    # reference: y = conv(prelu(zz)); d/dzz and d/da of sum(y*dy)
    F.conv2d(O.prelu(zz, a), w, None, padding=1).mul(dy).sum().backward()
    ctx = _ctx(dtype)
    wp = _pack(ctx, w, 2)
    dz = ctx.alloc((B, H, W, C))
    T = net.tiles(H, W)
    part = ctx.alloc((B * T, C), torch.float32)
    net.conv(ctx, nhwc(dy, dtype), wp, B, H, W, C, C, epi=L.EPI_PRELU_BWD, alpha=a.detach().to(DEV),
             pre_in=nhwc(z, dtype), y=dz, part=part)
    torch.cuda.synchronize()
    assert (nchw(dz) - zz.grad).abs().max() <= _tol(dtype, zz.grad)
    da = part.sum(0).cpu()
    rel = float((da - a.grad).norm() / a.grad.norm())
    assert rel <= (1e-5 if dtype == torch.float32 else 2e-2), rel


@pytest.mark.parametrize("dtype", DT)
def test_dgrad_unshuffle(dtype):
    from src.hip import lib as L, net
    torch.manual_seed(9)
    B, H, W, C = 1, 32, 32, 64         # dgrad conv output space (2H' x 2W')
    v = torch.randn(B, C, H, W)       # previous stage pre-activation
    dy = torch.randn(B, 4 * C, H, W)  # grad at the next conv's output
    w = torch.randn(4 * C, C, 3, 3) * 0.05
    a = torch.rand(C) * 0.5
    vv = v.clone().requires_grad_(True)
    F.conv2d(O.prelu(vv, a), w, None, padding=1).mul(dy).sum().backward()
    # du = unshuffle(dv): du[b, 4c+2i+j, h, w] = dv[b, c, 2h+i, 2w+j]
    ref = vv.grad.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H // 2, W // 2)
    ctx = _ctx(dtype)
    wp = _pack(ctx, w, 2)
    du = ctx.alloc((B, H // 2, W // 2, 4 * C))
    part = ctx.alloc((B * net.tiles(H, W), C), torch.float32)
    net.conv(ctx, nhwc(dy, dtype), wp, B, H, W, 4 * C, C, epi=L.EPI_PRELU_BWD | L.EPI_UNSHUFFLE, alpha=a.to(DEV),
             pre_in=nhwc(v, dtype), y=du, part=part)
    torch.cuda.synchronize()
    assert (nchw(du) - ref).abs().max() <= _tol(dtype, ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,HW,C,Cr", [(3, 4096, 64, 16), (2, 1024, 32, 8), (1, 256, 64, 16)])
def test_se_bwd_fused_matches_pair(dtype, B, HW, C, Cr):
    """fen_se_bwd_fused == fen_se_bwd + fen_se_bwd_apply bit for bit (the backward of
    ChannelAttention and the RCAB's scaled residual, blocks.py:88-92,150-153), and dt agrees
    with a float64 restatement of the chain."""
    from src.hip import lib as L
    from src.hip.program import ptr
    lib = L.load()
    code = L.dtype_code(dtype)
    stream = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(B * 7 + C)
    npart = int(lib.fen_pool_parts(HW))
    part = torch.randn(B * npart, C, device=DEV)
    mean = torch.randn(B, C, device=DEV) * 0.1
    hid = torch.relu(torch.randn(B, Cr, device=DEV))
    s = torch.sigmoid(torch.randn(B, C, device=DEV))
    w1 = torch.randn(Cr, C, device=DEV) * 0.3
    w2 = torch.randn(C, Cr, device=DEV) * 0.3
    dy = torch.randn(B, HW, C, device=DEV).to(dtype)
    rs = 0.2
    g = torch.empty(B, C, device=DEV)
    dw1p, dw2p = torch.empty(B, Cr * C, device=DEV), torch.empty(B, Cr * C, device=DEV)
    dt = torch.empty_like(dy)
    args = (npart, 1.0 / HW, rs, ptr(part), ptr(mean), ptr(hid), ptr(s), ptr(w1), ptr(w2))
    L.check(lib.fen_se_bwd(B, C, Cr, *args, ptr(g), ptr(dw1p), ptr(dw2p), stream), "se_bwd")
    L.check(lib.fen_se_bwd_apply(code, B, HW, C, ptr(dy), ptr(s), rs, ptr(g), ptr(dt), stream), "se_bwd_apply")
    g2 = torch.full_like(g, 7.0)
    f1, f2 = torch.full_like(dw1p, 7.0), torch.full_like(dw2p, 7.0)
    dt2 = torch.zeros_like(dy)
    L.check(lib.fen_se_bwd_fused(code, B, HW, C, Cr, *args, ptr(dy), ptr(g2), ptr(f1), ptr(f2), ptr(dt2), stream),
            "se_bwd_fused")
    torch.cuda.synchronize()
    assert torch.equal(g2, g)
    assert torch.equal(f1, dw1p) and torch.equal(f2, dw2p)
    assert torch.equal(dt2, dt)
    # float64 restatement: a = sum of partials, dz = a rs s (1-s), dh = relu'(hid) W2^T dz, g = W1^T dh / HW
    a = part.double().view(B, npart, C).sum(1)
    sd = s.double()
    dz = a * rs * sd * (1 - sd)
    dh = (dz @ w2.double()) * (hid.double() > 0)
    gref = dh @ w1.double() / HW
    dtref = dy.double() * rs * sd[:, None, :] + gref[:, None, :]
    tol = {torch.float32: 1e-5, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dtype]
    assert float((dt2.double() - dtref).abs().max() / dtref.abs().max()) <= tol


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 32, 32, 64, 64), (2, 16, 16, 128, 128), (1, 64, 48, 64, 128),
                                             (2, 16, 16, 256, 256), (3, 32, 16, 128, 256)])
def test_s2d_stride2_conv(dtype, B, H, W, Cin, Cout):
    """The discriminator's stride-2 3x3 conv (discriminator.py:47-82) as a stride-1 conv over
    the space-to-depth input (fen_s2d2) with the phase-major filter, only its filled taps run
    (fen_conv_desc.s2d_in / s2d_out): forward, data gradient (mode-2 pack, inverse fen_s2d2)
    and weight gradient (gathered back to OIHW) vs float64 autograd of F.conv2d(stride=2) on
    the same rounded operands; fp32 rel 1e-5, bf16 rel 1e-2 (output rounding) / 1e-5 (wgrad,
    fp32 accumulation of rounded operands)."""
    from src.hip import lib as L, net
    from src.hip.program import ptr
    torch.manual_seed(17)
    x = torch.randn(B, Cin, H, W).to(dtype).float()
    w = (torch.randn(Cout, Cin, 3, 3) * 0.05).to(dtype).float()
    dy = torch.randn(B, Cout, H // 2, W // 2).to(dtype).float()
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    y_ref = F.conv2d(xr, wr, padding=1, stride=2)
    y_ref.mul(dy.double()).sum().backward()
    ctx = _ctx(dtype)
    s = torch.cuda.current_stream().cuda_stream
    Ho, Wo = H // 2, W // 2
    xd = nhwc(x, dtype)
    xs = ctx.alloc((B, Ho, Wo, 4 * Cin))
    L.check(ctx.lib.fen_s2d2(ctx.code, B, H, W, Cin, ptr(xd), ptr(xs), 0, s), "s2d")
    w4 = net.s2d_filter(w.to(DEV))
    y = ctx.alloc((B, Ho, Wo, Cout))
    net.conv(ctx, xs, _pack(ctx, w4, 0), B, Ho, Wo, 4 * Cin, Cout, y=y, s2d_in=Cin)
    dyd = nhwc(dy, dtype)
    dxs = ctx.alloc((B, Ho, Wo, 4 * Cin))
    net.conv(ctx, dyd, _pack(ctx, w4, 2), B, Ho, Wo, Cout, 4 * Cin, y=dxs, s2d_out=Cin)
    dx = ctx.alloc((B, H, W, Cin))
    L.check(ctx.lib.fen_s2d2(ctx.code, B, H, W, Cin, ptr(dxs), ptr(dx), 1, s), "s2d_inv")
    dw4 = torch.zeros(Cout, 4 * Cin, 3, 3, device=DEV)
    net.wgrad(ctx, xs, dyd, B, Ho, Wo, 4 * Cin, Cout, dw4, None)
    dw = torch.empty(Cout, Cin, 3, 3, device=DEV)
    net.s2d_filter_grad(dw4, dw)
    torch.cuda.synchronize()
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(nchw(y), y_ref.detach()) <= tol
    assert rel(nchw(dx), xr.grad) <= tol
    assert rel(dw.cpu(), wr.grad) <= 1e-5
    # the s2d round trip is exact
    back = ctx.alloc((B, H, W, Cin))
    L.check(ctx.lib.fen_s2d2(ctx.code, B, H, W, Cin, ptr(xs), ptr(back), 1, s), "s2d_inv")
    torch.cuda.synchronize()
    assert torch.equal(back, xd)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,H,W,C", [(2, 64, 64, 64), (1, 36, 20, 64), (1, 40, 24, 32), (1, 32, 32, 128),
                                     (3, 256, 256, 64)])
def test_conv_last_dgrad(dtype, B, H, W, C):
    """fen_conv_last_dgrad (conv_last^T 3 -> C + the last upsampler stage's PReLU backward +
    PixelShuffle inverse + dalpha partials) against torch autograd of conv(prelu(v)) in fp32;
    16-bit at C = 64 runs the persistent pipelined kernel (k_cld_p) when the tiles are whole,
    other 16-bit C <= 64 the LDS pre-activation tile, the rest the per-pixel reads; H = 36 leaves
    a partial tile row; 3 x 256^2 has 768 tiles for 512 blocks (blocks take one or two tiles)."""
    from src.hip.program import ptr
    torch.manual_seed(21)
    Co = 3
    v = torch.randn(B, C, H, W)
    a = (torch.rand(C) * 0.5).requires_grad_(True)
    w = torch.randn(Co, C, 3, 3) * 0.05
    g = torch.randn(B, Co, H, W)
    ctx = _ctx(dtype)
    vq = nhwc(v, dtype)
    vv = nchw(vq).requires_grad_(True)            # the rounded operand the kernel sees
    F.conv2d(O.prelu(vv, a), w, None, padding=1).mul(g).sum().backward()
    ref = vv.grad.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H // 2, W // 2)
    dout = torch.zeros(B, H, W, 16)
    dout[..., :Co] = g.permute(0, 2, 3, 1)
    gq = dout.to(DEV, dtype)
    du = ctx.alloc((B, H // 2, W // 2, 4 * C))
    rows = ctx.lib.fen_conv_last_dgrad_part_rows(B, H, W)
    part = ctx.alloc((rows, C), torch.float32)
    wd, ad = w.to(DEV).contiguous(), a.detach().to(DEV)
    ctx.emit("conv_last_dgrad", ctx.lib.fen_conv_last_dgrad, ctx.code, B, H, W, C, Co, ptr(gq), ptr(wd), ptr(vq),
             None, ptr(ad), ptr(du), ptr(part))
    torch.cuda.synchronize()
    if dtype != torch.float32:                    # dout rounded to 16 bits too: compare against that
        gg = gq[..., :Co].float().cpu().permute(0, 3, 1, 2)
        vv.grad = None
        a.grad = None
        F.conv2d(O.prelu(vv, a), w, None, padding=1).mul(gg).sum().backward()
        ref = vv.grad.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H // 2, W // 2)
    assert (nchw(du) - ref).abs().max() <= _tol(dtype, ref)
    da = part.sum(0).cpu()
    rel = float((da - a.grad).norm() / a.grad.norm())
    assert rel <= (1e-5 if dtype == torch.float32 else 1e-4), rel


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("amode", ["pos", "mixed"])
@pytest.mark.parametrize("B,H,W,Co", [(2, 64, 64, 3), (3, 256, 256, 3), (1, 16, 48, 1)])
def test_conv_last_bwd(dtype, amode, B, H, W, Co):
    """fen_conv_last_bwd (conv_last's data, slope, weight and bias gradients in one MFMA pass)
    against torch autograd in fp32: du and dalpha of conv(prelu(v)) on the pre-activation the
    kernel sees (v where it reads pre, a / alpha recovered from post), dW / db of conv(a).  pre is NaN in the groups whose slopes are all > 0
    (read from post), post NaN in the others (read from pre, a rebuilt as rnd16(PReLU(v)))."""
    from src.hip.program import ptr
    torch.manual_seed(31)
    C = 64
    ctx = _ctx(dtype)
    assert ctx.lib.fen_conv_last_bwd_supported(ctx.code, B, H, W, C, Co)
    alpha = torch.rand(C) * 0.4 + 0.05
    if amode == "mixed":
        alpha[5], alpha[9], alpha[40] = -0.2, 0.0, -0.05
    mixed = torch.zeros(C, dtype=torch.bool)
    for c in range(0, C, 4):
        mixed[c:c + 4] = bool((alpha[c:c + 4] <= 0).any())
    v = torch.randn(B, H, W, C).to(dtype).float()                 # the stored pre-activation
    a = O.prelu(v.permute(0, 3, 1, 2), alpha).permute(0, 2, 3, 1).to(dtype).float()   # rnd16(PReLU(v))
    pre = v.to(DEV, dtype)
    pre[..., ~mixed.to(DEV)] = float("nan")
    post = a.to(DEV, dtype)
    post[..., mixed.to(DEV)] = float("nan")
    w = torch.randn(Co, C, 3, 3) * 0.05
    g = torch.randn(B, Co, H, W)
    dout = torch.zeros(B, H, W, 16)
    dout[..., :Co] = g.permute(0, 2, 3, 1)
    gq = dout.to(DEV, dtype)
    gg = gq[..., :Co].float().cpu().permute(0, 3, 1, 2)
    rows = ctx.lib.fen_conv_last_dgrad_part_rows(B, H, W)
    du = ctx.alloc((B, H // 2, W // 2, 4 * C))
    dal = ctx.alloc((rows, C), torch.float32)
    dwp = ctx.alloc((rows, Co * C * 9), torch.float32)
    dbp = ctx.alloc((rows, Co), torch.float32)
    wd, ad = w.to(DEV).contiguous(), alpha.to(DEV)
    ctx.emit("conv_last_bwd", ctx.lib.fen_conv_last_bwd, ctx.code, B, H, W, C, Co, ptr(gq), ptr(wd), ptr(pre),
             ptr(post), ptr(ad), ptr(du), ptr(dal), ptr(dwp), ptr(dbp))
    torch.cuda.synchronize()
    # the pre-activation the kernel sees: v where it reads pre, a / alpha recovered from post
    vk = torch.where(mixed, v, torch.where(a > 0, a, a / alpha))
    vv = vk.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    al = alpha.clone().requires_grad_(True)
    F.conv2d(O.prelu(vv, al), w, None, padding=1).mul(gg).sum().backward()
    ref = vv.grad.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H // 2, W // 2)
    assert bool(torch.isfinite(du.float()).all())
    assert (nchw(du) - ref).abs().max() <= _tol(dtype, ref)
    rel = float((dal.sum(0).cpu() - al.grad).norm() / al.grad.norm())
    assert rel <= 5e-4, rel
    aa = a.permute(0, 3, 1, 2).contiguous()
    wr = w.clone().requires_grad_(True)
    br = torch.zeros(Co, requires_grad=True)
    F.conv2d(aa, wr, br, padding=1).mul(gg).sum().backward()
    dw = dwp.sum(0).cpu().reshape(Co, C, 3, 3)
    db = dbp.sum(0).cpu()
    assert float((dw - wr.grad).norm() / wr.grad.norm()) <= 1e-4
    assert float((db - br.grad).abs().max()) <= 1e-4 * max(1.0, float(br.grad.abs().max()))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("amode", ["pos", "mixed"])
@pytest.mark.parametrize("H,W", [(16, 16), (8, 64)])
def test_pre_elide_upsampler(dtype, amode, H, W):
    """fen_conv_desc.pre_elide / post_in and fen_conv_last_dgrad's post: the upsampler stage's
    forward skips y_pre where every slope of its 64-channel block is > 0 (left NaN here), and the
    backward kernels recover v = a > 0 ? a : a / alpha for 4-channel groups whose slopes are all
    > 0 and read pre only for the others -- pre is NaN wherever it must not be read.  Results
    against torch autograd of conv(prelu(v)) on the kernel's own rounded v."""
    from src.hip import lib as L, net
    from src.hip.program import ptr
    torch.manual_seed(23)
    B, C = 2, 64
    alpha = torch.rand(C) * 0.4 + 0.05
    if amode == "mixed":
        alpha[5], alpha[9], alpha[40] = -0.2, 0.0, -0.05
    mixed_grp = torch.zeros(C, dtype=torch.bool)
    for c in range(0, C, 4):
        mixed_grp[c:c + 4] = bool((alpha[c:c + 4] <= 0).any())
    ctx = _ctx(dtype)
    x = torch.randn(B, C, H, W)
    w_up = torch.randn(4 * C, C, 3, 3) * 0.05
    b_up = torch.randn(4 * C) * 0.1
    wp = _pack(ctx, w_up, 1)
    a = ctx.alloc((B, 2 * H, 2 * W, C))
    v = torch.full((B, 2 * H, 2 * W, C), float("nan"), device=DEV, dtype=dtype)
    net.conv(ctx, nhwc(x, dtype), wp, B, H, W, C, 4 * C, bias=b_up.to(DEV), epi=L.EPI_PRELU | L.EPI_SHUFFLE,
             alpha=alpha.to(DEV), y=a, y_pre=v, pre_elide=1)
    torch.cuda.synchronize()
    if amode == "pos":
        assert bool(torch.isnan(v).all())                  # not written
        vref = torch.where(a.float() > 0, a.float(), a.float() / alpha.to(DEV))
    else:
        assert bool(torch.isfinite(v).all())               # the block has a slope <= 0: written
        vref = v.float()
    # backward 1: conv_last dgrad from (pre with NaN in the recoverable groups, post = a)
    Co, Hs, Ws = 3, 2 * H, 2 * W
    pre_bwd = v.clone()
    pre_bwd[..., ~mixed_grp.to(DEV)] = float("nan")
    wl = torch.randn(Co, C, 3, 3) * 0.05
    g = torch.randn(B, Co, Hs, Ws)
    dout = torch.zeros(B, Hs, Ws, 16)
    dout[..., :Co] = g.permute(0, 2, 3, 1)
    gq = dout.to(DEV, dtype)
    du = ctx.alloc((B, H, W, 4 * C))
    part = ctx.alloc((ctx.lib.fen_conv_last_dgrad_part_rows(B, Hs, Ws), C), torch.float32)
    wld, ad = wl.to(DEV).contiguous(), alpha.to(DEV)
    ctx.emit("conv_last_dgrad", ctx.lib.fen_conv_last_dgrad, ctx.code, B, Hs, Ws, C, Co, ptr(gq), ptr(wld),
             ptr(pre_bwd), ptr(a), ptr(ad), ptr(du), ptr(part))
    torch.cuda.synchronize()
    vv = vref.cpu().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    al = alpha.clone().requires_grad_(True)
    gg = gq[..., :Co].float().cpu().permute(0, 3, 1, 2)
    F.conv2d(O.prelu(vv, al), wl, None, padding=1).mul(gg).sum().backward()
    ref = vv.grad.reshape(B, C, H, 2, W, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H, W)
    assert bool(torch.isfinite(du.float()).all())
    assert (nchw(du) - ref).abs().max() <= _tol(dtype, ref)
    rel = float((part.sum(0).cpu() - al.grad).norm() / al.grad.norm())
    # "mixed": the reference's v is the kernel's rounded v, the kernel's recovered a / alpha
    # differs from it by the output rounding (bf16: 2^-9 relative) in the recovered groups
    assert rel <= (1e-3 if amode == "pos" else 1e-2), rel
    # backward 2: the stage dgrad epilogue (PRELU_BWD | UNSHUFFLE) with pre_in / post_in
    w2 = torch.randn(4 * C, C, 3, 3) * 0.05
    dy = torch.randn(B, 4 * C, Hs, Ws)
    wp2 = _pack(ctx, w2, 2)
    du2 = ctx.alloc((B, H, W, 4 * C))
    part2 = ctx.alloc((B * net.tiles(Hs, Ws), C), torch.float32)
    net.conv(ctx, nhwc(dy, dtype), wp2, B, Hs, Ws, 4 * C, C, epi=L.EPI_PRELU_BWD | L.EPI_UNSHUFFLE, alpha=ad,
             pre_in=pre_bwd, post_in=a, y=du2, part=part2)
    torch.cuda.synchronize()
    vv.grad = None
    al.grad = None
    dyq = nhwc(dy, dtype).float().cpu().permute(0, 3, 1, 2)
    F.conv2d(O.prelu(vv, al), w2, None, padding=1).mul(dyq).sum().backward()
    ref2 = vv.grad.reshape(B, C, H, 2, W, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H, W)
    assert bool(torch.isfinite(du2.float()).all())
    assert (nchw(du2) - ref2).abs().max() <= _tol(dtype, ref2)
    rel2 = float((part2.sum(0).cpu() - al.grad).norm() / al.grad.norm())
    assert rel2 <= 2e-2, rel2


def test_colsum_multi_split_jobs():
    """fen_colsum_multi over the shapes the backward queues (the strip backward's slope rows
    2048 x 64, conv_last's 8192 x 64, the SE rows 32 x 1024, a ragged 1000 x 96, the loss column),
    tall narrow jobs split into row slices with an ordered last-block combine: column sums
    (scaled, one accumulated) against float64 torch, and bit-identical on a repeat."""
    import ctypes
    from src.hip import lib as L
    torch.manual_seed(31)
    shapes = [(2048, 64), (8192, 64), (32, 1024), (1000, 96), (4096, 1), (700, 16)]
    parts = [torch.randn(r, c, device=DEV) for r, c in shapes]
    outs = [torch.randn(c, device=DEV) for _, c in shapes]
    init = [o.clone() for o in outs]
    lib = L.load()

    def run():
        arr = (L.ColsumJob * len(shapes))()
        for i, ((r, c), p, o) in enumerate(zip(shapes, parts, outs)):
            arr[i].part, arr[i].out, arr[i].rows, arr[i].cols = p.data_ptr(), o.data_ptr(), r, c
            arr[i].scale, arr[i].accumulate = 0.5, int(i == 2)
        L.check(lib.fen_colsum_multi(len(shapes), ctypes.cast(arr, ctypes.c_void_p),
                                     torch.cuda.current_stream().cuda_stream), "colsum_multi")
        torch.cuda.synchronize()

    run()
    for i, (p, o) in enumerate(zip(parts, outs)):
        ref = p.double().sum(0) * 0.5 + (init[i].double() if i == 2 else 0.0)
        assert float((o.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max())), i
    first = [o.clone() for o in outs]
    for i in range(len(outs)):
        if i == 2:
            outs[i].copy_(init[i])
    run()
    for a, b in zip(first, outs):
        assert torch.equal(a, b)
