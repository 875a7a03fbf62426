"""k_conv3x3_v (conv3x3.hip): the DMA-fed persistent conv that fen_conv3x3 takes for 16-bit convs
with Cin a multiple of 64 above 64 and Cout a multiple of 128 -- VGG19's conv2_2 .. conv3_4 and
their data gradients (perceptual.py:13-169), the discriminator's wide layers
(discriminator.py:58-90).  Against torch fp32 (F.conv2d on the same 16-bit operands) for every
epilogue mode it is instantiated for, partial tiles (H, W not multiples of 16), several tiles
per block and several 128-channel output tiles; and bit-identical between a one-block-per-tile
grid and a persistent grid (the pipeline across tiles) -- by comparing against the streamed
kernel (FEN_CONV_V=0 in a subprocess would be heavier: the two kernels sum the same 16-bit
products in fp32 in different orders, so that comparison is at fp32-rounding tolerance)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(dtype, B, H, W, Cin, Cout, seed=0):
    from src.hip.program import Ctx, ptr
    torch.manual_seed(seed)
    ctx = Ctx(dtype, DEV)
    x = torch.randn(B, H, W, Cin).to(dtype)
    w = (torch.randn(Cout, Cin, 3, 3) * (1.0 / (3 * Cin ** 0.5))).to(dtype).float()
    n = ctx.lib.fen_packed_elems(0, Cout, Cin)
    wp = torch.empty(n, dtype=dtype, device=DEV)
    wd = w.to(DEV).contiguous()
    ctx.emit("pack", ctx.lib.fen_pack_conv_w, ctx.code, 0, Cout, Cin, ptr(wd), ptr(wp))
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w, None, padding=1).permute(0, 2, 3, 1)   # NHWC fp32
    return ctx, x.to(DEV), wp, ref


def _close(got, ref, dtype):
    tol = (4e-3 if dtype == torch.bfloat16 else 1e-3) * float(ref.abs().max())
    err = float((got.float().cpu() - ref).abs().max())
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 32, 32, 128, 128), (3, 40, 24, 256, 128), (1, 16, 16, 512, 256),
                                             (2, 8, 8, 512, 512), (4, 64, 64, 128, 256)])
def test_wide_conv_bias_relu_and_pre(dtype, B, H, W, Cin, Cout):
    """bias + ReLU (PReLU with zero slopes: VGG's conv + ReLU) with the pre-activation copy
    (a VGG feature layer), and bias only (the feature layer that ends the extractor)."""
    from src.hip import lib as L, net
    ctx, x, wp, ref = _setup(dtype, B, H, W, Cin, Cout)
    b = torch.randn(Cout) * 0.1
    ref = ref + b
    y = torch.empty(B, H, W, Cout, device=DEV, dtype=dtype)
    yp = torch.empty_like(y)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, bias=b.to(DEV), epi=L.EPI_PRELU, alpha=torch.zeros(Cout, device=DEV),
             y=y, y_pre=yp)
    y2 = torch.empty_like(y)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, bias=b.to(DEV), y=y2)
    torch.cuda.synchronize()
    _close(yp, ref, dtype)
    _close(y2, ref, dtype)
    _close(y, ref.clamp_min(0), dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16])
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 32, 32, 256, 256), (3, 24, 40, 128, 128)])
def test_wide_conv_dgrad_relu_mask_and_plain(dtype, B, H, W, Cin, Cout):
    """the data-gradient modes: PReLU backward against a saved activation with its slope
    partials (VGG's mode-2 convs through a ReLU, zero slopes: dalpha = sum dy * pre where
    pre <= 0), and no epilogue (a gradient into a max pool / the discriminator's BN)."""
    from src.hip import lib as L, net
    ctx, x, wp, ref = _setup(dtype, B, H, W, Cin, Cout, seed=1)
    pre = torch.randn(B, H, W, Cout).to(dtype)
    alpha = torch.full((Cout,), 0.25)
    tiles = ((H + 15) // 16) * ((W + 15) // 16)
    part = torch.empty(B * tiles, Cout, device=DEV)
    y = torch.empty(B, H, W, Cout, device=DEV, dtype=dtype)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, epi=L.EPI_PRELU_BWD, alpha=alpha.to(DEV), pre_in=pre.to(DEV), y=y,
             part=part)
    y0 = torch.empty_like(y)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, y=y0)
    torch.cuda.synchronize()
    _close(y0, ref, dtype)
    pf = pre.float()
    _close(y, torch.where(pf > 0, ref, 0.25 * ref), dtype)
    dal = (ref * torch.where(pf > 0, torch.zeros_like(pf), pf)).sum((0, 1, 2))
    got = part.cpu().sum(0)
    assert float((got - dal).abs().max()) <= 1e-2 * float(dal.abs().max()) + 1e-3


def test_wide_conv_deterministic_and_grid_independent():
    """Two launches give identical bits, and a tile's result does not depend on which block (or
    how many tiles before it in the same block) computed it: the batch's first image computed
    alone (one tile chain per block) equals it computed inside a batch of 9."""
    from src.hip import net
    dtype = torch.bfloat16
    ctx, x, wp, ref = _setup(dtype, 9, 48, 48, 256, 256, seed=2)
    y1 = torch.empty(9, 48, 48, 256, device=DEV, dtype=dtype)
    y2 = torch.empty_like(y1)
    y3 = torch.empty(1, 48, 48, 256, device=DEV, dtype=dtype)
    net.conv(ctx, x, wp, 9, 48, 48, 256, 256, y=y1)
    net.conv(ctx, x, wp, 9, 48, 48, 256, 256, y=y2)
    net.conv(ctx, x[:1].contiguous(), wp, 1, 48, 48, 256, 256, y=y3)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.equal(y1[:1], y3)
    _close(y1, ref, dtype)
