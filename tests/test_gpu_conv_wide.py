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


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 40, 24, 64, 64), (2, 32, 32, 64, 128), (3, 24, 40, 128, 128),
                                             (2, 16, 48, 256, 256), (2, 20, 20, 128, 64), (1, 16, 16, 96, 32)])
def test_relu_bwd_mask(dtype, B, H, W, Cin, Cout):
    """FEN_EPI_RELU_BWD (the frozen VGG19's data gradients through its ReLUs, no slope partials):
    y = pre > 0 ? conv : 0 on every kernel fen_conv3x3 routes it to -- the ping-pong persistent
    kernel (Cin 64), the DMA-fed wide kernel (Cin >= 128, Cout % 128), the streamed kernel (other
    shapes, f32) -- against torch fp32, and equal to PRELU_BWD with zero slopes where both run on
    the same kernel (the wide one)."""
    from src.hip import lib as L, net
    ctx, x, wp, ref = _setup(dtype, B, H, W, Cin, Cout, seed=3)
    pre = torch.randn(B, H, W, Cout).to(dtype)
    pre[0, 0, :4] = 0                                        # pre == 0: no gradient (torch: relu'(0) = 0)
    y = torch.empty(B, H, W, Cout, device=DEV, dtype=dtype)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, epi=L.EPI_RELU_BWD, pre_in=pre.to(DEV), y=y)
    torch.cuda.synchronize()
    exp = torch.where(pre.float() > 0, ref, torch.zeros_like(ref))
    if dtype == torch.float32:
        assert float((y.cpu() - exp).abs().max()) <= 1e-4 * float(exp.abs().max())
    else:
        _close(y, exp, dtype)
    assert bool((y.cpu().float()[pre.float() <= 0] == 0).all())
    if Cin >= 128 and Cout % 128 == 0 and dtype != torch.float32:
        tiles = ((H + 15) // 16) * ((W + 15) // 16)
        part = torch.empty(B * tiles, Cout, device=DEV)
        y2 = torch.empty_like(y)
        net.conv(ctx, x, wp, B, H, W, Cin, Cout, epi=L.EPI_PRELU_BWD, alpha=torch.zeros(Cout, device=DEV),
                 pre_in=pre.to(DEV), y=y2, part=part)
        torch.cuda.synchronize()
        assert torch.equal(y, y2)


def test_relu_bwd_refusals():
    """RELU_BWD needs pre_in and does not combine with the other pre_in modes."""
    from src.hip import lib as L, net
    ctx, x, wp, ref = _setup(torch.bfloat16, 1, 16, 16, 64, 64)
    y = torch.empty(1, 16, 16, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(L.FenError):
        net.conv(ctx, x, wp, 1, 16, 16, 64, 64, epi=L.EPI_RELU_BWD, y=y)
    with pytest.raises(L.FenError):
        net.conv(ctx, x, wp, 1, 16, 16, 64, 64, epi=L.EPI_RELU_BWD | L.EPI_PRELU_BWD, pre_in=y, y=y,
                 alpha=torch.zeros(64, device=DEV), part=torch.empty(1, 64, device=DEV))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B,H,W,Cin,Cout,keep", [(4, 64, 64, 64, 64, 2), (2, 48, 40, 64, 128, 0),
                                                  (16, 64, 64, 128, 128, 4), (2, 16, 16, 128, 128, 1),
                                                  (3, 40, 24, 256, 256, 0), (2, 18, 22, 96, 64, 1)])
def test_fused_maxpool(dtype, B, H, W, Cin, Cout, keep):
    """fen_conv_desc.y_pool (VGG19's conv -> ReLU -> 'M', perceptual.py:50-53): the 2x2 max pool of
    the ReLU output stored from the epilogue on the persistent kernels (Cin 64: ping-pong; Cin >= 128,
    Cout % 128, enough tiles: DMA-fed wide), or by a second launch on every other route (small grids,
    Cin 96, f32).  y_pool equals torch's max_pool2d of the kernel's own y bit for bit (max commutes
    with the rounding), and y_images keeps y exact for the first `keep` images."""
    from src.hip import lib as L, net
    ctx, x, wp, ref = _setup(dtype, B, H, W, Cin, Cout, seed=4)
    b = torch.randn(Cout) * 0.1
    ref = (ref + b).clamp_min(0)
    y = torch.zeros(B, H, W, Cout, device=DEV, dtype=dtype)
    yp = torch.empty(B, H // 2, W // 2, Cout, device=DEV, dtype=dtype)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, bias=b.to(DEV), epi=L.EPI_PRELU, alpha=torch.zeros(Cout, device=DEV),
             y=y, y_pool=yp, y_images=keep)
    y_all = torch.empty_like(y)
    net.conv(ctx, x, wp, B, H, W, Cin, Cout, bias=b.to(DEV), epi=L.EPI_PRELU, alpha=torch.zeros(Cout, device=DEV),
             y=y_all)
    torch.cuda.synchronize()
    n = keep or B
    assert torch.equal(y[:n], y_all[:n])
    pooled = F.max_pool2d(y_all.float().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1).to(dtype)
    assert torch.equal(yp, pooled)
    if dtype == torch.float32:
        assert float((y_all.cpu() - ref).abs().max()) <= 1e-4 * float(ref.abs().max())
    else:
        _close(y_all, ref, dtype)


def test_fused_maxpool_refusals():
    """y_pool needs the PReLU epilogue and even H, W; y_images needs y_pool and 0 <= y_images <= B."""
    from src.hip import lib as L, net
    ctx, x, wp, ref = _setup(torch.bfloat16, 2, 16, 16, 64, 64)
    y = torch.empty(2, 16, 16, 64, device=DEV, dtype=torch.bfloat16)
    yp = torch.empty(2, 8, 8, 64, device=DEV, dtype=torch.bfloat16)
    z = torch.zeros(64, device=DEV)
    with pytest.raises(L.FenError):
        net.conv(ctx, x, wp, 2, 16, 16, 64, 64, y=y, y_pool=yp)                      # no PReLU epilogue
    with pytest.raises(L.FenError):
        net.conv(ctx, x, wp, 2, 16, 16, 64, 64, epi=L.EPI_PRELU, alpha=z, y=y, y_images=1)   # no y_pool
    with pytest.raises(L.FenError):
        net.conv(ctx, x, wp, 2, 16, 16, 64, 64, epi=L.EPI_PRELU, alpha=z, y=y, y_pool=yp, y_images=3)
    with pytest.raises(L.FenError):
        net.conv(ctx, x[:, :15].contiguous(), wp, 2, 15, 16, 64, 64, epi=L.EPI_PRELU, alpha=z, y=y, y_pool=yp)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,H,W,res", [(2, 64, 48, True), (3, 40, 24, False), (1, 16, 16, True)])
def test_thin_conv_cout16(dtype, B, H, W, res):
    """Cin 64 -> Cout 16 on the one-group persistent kernel with a 16-row resident filter: VGG
    conv1_1's data gradient added into dL/dsr (perceptual.py:84-95; residual = the L1 term)."""
    from src.hip import net
    ctx, x, wp, ref = _setup(dtype, B, H, W, 64, 16, seed=5)
    r = torch.randn(B, H, W, 16).to(dtype)
    y = torch.empty(B, H, W, 16, device=DEV, dtype=dtype)
    net.conv(ctx, x, wp, B, H, W, 64, 16, y=y, res=(r.to(DEV),) if res else ())
    torch.cuda.synchronize()
    _close(y, ref + (r.float() if res else 0), dtype)
