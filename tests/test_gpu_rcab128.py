"""GPU parity of fen_rcab_c128 -- the 128-channel ResidualGroup (BASELINE configs[4]: reference
blocks.py:161-189 with num_channels = 128, Cr = 32; RCAB blocks.py:135-153, ChannelAttention
blocks.py:83-92) as 2 * nb + 1 launches (conv1 with the previous RCAB's gate deferred into its
input, conv2 with the pool sums in its epilogue, the group conv with the last gate and the skip)
-- against the CPU oracle's residual_group on the same 16-bit-rounded weights and input, and
against the per-op launches (fen_conv3x3 + fen_se_fused).

Tolerances as test_gpu_group_strip.py: the kernels round x_j, a1 and t to the 16-bit format, so
the group output is compared at rel-L2 <= 5e-3 (bf16) / 1e-3 (fp16) per RCAB + 1, every gate s
within 2e-3.  A wrong halo row, tap, ring slot or gate shows up as O(1).  Shapes: the stress
config's (B=4, 128x128: 256 tiles = one per CU), one tile column (W=64), more tiles than CUs
(B=5, 320 tiles: blocks walk 2 tiles, the gate recomputed per image), a single tile row (H=4),
non-square images; graph replays are bit-identical."""
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"bf16": torch.bfloat16, "fp16": torch.float16}
C, CR = 128, 32


def _params(n, seed):
    g = torch.Generator().manual_seed(seed)
    q = {}
    for j in range(n):
        b = f"rg.blocks.{j}."
        q[b + "conv1.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.042
        q[b + "conv1.bias"] = torch.randn(C, generator=g) * 0.1
        q[b + "prelu.weight"] = torch.rand(C, generator=g) * 0.5
        q[b + "conv2.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.042
        q[b + "conv2.bias"] = torch.randn(C, generator=g) * 0.1
        q[b + "channel_attention.fc.0.weight"] = torch.randn(CR, C, generator=g) * 0.2
        q[b + "channel_attention.fc.2.weight"] = torch.randn(C, CR, generator=g) * 0.3
    q["rg.conv.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.035
    q["rg.conv.bias"] = torch.randn(C, generator=g) * 0.1
    return q


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def _run(q, n, x_nhwc, dtype, c128=True, record=False, ctx=None):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.RCAB_C128
    net.RCAB_C128 = c128
    try:
        ctx = ctx or Ctx(dtype, DEV, record=record)
        pd = {k: v.to(DEV) for k, v in q.items()}
        Wt = Weights(pd, dtype, DEV)
        ctx.keep(Wt)
        attn = {}
        fw = Forward(NetSpec(C=C, G=1, NB=n, Cr=CR), ctx, Wt, save=False, attn=attn)
        used = fw._c128_ok(x_nhwc)
        y, _ = fw.group(x_nhwc, 0, pre="rg.")
        if not record:
            torch.cuda.synchronize()
    finally:
        net.RCAB_C128 = old
    return y, attn, ctx, used


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
@pytest.mark.parametrize("B,H,W,n", [(4, 128, 128, 2), (2, 64, 64, 3), (5, 128, 128, 1), (1, 4, 64, 2),
                                     (2, 12, 192, 2), (1, 64, 128, 1)])
def test_rcab128_group_vs_oracle(prec, B, H, W, n):
    dtype = DT[prec]
    q = _params(n, seed=41 + n)
    g = torch.Generator().manual_seed(8)
    x = torch.randn(B, C, H, W, generator=g).to(dtype).float()
    qr = {k: (v.to(dtype).float() if v.dim() == 4 else v) for k, v in q.items()}
    attn_ref = {}
    ref = O.residual_group(x, qr, "rg.", n, 0.2, attn=attn_ref)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    y, attn, _, used = _run(q, n, xd, dtype)
    assert used, "outside fen_rcab_c128's envelope"
    out = y.float().cpu().permute(0, 3, 1, 2)
    tol = (5e-3 if prec == "bf16" else 1e-3) * (n + 1)
    r = _rel(out, ref)
    print(f"{prec} B={B} H={H} W={W} n={n}: rel {r:.2e}")
    assert r <= tol, r
    assert sorted(attn) == sorted(attn_ref)
    for k in attn:
        assert float((attn[k].cpu() - attn_ref[k]).abs().max()) <= 2e-3, k


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_rcab128_vs_perop(prec):
    """The fused launches and the per-op path agree at the stress shape with 4 RCABs (both round
    the same tensors; summation orders differ): rel-L2 <= 2e-3 (bf16) / 5e-4 (fp16) per RCAB."""
    dtype = DT[prec]
    n = 4
    q = _params(n, seed=6)
    x = torch.randn(4, 128, 128, C, generator=torch.Generator().manual_seed(10)).to(DEV, dtype)
    yf, attn_f, _, used = _run(q, n, x, dtype, c128=True)
    yp, attn_p, _, used_p = _run(q, n, x, dtype, c128=False)
    assert used and not used_p
    r = _rel(yf.float(), yp.float())
    print(f"{prec}: fused vs per-op rel {r:.2e}")
    assert r <= (2e-3 if prec == "bf16" else 5e-4) * n, r
    for k in attn_f:
        assert float((attn_f[k] - attn_p[k]).abs().max()) <= 2e-3, k


def test_rcab128_graph_replay():
    """Recorded and replayed from a hipGraph five times: bit-identical to the eager launches
    (deterministic: fixed-order tile sums, no atomics)."""
    dtype = torch.float16
    n = 3
    q = _params(n, seed=13)
    x = torch.randn(4, 128, 128, C, generator=torch.Generator().manual_seed(3)).to(DEV, dtype)
    y_e, _, _, _ = _run(q, n, x, dtype)
    y, _, ctx, _ = _run(q, n, x, dtype, record=True)
    assert [op[0] for op in ctx.ops] == ["rcab_c128_conv1", "rcab_c128_conv2"] * n + ["rcab_c128_group_conv"]
    ctx.run()
    torch.cuda.synchronize()
    assert torch.equal(y, y_e)
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        ctx.run()
    for _ in range(5):
        y.zero_()
        gph.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, y_e)


def test_rcab128_conv_modes_vs_torch():
    """Each mode alone against torch fp32 on the same rounded operands (B=2, 64x128, fp16):
    mode 1 without a gate = PReLU(conv + b) and its z1 copy; mode 2 = conv + b and the per-tile
    channel sums of the fp32 result; mode 3 without a gate = conv + b + res."""
    from src.hip import lib as L
    from src.hip.net import Weights
    from src.hip.program import Ctx
    dtype = torch.float16
    B, H, W = 2, 64, 128
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, C, H, W, generator=g).to(dtype).float()
    res = torch.randn(B, C, H, W, generator=g).to(dtype).float()
    w = (torch.randn(C, C, 3, 3, generator=g) * 0.04).to(dtype).float()
    bias = torch.randn(C, generator=g) * 0.1
    alpha = torch.rand(C, generator=g) * 0.5
    ctx = Ctx(dtype, DEV)
    Wt = Weights({"c.weight": w.to(DEV), "c.bias": bias.to(DEV)}, dtype, DEV)
    wp = Wt.packed("c", 0)
    conv = torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), padding=1)
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)   # noqa: E731
    xd, rd = nhwc(x), nhwc(res)
    bd, ad = bias.to(DEV), alpha.to(DEV)
    T = int(ctx.lib.fen_rcab_c128_tiles(H, W))
    outs = {}
    for mode in (1, 2, 3):
        d = L.RcabC128Desc()
        d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.mode, d.res_scale = ctx.code, B, H, W, C, CR, mode, 0.2
        y = torch.empty_like(xd)
        z1 = torch.empty_like(xd)
        part = torch.empty(B * T, C, device=DEV)
        d.x, d.w, d.bias, d.y = xd.data_ptr(), wp.data_ptr(), bd.data_ptr(), y.data_ptr()
        if mode == 1:
            d.alpha, d.z1 = ad.data_ptr(), z1.data_ptr()
        if mode == 2:
            d.part = part.data_ptr()
        if mode == 3:
            d.res = rd.data_ptr()
        L.check(ctx.lib.fen_rcab_c128(d, torch.cuda.current_stream().cuda_stream), "rcab_c128")
        torch.cuda.synchronize()
        outs[mode] = (y.double().cpu().permute(0, 3, 1, 2), z1.double().cpu().permute(0, 3, 1, 2), part.cpu())
    a = alpha.double()[None, :, None, None]
    tol = 2e-3
    assert _rel(outs[1][1], conv) <= tol
    assert _rel(outs[1][0], conv.clamp(min=0) + a * conv.clamp(max=0)) <= tol
    assert _rel(outs[2][0], conv) <= tol
    tiles = conv.reshape(B, C, H // 4, 4, W // 64, 64).sum(dim=(3, 5)).permute(0, 2, 3, 1).reshape(B * T, C)
    assert _rel(outs[2][2], tiles) <= 1e-4
    assert _rel(outs[3][0], conv + res.double()) <= tol


def test_rcab128_upsample_vs_torch():
    """Mode 4 (an upsampler stage: conv 128 -> 512, PixelShuffle(2), PReLU over the shuffled
    channels; custom.py's stage, blocks.py:211-227) against torch fp32 on the same rounded
    operands (B=2, 64x128, fp16), on the shuffle-permuted mode-1 pack."""
    from src.hip import lib as L
    from src.hip.net import Weights
    from src.hip.program import Ctx
    dtype = torch.float16
    B, H, W = 2, 64, 128
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, C, H, W, generator=g).to(dtype).float()
    w = (torch.randn(4 * C, C, 3, 3, generator=g) * 0.04).to(dtype).float()
    bias = torch.randn(4 * C, generator=g) * 0.1
    alpha = torch.rand(C, generator=g) * 0.5
    ctx = Ctx(dtype, DEV)
    Wt = Weights({"u.weight": w.to(DEV), "u.bias": bias.to(DEV)}, dtype, DEV)
    wp = Wt.packed("u", 1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    y = torch.empty(B, 2 * H, 2 * W, C, device=DEV, dtype=dtype)
    bd, ad = bias.to(DEV), alpha.to(DEV)
    d = L.RcabC128Desc()
    d.dtype, d.B, d.H, d.W, d.C, d.Cr, d.mode, d.res_scale = ctx.code, B, H, W, C, CR, 4, 0.2
    d.x, d.w, d.bias, d.alpha, d.y = xd.data_ptr(), wp.data_ptr(), bd.data_ptr(), ad.data_ptr(), y.data_ptr()
    L.check(ctx.lib.fen_rcab_c128(d, torch.cuda.current_stream().cuda_stream), "rcab_c128 mode 4")
    torch.cuda.synchronize()
    ref = torch.nn.functional.pixel_shuffle(torch.nn.functional.conv2d(x.double(), w.double(), bias.double(),
                                                                       padding=1), 2)
    a = alpha.double()[None, :, None, None]
    ref = ref.clamp(min=0) + a * ref.clamp(max=0)
    assert _rel(y.double().cpu().permute(0, 3, 1, 2), ref) <= 2e-3


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_rcab128_net_vs_oracle(prec):
    """A whole 128-channel net (2 groups x 2 RCAB, x4; seeded reference init) on the graph engine,
    64x64 -> 256x256, against the oracle's forward on the same 16-bit-rounded weights: every
    128-channel conv of the body, conv_after_body and both upsampler stages run on fen_rcab_c128
    (checked in the recorded program); output within the fp16 full-net bound of
    test_gpu_module.py (6e-3 per pixel; bf16 2e-2)."""
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    dtype = DT[prec]
    torch.manual_seed(3)
    m = FaceEnhanceNet(num_channels=C, num_groups=2, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       precision=prec)
    p = {k: v.detach().clone().float() for k, v in m.state_dict().items()}
    x = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(11))
    eng = FENEngine(m, batch=1, lr_hw=(64, 64), dtype=dtype, train=False, device=DEV)
    names = [op[0] for op in eng.ctx.ops]
    assert names.count("rcab_c128_conv1") == 4 and names.count("rcab_c128_conv2") == 4
    assert names.count("rcab_c128_group_conv") == 2 and names.count("c128_upsample") == 2
    assert names.count("c128_after_body") == 1
    out = eng.forward(x.to(DEV)).cpu()
    pr = {k: (v.to(dtype).float() if v.dim() == 4 and k != "conv_first.weight" else v) for k, v in p.items()}
    shape = O.NetShape(num_channels=C, num_groups=2, blocks_per_group=2, reduction_ratio=4, scale_factor=4)
    ref = O.forward(pr, x, shape, training=False)
    err = float((out - ref).abs().max())
    print(f"{prec}: max |out - oracle| {err:.2e}")
    assert err <= (6e-3 if prec == "fp16" else 2e-2), err


def test_rcab128_net_tail_chunks(monkeypatch):
    """The 128-channel engine with its upsampler + conv_last in chunks of 2 images (FEN_TAIL_CHUNK)
    is bit-identical to the one-pass engine at B=4."""
    from src.hip import net
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    torch.manual_seed(3)
    m = FaceEnhanceNet(num_channels=C, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       precision="fp16")
    x = torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(12)).to(DEV)
    outs = {}
    for c in (0, 2):
        monkeypatch.setattr(net, "TAIL_CHUNK", c)
        eng = FENEngine(m, batch=4, lr_hw=(64, 64), dtype=torch.float16, train=False, device=DEV)
        names = [op[0] for op in eng.ctx.ops]
        assert names.count("c128_upsample") == (2 if c == 0 else 4)
        outs[c] = eng.forward(x).cpu()
        del eng
    assert torch.equal(outs[2], outs[0])
