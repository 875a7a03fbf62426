"""GPU parity of the RCAB chain on fen_rcab_deferred (conv1 -> PReLU -> conv2 -> tile sums in one
launch per RCAB; each RCAB's SE gate and scaled residual applied by the next launch, the chain
end by fen_se_fused) against the CPU oracle's RCABs (reference blocks.py:135-153, chained as in
ResidualGroup blocks.py:185-188) and against the per-op HIP launches.

Tolerances: the kernels round x, the filters, a1 and t to the 16-bit format, so they are compared
to an fp32 oracle fed the same rounded x / weights, at rel-L2 <= 5e-3 per RCAB of chain length
for bf16 (1e-3 for fp16) on y -- a wrong tap, tile, halo, edge column or gate shows up as O(1) --
and the gates s at |d| <= 2e-3.  Shapes: one tile per block (32x32), 17 x 64x64 (544 tiles, two
or three per block), odd tile counts (48x80), a single tile (16x16), the bench shape (32 x 64x64)."""
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"bf16": torch.bfloat16, "fp16": torch.float16}


def _params(n, C=64, Cr=16, seed=3):
    g = torch.Generator().manual_seed(seed)
    p = {}
    for j in range(n):
        q = f"b{j}."
        p[q + "conv1.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
        p[q + "conv1.bias"] = torch.randn(C, generator=g) * 0.1
        p[q + "prelu.weight"] = torch.rand(C, generator=g) * 0.5
        p[q + "conv2.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
        p[q + "conv2.bias"] = torch.randn(C, generator=g) * 0.1
        p[q + "channel_attention.fc.0.weight"] = torch.randn(Cr, C, generator=g) * 0.3
        p[q + "channel_attention.fc.2.weight"] = torch.randn(C, Cr, generator=g) * 0.3
    return p


def _run(p, n, x_nhwc, train, mode, dtype, record=False):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.RCAB_MODE
    net.RCAB_MODE = mode
    try:
        ctx = Ctx(dtype, DEV, record=record)
        pd = {k: v.to(DEV) for k, v in p.items()}
        Wt = Weights(pd, dtype, DEV)
        attn = {}
        ctx.keep(Wt)   # a recorded program's launches reference the packed weights by address
        fw = Forward(NetSpec(C=64, G=1, NB=n, Cr=16), ctx, Wt, save=train, attn=attn)
        names = [f"r{j}" for j in range(n)]
        if mode == "deferred":
            y, svs = fw._chain(x_nhwc, [f"b{j}." for j in range(n)], names)
        else:
            y, svs = x_nhwc, []
            for j in range(n):
                y, sv = fw.rcab(y, f"b{j}.", name=names[j])
                svs.append(sv)
        if not record:
            torch.cuda.synchronize()
    finally:
        net.RCAB_MODE = old
    return y, svs, attn, ctx


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def _oracle(p, n, x, dtype):
    pr = {k: (v.to(dtype).float() if v.dim() == 4 else v) for k, v in p.items()}
    h, ss = x, []
    for j in range(n):
        q = f"b{j}."
        t = O.conv3x3(O.prelu(O.conv3x3(h, pr[q + "conv1.weight"], pr[q + "conv1.bias"]), pr[q + "prelu.weight"]),
                      pr[q + "conv2.weight"], pr[q + "conv2.bias"])
        ss.append(O.channel_attention(t, pr, q + "channel_attention."))
        h = O.rcab(h, pr, q, 0.2)
    return h, ss


@pytest.mark.parametrize("B,H,W", [(3, 32, 32), (17, 64, 64), (2, 48, 80), (1, 16, 16), (32, 64, 64)])
@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_rcab_chain(B, H, W, train, prec):
    from src.hip import lib as L
    dtype = DT[prec]
    code = L.dtype_code(dtype)
    if not L.load().fen_rcab_deferred_supported(code, B, H, W, 64, 16):
        pytest.skip("shape outside the deferred kernel's envelope")
    n = 3
    torch.manual_seed(11)
    p = _params(n)
    x = torch.randn(B, 64, H, W).to(dtype).float()
    ref, s_ref = _oracle(p, n, x, dtype)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    y, svs, attn, _ = _run(p, n, xd, train, "deferred", dtype)
    out = y.float().cpu().permute(0, 3, 1, 2)
    tol = (5e-3 if prec == "bf16" else 1e-3) * n
    assert _rel(out, ref) <= tol
    for j in range(n):
        assert float((attn[f"r{j}"].cpu() - s_ref[j]).abs().max()) <= 2e-3, j
    # the same chain again: every launch is independent of the previous launch's leftovers
    y2, _, _, _ = _run(p, n, xd, train, "deferred", dtype)
    assert torch.equal(y2, y)
    if train:
        # the saved tensors the backward reads equal the per-op launches' (bf16: same operands)
        yu, svu, _, _ = _run(p, n, xd, True, "perop", dtype)
        for j in range(n):
            for k in ("x", "z1", "a1", "t"):
                assert _rel(svs[j][k].float(), svu[j][k].float()) <= 5e-3, (j, k)
            for k in ("mean", "hid", "s"):
                assert float((svs[j][k] - svu[j][k]).abs().max()) <= 2e-3, (j, k)


def test_rcab_chain_graph_replay():
    """A 10-RCAB chain recorded into a program and replayed from a hipGraph three times must
    reproduce the eager result bit for bit, and match the per-op launches."""
    from src.hip import lib as L
    B, H, W = 4, 32, 32
    if not L.load().fen_rcab_deferred_supported(L.BF16, B, H, W, 64, 16):
        pytest.skip("shape outside the deferred kernel's envelope")
    torch.manual_seed(5)
    n = 10
    p = _params(n, seed=8)
    x = torch.randn(B, H, W, 64, device=DEV).to(torch.bfloat16)
    h, _, _, ctx = _run(p, n, x, False, "deferred", torch.bfloat16, record=True)
    assert sum(op[0] == "rcab_deferred" for op in ctx.ops) == n
    ctx.run()
    torch.cuda.synchronize()
    ref = h.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ctx.run()
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(h, ref)
    h2, _, _, _ = _run(p, n, x, False, "perop", torch.bfloat16)
    assert _rel(ref.float(), h2.float()) <= 1e-2


def _round(x, dtype):
    return x.to(dtype).float()


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("B,H,W,dot", [(2, 32, 32, True), (17, 64, 64, True), (1, 48, 80, False), (1, 16, 16, True),
                                        (32, 64, 64, True), (3, 32, 48, "res"), (32, 64, 64, "res")])
def test_rcab_bwd_fused(prec, B, H, W, dot):
    """fen_rcab_bwd (the RCAB backward's conv2^T -> PReLU' -> conv1^T + dy in one launch, + the
    next RCAB's DOT partials) vs a torch fp32 restatement on the same rounded operands:
    g2 = conv2^T(dt), dz1 = g2 * PReLU'(z1), dalpha per tile = sum g2 * z1 * (z1 <= 0),
    dx = conv1^T(dz1 as stored) + dy, DOT per tile = sum dx (as stored) * t_next; dot = "res":
    a second residual (dres, a group's first RCAB) added to dx instead of the DOT.
    rel-L2 <= 3e-3 (bf16) / 1e-3 (fp16) on dz1 and dx; 5e-3 / 2e-3 on the partial sums (a
    wrong tap, halo row, edge fragment or tile shows up as O(1))."""
    import torch.nn.functional as F
    from src.hip import lib as L
    from src.hip.net import Weights, tiles
    from src.hip.program import Ctx, ptr
    dtype = DT[prec]
    g = torch.Generator().manual_seed(9)
    C = 64
    w1 = torch.randn(C, C, 3, 3, generator=g) * 0.06
    w2 = torch.randn(C, C, 3, 3, generator=g) * 0.06
    alpha = torch.rand(C, generator=g) * 0.5
    dt = _round(torch.randn(B, C, H, W, generator=g), dtype)
    z1 = _round(torch.randn(B, C, H, W, generator=g), dtype)
    dy = _round(torch.randn(B, C, H, W, generator=g), dtype)
    tn = _round(torch.randn(B, C, H, W, generator=g), dtype)
    w1r, w2r = _round(w1, dtype), _round(w2, dtype)
    # reference
    g2 = F.conv_transpose2d(dt, w2r, padding=1)
    a = alpha.view(1, C, 1, 1)
    dz1_ref = g2 * torch.where(z1 > 0, torch.ones_like(z1), a.expand_as(z1))
    dal_ref = (g2 * z1 * (z1 <= 0)).view(B, C, H // 16, 16, W // 16, 16).sum((3, 5))
    dal_ref = dal_ref.permute(0, 2, 3, 1).reshape(B * tiles(H, W), C)
    dx_ref = F.conv_transpose2d(_round(dz1_ref, dtype), w1r, padding=1) + dy
    if dot == "res":                                   # a group's first RCAB: + the group's dy
        dx_ref = dx_ref + tn
    dot_ref = (_round(dx_ref, dtype) * tn).view(B, C, H // 16, 16, W // 16, 16).sum((3, 5))
    dot_ref = dot_ref.permute(0, 2, 3, 1).reshape(B * tiles(H, W), C)

    nh = lambda t: t.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    ctx = Ctx(dtype, DEV)
    Wt = Weights({"c1.weight": w1.to(DEV), "c2.weight": w2.to(DEV)}, dtype, DEV)
    T = tiles(H, W)
    dtd, z1d, dyd, tnd = nh(dt), nh(z1), nh(dy), nh(tn)
    dz1 = ctx.alloc((B, H, W, C))
    dx = ctx.alloc((B, H, W, C))
    dal = ctx.alloc((B * T, C), torch.float32)
    dotp = ctx.alloc((B * T, C), torch.float32)
    ad = alpha.to(DEV)
    d = L.RcabBwdDesc()
    d.dtype, d.B, d.H, d.W, d.C = ctx.code, B, H, W, C
    d.dt, d.w2t, d.z1, d.alpha = ptr(dtd), ptr(Wt.packed("c2", 2)), ptr(z1d), ptr(ad)
    d.w1t, d.dy, d.dz1, d.dalpha_part, d.dx = ptr(Wt.packed("c1", 2)), ptr(dyd), ptr(dz1), ptr(dal), ptr(dx)
    if dot == "res":
        d.dres = ptr(tnd)
    elif dot:
        d.dot_t, d.dot_part = ptr(tnd), ptr(dotp)
    L.check(ctx.lib.fen_rcab_bwd(d, torch.cuda.current_stream().cuda_stream), "rcab_bwd")
    torch.cuda.synchronize()
    tol, tolp = (3e-3, 5e-3) if prec == "bf16" else (1e-3, 2e-3)
    rel = lambda a_, b_: float((a_ - b_).norm() / b_.norm())
    nc = lambda t: t.float().cpu().permute(0, 3, 1, 2)
    assert rel(nc(dz1), dz1_ref) <= tol
    assert rel(nc(dx), dx_ref) <= tol
    assert rel(dal.cpu(), dal_ref) <= tolp
    if dot is True:
        assert rel(dotp.cpu(), dot_ref) <= tolp


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("B,H,W", [(2, 32, 48), (3, 64, 64), (32, 64, 64), (40, 64, 64)])
def test_rcab_bwd_se_fold(prec, B, H, W):
    """fen_rcab_bwd with the SE backward folded in (se_part set: dt built on each tile's dy halo)
    against fen_se_bwd_fused followed by the plain fen_rcab_bwd on the same inputs: dt, the FC
    weight-gradient rows, dz1, dx, the slope and DOT partials all bit-identical (same arithmetic
    in the same order).  B = 40 puts 3 tiles on a block (the in-loop fold of tiles 2 and 3)."""
    from src.hip import lib as L
    from src.hip.net import Weights, tiles
    from src.hip.program import Ctx, ptr
    dtype = DT[prec]
    g = torch.Generator().manual_seed(11)
    C, Cr = 64, 16
    T = tiles(H, W)
    ctx = Ctx(dtype, DEV)
    if not ctx.lib.fen_rcab_bwd_se_supported(ctx.code, B, H, W, C, Cr):
        pytest.skip("outside the folded envelope on this device")
    w1 = torch.randn(C, C, 3, 3, generator=g) * 0.06
    w2 = torch.randn(C, C, 3, 3, generator=g) * 0.06
    Wt = Weights({"c1.weight": w1.to(DEV), "c2.weight": w2.to(DEV)}, dtype, DEV)
    nh = lambda t: t.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    z1, dy, tn = (nh(torch.randn(B, C, H, W, generator=g)) for _ in range(3))
    alpha = (torch.rand(C, generator=g) * 0.5).to(DEV)
    part = (torch.randn(B * T, C, generator=g) * 3).to(DEV)
    sg = torch.sigmoid(torch.randn(B, C, generator=g)).to(DEV)
    mean = torch.randn(B, C, generator=g).to(DEV)
    hid = torch.randn(B, Cr, generator=g).clamp_min(0).to(DEV)      # some units exactly 0
    fc1 = (torch.randn(Cr, C, generator=g) * 0.2).to(DEV)
    fc2 = (torch.randn(C, Cr, generator=g) * 0.2).to(DEV)
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for fold in (False, True):
        dt = ctx.alloc((B, H, W, C))
        dw1p = ctx.alloc((B, Cr * C), torch.float32)
        dw2p = ctx.alloc((B, Cr * C), torch.float32)
        dz1, dx = ctx.alloc((B, H, W, C)), ctx.alloc((B, H, W, C))
        dal, dotp = ctx.alloc((B * T, C), torch.float32), ctx.alloc((B * T, C), torch.float32)
        if not fold:
            L.check(ctx.lib.fen_se_bwd_fused(ctx.code, B, H * W, C, Cr, T, 1.0 / (H * W), 0.2, ptr(part), ptr(mean),
                                             ptr(hid), ptr(sg), ptr(fc1), ptr(fc2), ptr(dy), None, ptr(dw1p),
                                             ptr(dw2p), ptr(dt), stream), "se_bwd_fused")
        d = L.RcabBwdDesc()
        d.dtype, d.B, d.H, d.W, d.C = ctx.code, B, H, W, C
        d.dt, d.w2t, d.z1, d.alpha = ptr(dt), ptr(Wt.packed("c2", 2)), ptr(z1), ptr(alpha)
        d.w1t, d.dy, d.dz1, d.dalpha_part, d.dx = ptr(Wt.packed("c1", 2)), ptr(dy), ptr(dz1), ptr(dal), ptr(dx)
        d.dot_t, d.dot_part = ptr(tn), ptr(dotp)
        if fold:
            d.se_part, d.se_s, d.se_mean, d.se_hid = ptr(part), ptr(sg), ptr(mean), ptr(hid)
            d.se_w1, d.se_w2, d.se_dw1p, d.se_dw2p = ptr(fc1), ptr(fc2), ptr(dw1p), ptr(dw2p)
            d.se_res_scale, d.se_Cr = 0.2, Cr
        L.check(ctx.lib.fen_rcab_bwd(d, stream), "rcab_bwd")
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (dt, dw1p, dw2p, dz1, dx, dal, dotp)])
    for name, a_, b_ in zip(("dt", "dw1p", "dw2p", "dz1", "dx", "dalpha", "dot"), outs[0], outs[1]):
        assert torch.equal(a_, b_), name


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("B,H,W,train", [(2, 32, 32, False), (17, 64, 64, True), (1, 48, 80, False),
                                          (32, 64, 64, False), (3, 16, 16, True)])
def test_group_end_fused(prec, B, H, W, train):
    """fen_rcab_group_end (the last RCAB's gate + residual applied while building the input,
    then the group conv + bias + the group's residual, one launch) vs the split chain end
    (fen_se_fused, then fen_conv3x3 with the residual epilogue) in Forward.group: the group
    output at rel-L2 <= 2e-3 (bf16) / 5e-4 (fp16) -- both round y to the 16-bit format before
    the conv; the gate product's fp32 order and the accumulation order differ -- and, in
    training, the saved chain output (the group conv's weight-gradient operand, same bound)
    and the last RCAB's gate s (|d| <= 1e-5)."""
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    dtype = DT[prec]
    n = 3
    p = _params(n)
    g = torch.Generator().manual_seed(21)
    q = {}
    for k, v in p.items():
        q["rg." + k.replace("b", "blocks.", 1)] = v
    q["rg.conv.weight"] = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    q["rg.conv.bias"] = torch.randn(64, generator=g) * 0.1
    x = torch.randn(B, H, W, 64, generator=g).to(DEV, dtype)
    outs = {}
    for fused in (True, False):
        old = net.GROUP_END_FUSED
        net.GROUP_END_FUSED = fused
        try:
            ctx = Ctx(dtype, DEV)
            pd = {k: v.to(DEV) for k, v in q.items()}
            Wt = Weights(pd, dtype, DEV)
            fw = Forward(NetSpec(C=64, G=1, NB=n, Cr=16), ctx, Wt, save=train)
            y, sv = fw.group(x, 0, pre="rg.")
            torch.cuda.synchronize()
            outs[fused] = (y.float().cpu(), sv)
        finally:
            net.GROUP_END_FUSED = old
    tol = 2e-3 if prec == "bf16" else 5e-4
    rel = lambda a_, b_: float((a_ - b_).norm() / b_.norm())
    assert rel(outs[True][0], outs[False][0]) <= tol
    if train:
        a, b_ = outs[True][1], outs[False][1]
        assert rel(a["x_last"].float().cpu(), b_["x_last"].float().cpu()) <= tol
        assert float((a["blocks"][-1]["s"] - b_["blocks"][-1]["s"]).abs().max()) <= 1e-5


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("B,H,W", [(3, 64, 64), (32, 64, 64), (40, 64, 64)])
def test_rcab_bwd_se_fold_vs_oracle(prec, B, H, W):
    """The SE-folded fen_rcab_bwd against a torch fp32 restatement of the reference's autograd
    (blocks.py:83-92,135-153), not another HIP path.  SE backward: ds = sum_hw dy*t (the DOT
    partials), dz = ds*rs*s*(1-s), dh = W2^T dz masked by hid > 0, dt = dy*rs*s + (W1^T dh)/HW;
    FC weight-gradient rows dz x hid, dh x mean; then conv2^T -> PReLU' -> conv1^T + dy as in
    test_rcab_bwd_fused, each on the operands as the kernel stores them.  B = 32 / 40: 2 / 3
    tiles per block at the bench's image size.  rel-L2 bounds as test_rcab_bwd_fused; the FC
    rows 1e-4 (fp32 arithmetic on fp32 operands)."""
    import torch.nn.functional as F
    from src.hip import lib as L
    from src.hip.net import Weights, tiles
    from src.hip.program import Ctx, ptr
    dtype = DT[prec]
    g = torch.Generator().manual_seed(13)
    C, Cr, rs = 64, 16, 0.2
    T = tiles(H, W)
    ctx = Ctx(dtype, DEV)
    if not ctx.lib.fen_rcab_bwd_se_supported(ctx.code, B, H, W, C, Cr):
        pytest.skip("outside the folded envelope on this device")
    w1 = torch.randn(C, C, 3, 3, generator=g) * 0.06
    w2 = torch.randn(C, C, 3, 3, generator=g) * 0.06
    z1, dy, tn = (_round(torch.randn(B, C, H, W, generator=g), dtype) for _ in range(3))
    alpha = torch.rand(C, generator=g) * 0.5
    part = torch.randn(B * T, C, generator=g) * 3
    sg = torch.sigmoid(torch.randn(B, C, generator=g))
    mean = torch.randn(B, C, generator=g)
    hid = torch.randn(B, Cr, generator=g).clamp_min(0)
    fc1 = torch.randn(Cr, C, generator=g) * 0.2
    fc2 = torch.randn(C, Cr, generator=g) * 0.2
    # reference (fp32)
    ds = part.view(B, T, C).sum(1)
    dz = ds * rs * sg * (1 - sg)
    dh = (dz @ fc2) * (hid > 0)
    ga = (dh @ fc1) / (H * W)
    dt_ref = dy * rs * sg[:, :, None, None] + ga[:, :, None, None]
    dw2_ref = dz[:, :, None] * hid[:, None, :]              # [B][C][Cr]
    dw1_ref = dh[:, :, None] * mean[:, None, :]             # [B][Cr][C]
    w1r, w2r = _round(w1, dtype), _round(w2, dtype)
    g2 = F.conv_transpose2d(_round(dt_ref, dtype), w2r, padding=1)
    dz1_ref = g2 * torch.where(z1 > 0, torch.ones_like(z1), alpha.view(1, C, 1, 1).expand_as(z1))
    dal_ref = (g2 * z1 * (z1 <= 0)).view(B, C, H // 16, 16, W // 16, 16).sum((3, 5))
    dal_ref = dal_ref.permute(0, 2, 3, 1).reshape(B * T, C)
    dx_ref = F.conv_transpose2d(_round(dz1_ref, dtype), w1r, padding=1) + dy
    dot_ref = (_round(dx_ref, dtype) * tn).view(B, C, H // 16, 16, W // 16, 16).sum((3, 5))
    dot_ref = dot_ref.permute(0, 2, 3, 1).reshape(B * T, C)
    # HIP (folded)
    nh = lambda t: t.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    Wt = Weights({"c1.weight": w1.to(DEV), "c2.weight": w2.to(DEV)}, dtype, DEV)
    dt = ctx.alloc((B, H, W, C))
    dw1p, dw2p = ctx.alloc((B, Cr * C), torch.float32), ctx.alloc((B, Cr * C), torch.float32)
    dz1, dx = ctx.alloc((B, H, W, C)), ctx.alloc((B, H, W, C))
    dal, dotp = ctx.alloc((B * T, C), torch.float32), ctx.alloc((B * T, C), torch.float32)
    dev = lambda t: t.contiguous().to(DEV)
    z1d, dyd, tnd = nh(z1), nh(dy), nh(tn)
    partd, sgd, meand, hidd, fc1d, fc2d, ad = map(dev, (part, sg, mean, hid, fc1, fc2, alpha))
    d = L.RcabBwdDesc()
    d.dtype, d.B, d.H, d.W, d.C = ctx.code, B, H, W, C
    d.dt, d.w2t, d.z1, d.alpha = ptr(dt), ptr(Wt.packed("c2", 2)), ptr(z1d), ptr(ad)
    d.w1t, d.dy, d.dz1, d.dalpha_part, d.dx = ptr(Wt.packed("c1", 2)), ptr(dyd), ptr(dz1), ptr(dal), ptr(dx)
    d.dot_t, d.dot_part = ptr(tnd), ptr(dotp)
    d.se_part, d.se_s, d.se_mean, d.se_hid = ptr(partd), ptr(sgd), ptr(meand), ptr(hidd)
    d.se_w1, d.se_w2, d.se_dw1p, d.se_dw2p = ptr(fc1d), ptr(fc2d), ptr(dw1p), ptr(dw2p)
    d.se_res_scale, d.se_Cr = rs, Cr
    L.check(ctx.lib.fen_rcab_bwd(d, torch.cuda.current_stream().cuda_stream), "rcab_bwd")
    torch.cuda.synchronize()
    tol, tolp = (3e-3, 5e-3) if prec == "bf16" else (1e-3, 2e-3)
    rel = lambda a_, b_: float((a_.double() - b_.double()).norm() / b_.double().norm())
    nc = lambda t: t.float().cpu().permute(0, 3, 1, 2)
    assert rel(nc(dt), dt_ref) <= tol      # one 16-bit rounding of dt (bf16: ~1.7e-3 rel-L2)
    # the FC weight-gradient rows: the per-image rows for every image (summed by the caller)
    assert rel(dw2p.cpu().view(B, C, Cr), dw2_ref) <= 1e-4
    assert rel(dw1p.cpu().view(B, Cr, C), dw1_ref) <= 1e-4
    assert rel(nc(dz1), dz1_ref) <= tol
    assert rel(nc(dx), dx_ref) <= tol
    assert rel(dal.cpu(), dal_ref) <= tolp
    assert rel(dotp.cpu(), dot_ref) <= tolp


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("B,H,W", [(3, 32, 32), (32, 64, 64), (40, 64, 64)])
def test_group_end_vs_oracle(prec, B, H, W):
    """A ResidualGroup on the production path (deferred RCAB chain + fen_rcab_group_end) against
    the oracle's residual_group (blocks.py:185-189) on the same rounded weights and input, not
    another HIP path: group output rel-L2 <= 5e-3 (bf16) / 1e-3 (fp16) per RCAB + 1 (as
    test_rcab_chain), and every gate within 2e-3."""
    from src.hip import lib as L
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    dtype = DT[prec]
    if not L.load().fen_rcab_deferred_supported(L.dtype_code(dtype), B, H, W, 64, 16):
        pytest.skip("shape outside the deferred kernel's envelope")
    n = 3
    p = _params(n, seed=17)
    g = torch.Generator().manual_seed(23)
    q = {"rg." + k.replace("b", "blocks.", 1): v for k, v in p.items()}
    q["rg.conv.weight"] = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    q["rg.conv.bias"] = torch.randn(64, generator=g) * 0.1
    x = torch.randn(B, 64, H, W, generator=g).to(dtype).float()
    qr = {k: (v.to(dtype).float() if v.dim() == 4 else v) for k, v in q.items()}
    attn_ref = {}
    ref = O.residual_group(x, qr, "rg.", n, 0.2, attn=attn_ref)
    old = net.GROUP_END_FUSED
    net.GROUP_END_FUSED = True
    try:
        ctx = Ctx(dtype, DEV)
        pd = {k: v.to(DEV) for k, v in q.items()}
        Wt = Weights(pd, dtype, DEV)
        attn = {}
        fw = Forward(NetSpec(C=64, G=1, NB=n, Cr=16), ctx, Wt, save=False, attn=attn)
        y, _ = fw.group(x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype), 0, pre="rg.")
        torch.cuda.synchronize()
    finally:
        net.GROUP_END_FUSED = old
    out = y.float().cpu().permute(0, 3, 1, 2)
    tol = (5e-3 if prec == "bf16" else 1e-3) * (n + 1)
    assert _rel(out, ref) <= tol
    assert len(attn) == n
    for (k, s), (kr, sr) in zip(sorted(attn.items()), sorted(attn_ref.items())):
        assert float((s.cpu() - sr).abs().max()) <= 2e-3, (k, kr)
