"""GPU parity of the fused RCAB forward (fen_rcab_fused: conv1 -> PReLU -> conv2 -> SE gate
-> scaled residual in one launch) against the CPU oracle's RCAB (reference blocks.py:135-153)
and against the per-op HIP path on the same bf16 operands.

Tolerances: the fused kernel rounds x, the filters and a1 to bf16 (like the per-op path) but
keeps t in fp32 up to the residual add, so it is compared to an fp32 oracle fed the same
bf16-rounded x/weights at rel-L2 <= 5e-3 on y (a wrong tap, tile, halo or gate shows up as
O(1)), and the gate s at |d| <= 2e-3.  Shapes: one tile per block (32x32), two rounds of
whole images (17 x 64x64 on 256 CUs), odd tile counts (48x80), a single tile (16x16)."""
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(C=64, Cr=16, seed=3):
    g = torch.Generator().manual_seed(seed)
    p = {
        "conv1.weight": torch.randn(C, C, 3, 3, generator=g) * 0.06,
        "conv1.bias": torch.randn(C, generator=g) * 0.1,
        "prelu.weight": torch.rand(C, generator=g) * 0.5,
        "conv2.weight": torch.randn(C, C, 3, 3, generator=g) * 0.06,
        "conv2.bias": torch.randn(C, generator=g) * 0.1,
        "channel_attention.fc.0.weight": torch.randn(Cr, C, generator=g) * 0.3,
        "channel_attention.fc.2.weight": torch.randn(C, Cr, generator=g) * 0.3,
    }
    return p


def _run(p, x_nhwc, train, fused, twice=False):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.FUSED_RCAB
    net.FUSED_RCAB = fused
    try:
        ctx = Ctx(torch.bfloat16, DEV)
        pd = {k: v.to(DEV) for k, v in p.items()}
        Wt = Weights(pd, torch.bfloat16, DEV)
        fw = Forward(NetSpec(C=64, G=1, NB=1, Cr=16), ctx, Wt, save=train)
        y, sv = fw.rcab(x_nhwc, "")
        if twice:   # same sync words: the first launch must have left them clean
            y2, _ = fw.rcab(x_nhwc, "")
            sv = dict(sv, y2=y2)
        torch.cuda.synchronize()
    finally:
        net.FUSED_RCAB = old
    return y, sv, ctx


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("B,H,W", [(3, 32, 32), (17, 64, 64), (2, 48, 80), (1, 16, 16)])
@pytest.mark.parametrize("train", [False, True])
def test_fused_rcab(B, H, W, train):
    from src.hip import lib as L
    if not L.load().fen_rcab_supported(L.BF16, B, H, W, 64, 16):
        pytest.skip("shape outside the fused kernel's envelope")
    torch.manual_seed(11)
    p = _params()
    x = torch.randn(B, 64, H, W).to(torch.bfloat16).float()
    pr = {k: (v.to(torch.bfloat16).float() if v.dim() == 4 else v) for k, v in p.items()}
    ref = O.rcab(x, pr, "", 0.2)
    s_ref = O.channel_attention(O.conv3x3(O.prelu(O.conv3x3(x, pr["conv1.weight"], pr["conv1.bias"]),
                                                  pr["prelu.weight"]), pr["conv2.weight"], pr["conv2.bias"]), pr,
                                "channel_attention.")
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, torch.bfloat16)
    y, sv, ctx = _run(p, xd, train, True, twice=True)
    out = y.float().cpu().permute(0, 3, 1, 2)
    assert _rel(out, ref) <= 5e-3
    assert float((sv["s"].cpu() - s_ref).abs().max()) <= 2e-3
    lib = L.load()
    assert lib.fen_rcab_workspace_status(ctx._shared["rcab_ws"].ptr, B, H, W) == 0, \
        "sync words must be left zeroed (self-cleaning, no poll timeout)"
    if train:
        yu, svu, _ = _run(p, xd, True, False)
        for k in ("z1", "a1", "t"):
            assert _rel(sv[k].float(), svu[k].float()) <= 5e-3, k
        for k in ("mean", "hid"):
            assert float((sv[k] - svu[k]).abs().max()) <= 2e-3, k
    assert _rel(sv["y2"].float(), y.float()) <= 1e-6


def test_fused_rcab_graph_replay():
    """Ten chained fused RCABs recorded into a program and replayed from a hipGraph three
    times: the self-cleaning gate counters must let back-to-back launches run, and every
    replay must reproduce the eager result bit for bit."""
    from src.hip import lib as L, net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    B, H, W = 4, 32, 32
    if not L.load().fen_rcab_supported(L.BF16, B, H, W, 64, 16):
        pytest.skip("shape outside the fused kernel's envelope")
    torch.manual_seed(5)
    p = {k: v.to(DEV) for k, v in _params().items()}
    x = torch.randn(B, H, W, 64, device=DEV).to(torch.bfloat16)
    ctx = Ctx(torch.bfloat16, DEV, record=True)
    fw = Forward(NetSpec(C=64, G=1, NB=1, Cr=16), ctx, Weights(p, torch.bfloat16, DEV), save=False)
    h = x
    old = net.FUSED_RCAB
    net.FUSED_RCAB = True
    try:
        for i in range(10):
            h, _ = fw.rcab(h, "", out=ctx.scratch(f"pp{i & 1}", x.shape))
    finally:
        net.FUSED_RCAB = old
    assert sum(op[0] == "rcab_fused" for op in ctx.ops) == 10
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
    # the chain matches the per-op launches (a stale gate read by a later launch would not)
    old = net.FUSED_RCAB
    net.FUSED_RCAB = False
    try:
        ctx2 = Ctx(torch.bfloat16, DEV)
        fw2 = Forward(NetSpec(C=64, G=1, NB=1, Cr=16), ctx2, Weights(p, torch.bfloat16, DEV), save=False)
        h2 = x
        for i in range(10):
            h2, _ = fw2.rcab(h2, "")
        torch.cuda.synchronize()
    finally:
        net.FUSED_RCAB = old
    assert _rel(ref.float(), h2.float()) <= 1e-2
    assert L.load().fen_rcab_workspace_status(ctx._shared["rcab_ws"].ptr, B, H, W) == 0
