"""GPU parity of fen_group_strip -- a whole ResidualGroup (reference blocks.py:161-189: RCABs
blocks.py:135-153 with ChannelAttention blocks.py:83-92, then conv + the group's skip) as ONE
persistent strip-resident launch -- against the CPU oracle's residual_group on the same
16-bit-rounded weights and input, and against the per-RCAB launches (fen_rcab_deferred +
fen_rcab_group_end).

Tolerances as test_gpu_rcab.py's chain tests: the kernels round x_j, a1 and t to the 16-bit
format, so the group output is compared at rel-L2 <= 5e-3 (bf16) / 1e-3 (fp16) per RCAB + 1,
every gate s within 2e-3.  A wrong halo row, strip hand-off, tap or gate shows up as O(1).
Shapes: the bench's (B=32, 64x64, 10 RCABs: 256 strips = one per CU), one strip per image
(H=8), two / three strips (H=16, 24), 16 strips (H=128), more strips than CUs (B=40, 320
blocks: later tickets wait for a CU), single image.  Every launch leaves its counters at zero and
its error word clear; graph replays are bit-identical."""
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"bf16": torch.bfloat16, "fp16": torch.float16}


def _params(n, seed):
    g = torch.Generator().manual_seed(seed)
    C, Cr = 64, 16
    q = {}
    for j in range(n):
        b = f"rg.blocks.{j}."
        q[b + "conv1.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
        q[b + "conv1.bias"] = torch.randn(C, generator=g) * 0.1
        q[b + "prelu.weight"] = torch.rand(C, generator=g) * 0.5
        q[b + "conv2.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
        q[b + "conv2.bias"] = torch.randn(C, generator=g) * 0.1
        q[b + "channel_attention.fc.0.weight"] = torch.randn(Cr, C, generator=g) * 0.3
        q[b + "channel_attention.fc.2.weight"] = torch.randn(C, Cr, generator=g) * 0.3
    q["rg.conv.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.05
    q["rg.conv.bias"] = torch.randn(C, generator=g) * 0.1
    return q


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def _run(q, n, x_nhwc, dtype, strip=True, record=False, ctx=None):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.GROUP_STRIP
    net.GROUP_STRIP = strip
    try:
        ctx = ctx or Ctx(dtype, DEV, record=record)
        pd = {k: v.to(DEV) for k, v in q.items()}
        Wt = Weights(pd, dtype, DEV)
        ctx.keep(Wt)
        attn = {}
        fw = Forward(NetSpec(C=64, G=1, NB=n, Cr=16), ctx, Wt, save=False, attn=attn)
        used = fw._strip_ok(x_nhwc)
        y, _ = fw.group(x_nhwc, 0, pre="rg.")
        if not record:
            torch.cuda.synchronize()
    finally:
        net.GROUP_STRIP = old
    return y, attn, ctx, used


def _work_error(ctx):
    from src.hip import lib as L
    L.check_strip_status()          # a timed-out wait is reported there (and cleared from `work`)
    bufs = [v for k, v in ctx._shared.items() if k.startswith("pz:group_strip")]
    assert bufs
    ints = [b[:256].view(torch.int32).cpu() for b in bufs]
    return [(int(t[0]), int(t[1]), int(t[2])) for t in ints]   # ticket, done, error


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
@pytest.mark.parametrize("B,H,n", [(32, 64, 10), (2, 64, 3), (3, 8, 2), (4, 16, 3), (2, 24, 2), (2, 128, 2),
                                   (40, 64, 2), (1, 64, 1)])
def test_group_strip_vs_oracle(prec, B, H, n):
    dtype = DT[prec]
    q = _params(n, seed=31 + n)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, 64, H, 64, generator=g).to(dtype).float()
    qr = {k: (v.to(dtype).float() if v.dim() == 4 else v) for k, v in q.items()}
    attn_ref = {}
    ref = O.residual_group(x, qr, "rg.", n, 0.2, attn=attn_ref)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    y, attn, ctx, used = _run(q, n, xd, dtype)
    assert used, "outside fen_group_strip's envelope"
    assert _work_error(ctx) == [(0, 0, 0)]
    out = y.float().cpu().permute(0, 3, 1, 2)
    tol = (5e-3 if prec == "bf16" else 1e-3) * (n + 1)
    r = _rel(out, ref)
    print(f"{prec} B={B} H={H} n={n}: rel {r:.2e}")
    assert r <= tol, r
    assert sorted(attn) == sorted(attn_ref)
    for k in attn:
        assert float((attn[k].cpu() - attn_ref[k]).abs().max()) <= 2e-3, k
    # again: deterministic (fixed-order partial sums), counters reset by the first launch
    y2, _, ctx2, _ = _run(q, n, xd, dtype, ctx=ctx)
    assert torch.equal(y2, y)
    assert _work_error(ctx2) == [(0, 0, 0)]


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_group_strip_vs_deferred_chain(prec):
    """The strip kernel and the per-RCAB launches agree at the bench shape (both round the same
    tensors; summation orders differ): rel-L2 <= 2e-3 (bf16) / 5e-4 (fp16) per RCAB."""
    dtype = DT[prec]
    n = 10
    q = _params(n, seed=5)
    x = torch.randn(32, 64, 64, 64, generator=torch.Generator().manual_seed(9)).to(DEV, dtype)
    ys, attn_s, _, used = _run(q, n, x, dtype, strip=True)
    yd, attn_d, _, used_d = _run(q, n, x, dtype, strip=False)
    assert used and not used_d
    tol = (2e-3 if prec == "bf16" else 5e-4) * n
    assert _rel(ys.float(), yd.float()) <= tol
    for k in attn_s:
        assert float((attn_s[k] - attn_d[k]).abs().max()) <= 2e-3, k


def test_group_strip_graph_replay():
    """Recorded and replayed from a hipGraph five times: bit-identical to the eager launch, the
    counters back at zero after every replay (the last block resets them)."""
    dtype = torch.float16
    n = 10
    q = _params(n, seed=12)
    x = torch.randn(32, 64, 64, 64, generator=torch.Generator().manual_seed(3)).to(DEV, dtype)
    y_e, _, _, _ = _run(q, n, x, dtype)
    y, _, ctx, _ = _run(q, n, x, dtype, record=True)
    assert [op[0] for op in ctx.ops] == ["group_strip"]
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
        assert _work_error(ctx) == [(0, 0, 0)]


def _run_save(q, n, x_nhwc, dtype, strip):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.GROUP_STRIP, net.GROUP_STRIP_TRAIN
    net.GROUP_STRIP = net.GROUP_STRIP_TRAIN = strip
    try:
        ctx = Ctx(dtype, DEV)
        Wt = Weights({k: v.to(DEV) for k, v in q.items()}, dtype, DEV)
        fw = Forward(NetSpec(C=64, G=1, NB=n, Cr=16), ctx, Wt, save=True)
        used = fw._strip_ok(x_nhwc)
        y, sv = fw.group(x_nhwc, 0, pre="rg.")
        torch.cuda.synchronize()
    finally:
        net.GROUP_STRIP, net.GROUP_STRIP_TRAIN = old
    return y, sv, used


@pytest.mark.parametrize("B,H", [(32, 64), (3, 16)])
def test_group_strip_training_saves_match_chain(B, H):
    """Training form (bf16): the launch also writes what the backward reads -- every RCAB's
    x_j, z1, a1, t_j, s, mean, hid and the chain's output -- equal to the per-RCAB training
    launches' saved tensors within the chain tolerance (2e-3 rel per RCAB; the two kernels sum
    in different orders), the gates within 2e-3; the output as in test_group_strip_vs_deferred_chain."""
    from src.hip import net
    dtype, n = torch.bfloat16, 4
    q = _params(n, seed=21)
    x = torch.randn(B, H, 64, 64, generator=torch.Generator().manual_seed(4)).to(DEV, dtype)
    old_pe, net.PRE_ELIDE = net.PRE_ELIDE, False      # every saved tensor written (z1 included)
    try:
        ys, svs, used = _run_save(q, n, x, dtype, True)
    finally:
        net.PRE_ELIDE = old_pe
    yd, svd, used_d = _run_save(q, n, x, dtype, False)
    assert used and not used_d
    tol = 2e-3 * (n + 1)
    assert _rel(ys.float(), yd.float()) <= tol
    assert _rel(svs["x_last"].float(), svd["x_last"].float()) <= tol
    for j, (a, b) in enumerate(zip(svs["blocks"], svd["blocks"])):
        for k in ("x", "z1", "a1", "t", "mean", "hid"):
            r = _rel(a[k].float(), b[k].float())
            assert r <= 2e-3 * (j + 1), (j, k, r)
        assert float((a["s"] - b["s"]).abs().max()) <= 2e-3, j
    assert svs["blocks"][0]["x"].data_ptr() == x.data_ptr()
