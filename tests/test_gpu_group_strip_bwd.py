"""GPU parity of fen_group_strip_bwd -- a whole ResidualGroup's backward (autograd of reference
blocks.py:185-189: the group conv and its skip, then each RCAB blocks.py:135-153 with its
ChannelAttention blocks.py:83-92, in reverse) as ONE strip-resident launch, followed by the
batched weight gradients and column sums -- against autograd of the CPU oracle's
residual_group on the same 16-bit-rounded weights and input, and against the per-RCAB
backward launches (fen_rcab_bwd with the folded SE backward) on the same saved tensors.

Tolerances.  Both HIP paths round dt, dz1 and every RCAB's input gradient to the 16-bit format
(their SE-backward sums run in different orders: strips vs 16x16 tiles), so in bf16 (the
training precision) each is compared to the fp32 oracle and the strip path must be no further
from it than the per-RCAB path (x 1.25, + a floor of 1e-2 rel-L2 for tensors both get almost
exactly), whole-tensor rel-L2 for dx and for every parameter gradient; in fp16 (data path and
PReLU / SE gradients only: the weight-gradient kernels are bf16 / fp32) at absolute bounds, dx
5e-3 and those gradients 2e-2.  A wrong halo row, hand-off, tap, gate or SE term shows up as O(1).
Shapes: the bench's (B=32, 64x64, 10 RCABs), a single strip per image (H=8), three strips
(H=24), 16 strips (H=128), more strips than CUs (B=40: 320 blocks), with the second residual
(the body's first group).  Every launch leaves its counters at zero and its error word clear;
repeats and graph replays are bit-identical."""
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
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


class _NoWgrad:
    """Stands in for the backward's weight-gradient batch (fp16: fen_wgrad3x3 is bf16 / fp32)."""

    def add(self, *a):
        pass

    def flush(self):
        pass


def _fwd_bwd(q, n, x, dy, dtype, strip_bwd, dres=None, record=False, wgrads=True):
    """Forward (training, strip kernel) + the group's backward; -> (dx, grads, ctx, used)."""
    from src.hip import net
    from src.hip.net import Backward, Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.GROUP_STRIP_BWD
    net.GROUP_STRIP_BWD = strip_bwd
    try:
        ctx = Ctx(dtype, DEV, record=record)
        pd = {k: v.to(DEV) for k, v in q.items()}
        Wt = Weights(pd, dtype, DEV)
        ctx.keep(Wt)
        spec = NetSpec(C=64, G=1, NB=n, Cr=16)
        fw = Forward(spec, ctx, Wt, save=True)
        _, sv = fw.group(x, 0, pre="rg.")
        G = {k: torch.zeros_like(v) for k, v in pd.items()}
        ctx.keep(G)
        bw = Backward(spec, ctx, Wt, G)
        if not wgrads:
            bw.wb = _NoWgrad()
        extra = (dres,) if dres is not None else ()
        used = bw._strip_bwd_ok(sv, dy, extra)
        dx = bw.group(sv, dy, 0, extra_res=extra, pre="rg.")
        if not record:
            torch.cuda.synchronize()
    finally:
        net.GROUP_STRIP_BWD = old
    return dx, G, ctx, used


def _oracle(q, n, x_nchw, dy_nchw, dtype, dres_nchw=None):
    """fp32 autograd of the oracle's residual_group on the 16-bit-rounded conv weights."""
    leaves = {k: (v.to(dtype).float() if v.dim() == 4 else v.clone()).requires_grad_(True) for k, v in q.items()}
    xl = x_nchw.clone().requires_grad_(True)
    y = O.residual_group(xl, leaves, "rg.", n, 0.2)
    (y * dy_nchw).sum().backward()
    dx = xl.grad + (dres_nchw if dres_nchw is not None else 0.0)
    return dx, {k: v.grad for k, v in leaves.items()}


def _work_error(ctx):
    from src.hip import lib as L
    L.check_strip_status()
    bufs = [v for k, v in ctx._shared.items() if k.startswith("pz:group_strip_bwd")]
    assert bufs
    ints = [b[:256].view(torch.int32).cpu() for b in bufs]
    return [(int(t[0]), int(t[1]), int(t[2])) for t in ints]   # ticket, done, error


def _inputs(B, H, dtype, seed, dres=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 64, H, 64, generator=g).to(dtype).float()
    dy = (torch.randn(B, 64, H, 64, generator=g) * 1e-2).to(dtype).float()
    r = (torch.randn(B, 64, H, 64, generator=g) * 1e-2).to(dtype).float() if dres else None
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().to(DEV, dtype) if t is not None else None
    return x, dy, r, nhwc(x), nhwc(dy), nhwc(r)


SHAPES = [(4, 64, 10, False), (3, 8, 2, False), (2, 24, 3, True), (2, 128, 2, False), (40, 64, 2, False)]


@pytest.mark.parametrize("B,H,n,dres", SHAPES)
def test_group_strip_bwd_vs_oracle(B, H, n, dres):
    """bf16 (the training precision): dx and every parameter gradient vs the oracle, no further
    from it than the per-RCAB backward."""
    prec = "bf16"
    dtype = DT[prec]
    q = _params(n, seed=41 + n)
    x, dy, r, xd, dyd, rd = _inputs(B, H, dtype, seed=B + H, dres=dres)
    dx_ref, g_ref = _oracle(q, n, x, dy, dtype, r)
    dx_s, g_s, ctx, used = _fwd_bwd(q, n, xd, dyd, dtype, True, dres=rd)
    assert used, "outside fen_group_strip_bwd's envelope"
    assert _work_error(ctx) == [(0, 0, 0)]
    dx_p, g_p, _, used_p = _fwd_bwd(q, n, xd, dyd, dtype, False, dres=rd)
    assert not used_p
    nchw = lambda t: t.float().cpu().permute(0, 3, 1, 2)
    floor = 1e-2
    es, ep = _rel(nchw(dx_s), dx_ref), _rel(nchw(dx_p), dx_ref)
    print(f"{prec} B={B} H={H} n={n} dres={dres}: dx strip {es:.2e} per-RCAB {ep:.2e}")
    assert es <= 1.25 * ep + floor, (es, ep)
    worst = (0.0, "")
    for k in g_ref:
        es, ep = _rel(g_s[k], g_ref[k]), _rel(g_p[k], g_ref[k])
        worst = max(worst, (es, k))
        assert es <= 1.25 * ep + floor, (k, es, ep)
    print(f"  worst parameter gradient: {worst[1]} rel {worst[0]:.2e}")
    # again: deterministic (fixed-order sums), counters reset by the first launch
    dx2, g2, ctx2, _ = _fwd_bwd(q, n, xd, dyd, dtype, True, dres=rd)
    assert torch.equal(dx2, dx_s)
    for k in g_s:
        assert torch.equal(g2[k], g_s[k]), k
    assert _work_error(ctx2) == [(0, 0, 0)]


@pytest.mark.parametrize("B,H,n,dres", SHAPES)
def test_group_strip_bwd_fp16_vs_oracle(B, H, n, dres):
    """fp16 (the kernel's other 16-bit form; the weight-gradient kernels are bf16 / fp32, so the
    data path only): dx within 5e-3 and the PReLU / SE weight gradients within 2e-2 rel-L2 of the
    oracle's fp32 autograd."""
    dtype = torch.float16
    q = _params(n, seed=41 + n)
    x, dy, r, xd, dyd, rd = _inputs(B, H, dtype, seed=B + H, dres=dres)
    dx_ref, g_ref = _oracle(q, n, x, dy, dtype, r)
    dx_s, g_s, ctx, used = _fwd_bwd(q, n, xd, dyd, dtype, True, dres=rd, wgrads=False)
    assert used and _work_error(ctx) == [(0, 0, 0)]
    e = _rel(dx_s.float().cpu().permute(0, 3, 1, 2), dx_ref)
    worst = (0.0, "")
    for k in g_ref:
        if "prelu" in k or "channel_attention" in k:
            worst = max(worst, (_rel(g_s[k], g_ref[k]), k))
    print(f"fp16 B={B} H={H} n={n} dres={dres}: dx {e:.2e}, worst PReLU/SE gradient {worst[1]} {worst[0]:.2e}")
    assert e <= 5e-3
    assert worst[0] <= 2e-2, worst


def test_group_strip_bwd_vs_per_rcab_bench_shape():
    """The bench's shape (B=32, 64x64, 10 RCABs: one strip per CU), bf16: the strip backward and
    the per-RCAB launches on the same saved tensors agree within the summation-order difference
    (rel-L2 2e-2 on dx and every parameter gradient)."""
    prec = "bf16"
    dtype = DT[prec]
    n = 10
    q = _params(n, seed=8)
    _, _, _, xd, dyd, _ = _inputs(32, 64, dtype, seed=6)
    dx_s, g_s, ctx, used = _fwd_bwd(q, n, xd, dyd, dtype, True)
    dx_p, g_p, _, _ = _fwd_bwd(q, n, xd, dyd, dtype, False)
    assert used and _work_error(ctx) == [(0, 0, 0)]
    tol = 2e-2
    r = _rel(dx_s.float(), dx_p.float())
    worst = (0.0, "")
    for k in g_s:
        worst = max(worst, (_rel(g_s[k], g_p[k]), k))
    print(f"{prec}: dx {r:.2e}, worst gradient {worst[1]} {worst[0]:.2e}")
    assert r <= tol
    assert worst[0] <= tol, worst


def test_group_strip_bwd_graph_replay():
    """Forward + backward recorded and replayed from a hipGraph three times: bit-identical to
    the eager run, the counters back at zero after every replay."""
    dtype, n = torch.bfloat16, 10
    q = _params(n, seed=13)
    _, _, _, xd, dyd, _ = _inputs(32, 64, dtype, seed=2)
    dx_e, g_e, _, _ = _fwd_bwd(q, n, xd, dyd, dtype, True)
    dx, G, ctx, used = _fwd_bwd(q, n, xd, dyd, dtype, True, record=True)
    assert used and "group_strip_bwd" in [op[0] for op in ctx.ops]
    ctx.run()
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_e)
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        ctx.run()
    for _ in range(3):
        dx.zero_()
        for v in G.values():
            v.zero_()
        gph.replay()
        torch.cuda.synchronize()
        assert torch.equal(dx, dx_e)
        for k in G:
            assert torch.equal(G[k], g_e[k]), k
        assert _work_error(ctx) == [(0, 0, 0)]


@pytest.mark.parametrize("mixed", [False, True])
def test_group_strip_pre_elide(mixed, monkeypatch):
    """fen_group_strip_desc.pre_elide / fen_group_strip_bwd_desc.a1 (net.PRE_ELIDE): the training
    forward leaves z1 unwritten for an RCAB whose slopes are all > 0 and the backward recovers
    it from a1.  PReLU' depends on z1's sign only, so dx and every gradient but the slopes' are
    bit-identical to the run that saves z1; the slopes' gradient (sum g * z1 over z1 <= 0)
    differs by a1's rounding (bf16: 2^-9 relative per term).  mixed: RCAB 1 has one slope
    <= 0 -- it saves and reads z1, so its slope gradient is bit-identical too."""
    from src.hip import net
    B, H, n = 4, 64, 3
    q = _params(n, seed=31)
    if mixed:
        q["rg.blocks.1.prelu.weight"][3] = -0.1
    _, _, _, x, dy, _ = _inputs(B, H, torch.bfloat16, seed=32)
    out = {}
    for el in (False, True):
        monkeypatch.setattr(net, "PRE_ELIDE", el)
        dx, G, ctx, used = _fwd_bwd(q, n, x, dy, torch.bfloat16, True)
        assert used
        assert all(e == 0 for (_, _, e) in _work_error(ctx))
        out[el] = (dx.clone(), {k: v.clone() for k, v in G.items()})
    assert torch.equal(out[True][0], out[False][0])
    for k, g0 in out[False][1].items():
        g1 = out[True][1][k]
        if k.endswith("prelu.weight") and not (mixed and k.startswith("rg.blocks.1.")):
            assert _rel(g1, g0) <= 1e-2, (k, _rel(g1, g0))
        else:
            assert torch.equal(g1, g0), k
