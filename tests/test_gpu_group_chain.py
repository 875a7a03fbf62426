"""GPU parity of fen_group_strip_chain -- the body's G ResidualGroups (reference
custom.py:168-169; each group blocks.py:185-189 with RCABs blocks.py:135-153) as ONE launch in
which every strip stays on its CU across the groups -- against a fen_group_strip launch per
group (itself oracle-checked in test_gpu_group_strip.py) and against the CPU oracle.

The chain does the per-group launches' arithmetic exactly (a group's output rounded to the
16-bit format, then kept in registers as the next group's x_0; the neighbours' rows of it by
hand-off; the skip input re-read from the output buffer), so the outputs and every gate are
compared BIT-EXACT with the per-group launches; the oracle bound is the per-group test's
(5e-3 bf16 / 1e-3 fp16 rel-L2 per RCAB + 1) summed over the groups.  Shapes: the bench's
(B=32, 64x64, 6 groups x 10 RCABs), one strip per image (H=8), 16 strips (H=128), more strips
than CUs (B=40), one image, 2 / 3 groups.  Graph replays are bit-identical with the counters
back at zero; a skipped hand-off flag surfaces as FenError."""
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"bf16": torch.bfloat16, "fp16": torch.float16}


def _params(G, n, seed):
    g = torch.Generator().manual_seed(seed)
    C, Cr = 64, 16
    q = {}
    for gi in range(G):
        pre = f"residual_groups.{gi}."
        for j in range(n):
            b = f"{pre}blocks.{j}."
            q[b + "conv1.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
            q[b + "conv1.bias"] = torch.randn(C, generator=g) * 0.1
            q[b + "prelu.weight"] = torch.rand(C, generator=g) * 0.5
            q[b + "conv2.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
            q[b + "conv2.bias"] = torch.randn(C, generator=g) * 0.1
            q[b + "channel_attention.fc.0.weight"] = torch.randn(Cr, C, generator=g) * 0.3
            q[b + "channel_attention.fc.2.weight"] = torch.randn(C, Cr, generator=g) * 0.3
        q[pre + "conv.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.05
        q[pre + "conv.bias"] = torch.randn(C, generator=g) * 0.1
    return q


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def _run(q, G, n, x, dtype, chain=True, record=False, fault=0):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.GROUP_CHAIN, net.GS_FAULT
    net.GROUP_CHAIN, net.GS_FAULT = chain, fault
    try:
        ctx = Ctx(dtype, DEV, record=record)
        Wt = Weights({k: v.to(DEV) for k, v in q.items()}, dtype, DEV)
        ctx.keep(Wt)
        attn = {}
        fw = Forward(NetSpec(C=64, G=G, NB=n, Cr=16), ctx, Wt, save=False, attn=attn)
        used = fw._chain_ok(x)
        outs = [torch.empty_like(x), torch.empty_like(x)]
        ctx.keep(outs)
        h, _ = fw.body(x, [outs[g & 1] for g in range(G)])
        if not record:
            torch.cuda.synchronize()
    finally:
        net.GROUP_CHAIN, net.GS_FAULT = old
    return h, attn, ctx, used


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
@pytest.mark.parametrize("B,H,G,n", [(32, 64, 6, 10), (2, 64, 3, 2), (3, 8, 2, 2), (2, 128, 2, 1), (40, 64, 2, 2),
                                     (1, 64, 3, 1)])
def test_group_chain_bit_exact_vs_per_group(prec, B, H, G, n):
    from src.hip import lib as L
    dtype = DT[prec]
    q = _params(G, n, seed=40 + G + n)
    x = torch.randn(B, H, 64, 64, generator=torch.Generator().manual_seed(11)).to(DEV, dtype)
    yc, attn_c, ctx, used = _run(q, G, n, x, dtype, chain=True)
    assert used, "outside fen_group_strip_chain's envelope"
    L.check_strip_status()
    yg, attn_g, _, _ = _run(q, G, n, x, dtype, chain=False)
    assert torch.equal(yc, yg)
    assert sorted(attn_c) == sorted(attn_g) and len(attn_c) == G * n
    for k in attn_c:
        assert torch.equal(attn_c[k], attn_g[k]), k
    # again on the same workspace: deterministic, counters reset by the first launch
    yc2, _, _, _ = _run(q, G, n, x, dtype, chain=True)
    assert torch.equal(yc2, yc)


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_group_chain_vs_oracle(prec):
    dtype = DT[prec]
    B, H, G, n = 2, 16, 3, 2
    q = _params(G, n, seed=9)
    x = torch.randn(B, 64, H, 64, generator=torch.Generator().manual_seed(5)).to(dtype).float()
    qr = {k: (v.to(dtype).float() if v.dim() == 4 else v) for k, v in q.items()}
    ref = x
    for g in range(G):
        ref = O.residual_group(ref, qr, f"residual_groups.{g}.", n, 0.2)
        ref = ref.to(dtype).float()                       # the group output as stored
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dtype)
    y, _, _, used = _run(q, G, n, xd, dtype)
    assert used
    r = _rel(y.float().cpu().permute(0, 3, 1, 2), ref)
    tol = (5e-3 if prec == "bf16" else 1e-3) * (n + 1) * G
    print(f"{prec}: rel {r:.2e}")
    assert r <= tol, r


def test_group_chain_graph_replay():
    """Recorded (one op) and replayed from a hipGraph five times: bit-identical to the eager
    launch, no wait timed out."""
    from src.hip import lib as L
    dtype, G, n = torch.float16, 6, 10
    q = _params(G, n, seed=12)
    x = torch.randn(32, 64, 64, 64, generator=torch.Generator().manual_seed(3)).to(DEV, dtype)
    y_e, _, _, _ = _run(q, G, n, x, dtype)
    y, _, ctx, _ = _run(q, G, n, x, dtype, record=True)
    assert [op[0] for op in ctx.ops] == ["group_strip_chain"]
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
        L.check_strip_status()


def test_group_chain_failed_wait_raises():
    """Fault injection (test-only flag): the block with ticket 1 skips its first a1 flag; the
    neighbour's bounded wait expires and the launch reports it -- FenError, not an output."""
    from src.hip import lib as L
    dtype, G, n = torch.bfloat16, 2, 1
    q = _params(G, n, seed=3)
    x = torch.randn(2, 64, 64, 64, generator=torch.Generator().manual_seed(1)).to(DEV, dtype)
    _run(q, G, n, x, dtype, fault=1)
    with pytest.raises(L.FenError):
        L.check_strip_status()
    L.check_strip_status()                                # cleared
    y, _, _, _ = _run(q, G, n, x, dtype)                  # the workspace is usable again
    yg, _, _, _ = _run(q, G, n, x, dtype, chain=False)
    assert torch.equal(y, yg)


def test_group_chain_refuses_unprepared():
    """The parameter table is checked by the kernel (ADVICE/VERDICT r4): a launch whose
    descriptors differ from the prepared table, or whose workspace was reallocated (a fresh
    zeroed buffer, and a stale copy of another table) and not prepared again, computes nothing
    and raises FenError at the next status check -- never a launch on a stale or null row.  A
    broken chain is refused on the host (FEN_EINVAL).  After prepare on the caller's stream
    (asynchronous) the launch matches the original output bit for bit."""
    from src.hip import lib as L
    dtype, G, n = torch.float16, 2, 1
    q = _params(G, n, seed=4)
    x = torch.randn(1, 64, 64, 64, generator=torch.Generator().manual_seed(2)).to(DEV, dtype)
    y_ref, _, _, _ = _run(q, G, n, x, dtype)
    L.check_strip_status()
    y, _, ctx, _ = _run(q, G, n, x, dtype, record=True)
    name, fn, (ds, ng, tp) = ctx.ops[0]
    assert name == "group_strip_chain"
    lib = L.load()
    s = torch.cuda.current_stream().cuda_stream
    # valid descriptors, not the prepared table's: refused by the kernel, nothing written
    old = ds[1].fc1[0]
    ds[1].fc1[0] = ds[1].fc2[0]
    try:
        y.fill_(7.0)
        assert fn(ds, ng, tp, s) == 0
        torch.cuda.synchronize()
        with pytest.raises(L.FenError, match="no parameter table"):
            L.check_strip_status()
        assert bool((y == 7.0).all())
    finally:
        ds[1].fc1[0] = old
    # not a chain (x aliases y): refused on the host
    old = ds[1].x
    ds[1].x = ds[1].y
    try:
        assert fn(ds, ng, tp, s) == -1
    finally:
        ds[1].x = old
    # a reallocated workspace (zeros), launched without prepare
    nbytes = int(ds[0].work_bytes)
    work2 = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
    old_work = ds[0].work
    for g in range(ng):
        ds[g].work = work2.data_ptr()
    assert fn(ds, ng, tp, s) == 0
    torch.cuda.synchronize()
    with pytest.raises(L.FenError, match="no parameter table"):
        L.check_strip_status()
    # a stale table of other descriptors in it (prepared, then the descriptors change)
    old = ds[0].b1[0]
    ds[0].b1[0] = ds[0].b2[0]
    assert lib.fen_group_strip_chain_prepare(ds, ng, tp, s) == 0
    ds[0].b1[0] = old
    assert fn(ds, ng, tp, s) == 0
    torch.cuda.synchronize()
    with pytest.raises(L.FenError, match="no parameter table"):
        L.check_strip_status()
    # prepared for these descriptors (async, on the stream): runs, bit-exact
    assert lib.fen_group_strip_chain_prepare(ds, ng, tp, s) == 0
    y.zero_()
    assert fn(ds, ng, tp, s) == 0
    torch.cuda.synchronize()
    L.check_strip_status()
    assert torch.equal(y, y_ref)
    for g in range(ng):
        ds[g].work = old_work


def _run_save(q, G, n, x, dtype, chain):
    from src.hip import net
    from src.hip.net import Forward, NetSpec, Weights
    from src.hip.program import Ctx
    old = net.GROUP_CHAIN
    net.GROUP_CHAIN = chain
    try:
        ctx = Ctx(dtype, DEV)
        Wt = Weights({k: v.to(DEV) for k, v in q.items()}, dtype, DEV)
        ctx.keep(Wt)
        fw = Forward(NetSpec(C=64, G=G, NB=n, Cr=16), ctx, Wt, save=True)
        used = fw._chain_ok(x)
        outs = [torch.empty_like(x) for _ in range(G)]
        ctx.keep(outs)
        h, saved = fw.body(x, outs)
        torch.cuda.synchronize()
    finally:
        net.GROUP_CHAIN = old
    return h, saved, used


@pytest.mark.parametrize("B,H,G,n,elide", [(32, 64, 6, 10, True), (2, 64, 3, 2, False), (3, 16, 2, 3, True)])
def test_group_chain_training_saves_bit_exact(B, H, G, n, elide):
    """Training form (bf16): the chained launch writes every group's saved set -- each RCAB's
    x_j, z1 (unless elided), a1, t_j, s, mean, hid and the chain's output -- bit-identical to a
    training launch per group, and the same outputs."""
    from src.hip import lib as L, net
    dtype = torch.bfloat16
    q = _params(G, n, seed=60 + n)
    x = torch.randn(B, H, 64, 64, generator=torch.Generator().manual_seed(8)).to(DEV, dtype)
    old_pe, net.PRE_ELIDE = net.PRE_ELIDE, elide
    try:
        yc, svc, used = _run_save(q, G, n, x, dtype, True)
        yg, svg, used_g = _run_save(q, G, n, x, dtype, False)
    finally:
        net.PRE_ELIDE = old_pe
    L.check_strip_status()
    assert used and not used_g
    assert torch.equal(yc, yg)
    assert len(svc) == len(svg) == G
    for g in range(G):
        a, b = svc[g], svg[g]
        assert a["z1_elided"] == b["z1_elided"]
        assert torch.equal(a["x"], b["x"]) and torch.equal(a["x_last"], b["x_last"]), g
        for j, (u, v) in enumerate(zip(a["blocks"], b["blocks"])):
            keys = ("x", "a1", "t", "mean", "hid", "s") + (() if a["z1_elided"] else ("z1",))
            for k in keys:
                assert torch.equal(u[k], v[k]), (g, j, k)


@pytest.mark.parametrize("prec", ["fp16", "bf16"])
@pytest.mark.parametrize("B,H,G,n", [(32, 64, 6, 10), (3, 16, 2, 1)])
def test_group_chain_after_body(prec, B, H, G, n):
    """conv_after_body (custom.py:172-175) as the chain's last step (a group of no RCABs):
    fb = conv(body output) + bias + feat0 against the per-op conv launch on the chain's own body
    output (same rounding points; the two kernels sum the 576 products in different orders:
    rel-L2 <= 1e-3 fp16 / 5e-3 bf16), the body output itself bit-exact."""
    from src.hip import lib as L, net
    from src.hip.net import Forward, NetSpec, Weights, conv
    from src.hip.program import Ctx
    dtype = DT[prec]
    q = _params(G, n, seed=77)
    g = torch.Generator().manual_seed(78)
    q["conv_after_body.weight"] = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    q["conv_after_body.bias"] = torch.randn(64, generator=g) * 0.1
    x = torch.randn(B, H, 64, 64, generator=torch.Generator().manual_seed(6)).to(DEV, dtype)
    ctx = Ctx(dtype, DEV)
    Wt = Weights({k: v.to(DEV) for k, v in q.items()}, dtype, DEV)
    ctx.keep(Wt)
    fw = Forward(NetSpec(C=64, G=G, NB=n, Cr=16), ctx, Wt, save=False)
    outs = [torch.empty_like(x), torch.empty_like(x)]
    fb = torch.empty_like(x)
    h, _ = fw.body(x, [outs[i & 1] for i in range(G)], fb=fb)
    assert fw.fb_done and fw._chain_ok(x)
    torch.cuda.synchronize()
    L.check_strip_status()
    ref = torch.empty_like(x)
    conv(ctx, h, Wt.packed("conv_after_body", 0), B, H, 64, 64, 64, bias=Wt.p["conv_after_body.bias"], y=ref,
         res=(x,))
    torch.cuda.synchronize()
    r = _rel(fb.float(), ref.float())
    print(f"{prec} B={B}: conv_after_body rel {r:.2e}")
    assert r <= (5e-3 if prec == "bf16" else 1e-3), r
    old = net.CHAIN_AFTER_BODY
    net.CHAIN_AFTER_BODY = False
    try:
        fw2 = Forward(NetSpec(C=64, G=G, NB=n, Cr=16), ctx, Wt, save=False)
        h2, _ = fw2.body(x, [torch.empty_like(x) for _ in range(G)], fb=torch.empty_like(x))
        assert not fw2.fb_done
        torch.cuda.synchronize()
    finally:
        net.CHAIN_AFTER_BODY = old
    assert torch.equal(h, h2)


@pytest.mark.parametrize("train", [False, True])
def test_engine_program_uses_the_chain(train):
    """The bench's engine (B=32, 6x10, 64x64; inference fp16, training bf16) records the body as
    ONE group_strip_chain launch with conv_after_body inside it: no per-group strip launches and
    no separate conv_after_body conv (its 64->64 conv at 64x64 with the feat0 residual)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import build_model
    from src.hip.engine import FENEngine
    prec = "bf16" if train else "fp16"
    eng = FENEngine(build_model(prec), batch=32, lr_hw=(64, 64), dtype=DT[prec], train=train, device=DEV)
    ops = [op[0] for op in eng.ctx.ops]
    assert ops.count("group_strip_chain") == 1 and "group_strip" not in ops, ops[:6]
    name, fn, (ds, ng, tail) = next(op for op in eng.ctx.ops if op[0] == "group_strip_chain")
    assert ng == 6 and tail is not None and ds[0].save == int(train)
    if not train:   # (training's program also holds the backward's 64->64 dgrads)
        convs = [op[2][0]._obj for op in eng.ctx.ops if op[0] == "conv3x3" and op[1] is not None]
        assert not any(d.Cin == 64 and d.Cout == 64 and d.H == 64 and d.W == 64 for d in convs)
