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
