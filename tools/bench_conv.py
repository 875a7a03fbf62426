"""Microbenchmark of the conv3x3 kernels at the network's shapes (bf16, B=32).
Usage: FEN_CONV_VARIANT=k python tools/bench_conv.py   (prints one JSON line)"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch
from src.hip import lib as L, net
from src.hip.program import Ctx, ptr
torch.manual_seed(0)
dt = torch.bfloat16
ctx = Ctx(dt, 'cuda')
res = {"variant": os.environ.get("FEN_CONV_VARIANT", "0")}
def pack(w, mode):
    n = ctx.lib.fen_packed_elems(mode, w.shape[0], w.shape[1]); buf = torch.empty(n, dtype=dt, device='cuda')
    ctx.emit('p', ctx.lib.fen_pack_conv_w, ctx.code, mode, w.shape[0], w.shape[1], ptr(w), ptr(buf)); return buf
def timeit(fn, reps=20):
    """Kernel time without host gaps: `reps` launches captured in one hipGraph, replayed."""
    for _ in range(2): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3): g.replay()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps) * 1e3  # us
B = 32
# RCAB conv1 fwd: 64->64 @64x64 with PReLU
x = torch.randn(B, 64, 64, 64, device='cuda', dtype=dt)
w = torch.randn(64, 64, 3, 3, device='cuda') * 0.05
bias = torch.zeros(64, device='cuda'); al = torch.full((64,), 0.25, device='cuda')
wp = pack(w, 0); y = torch.empty_like(x)
flop = 2 * B * 64 * 64 * 64 * 576
us = timeit(lambda: net.conv(ctx, x, wp, B, 64, 64, 64, 64, bias=bias, epi=L.EPI_PRELU, alpha=al, y=y))
res["rcab_fwd_us"] = round(us, 2); res["rcab_fwd_tflops"] = round(flop / us / 1e6, 1)
if os.environ.get("ABLATE"):
    from src.hip.program import byref
    for dbg in (1, 2, 3):
        dd = L.ConvDesc(); dd.dtype, dd.B, dd.H, dd.W, dd.Cin, dd.Cout = ctx.code, B, 64, 64, 64, 64
        dd.x, dd.w, dd.bias, dd.epi, dd.alpha, dd.y = ptr(x), ptr(wp), ptr(bias), L.EPI_BIAS | L.EPI_PRELU, ptr(al), ptr(y)
        dd.debug = dbg
        us = timeit(lambda: ctx.emit("c", ctx.lib.fen_conv3x3, byref(dd)))
        res[f"rcab_fwd_debug{dbg}_us"] = round(us, 2)
part = torch.empty(B * 16, 64, device='cuda')
us = timeit(lambda: net.conv(ctx, x, wp, B, 64, 64, 64, 64, bias=bias, epi=L.EPI_POOL, y=y, part=part))
res["rcab_pool_us"] = round(us, 2)
if os.environ.get("ONLY_RCAB"):
    print(json.dumps(res)); sys.exit(0)
# upsample stage 1: 64->256 @128x128 shuffle prelu
x1 = torch.randn(B, 128, 128, 64, device='cuda', dtype=dt)
w1 = torch.randn(256, 64, 3, 3, device='cuda') * 0.05; b1 = torch.zeros(256, device='cuda')
wp1 = pack(w1, 1); y1 = torch.empty(B, 256, 256, 64, device='cuda', dtype=dt)
us = timeit(lambda: net.conv(ctx, x1, wp1, B, 128, 128, 64, 256, bias=b1, epi=L.EPI_PRELU | L.EPI_SHUFFLE, alpha=al, y=y1), 10)
res["up1_us"] = round(us, 2); res["up1_tflops"] = round(2 * B * 128 * 128 * 256 * 576 / us / 1e6, 1)
# conv_last fwd 64->3 @256x256 + bicubic
wl = torch.randn(3, 64, 3, 3, device='cuda') * 0.01; bl = torch.zeros(3, device='cuda')
wpl = pack(wl, 0); out = torch.empty(B, 3, 256, 256, device='cuda'); lr = torch.rand(B, 3, 64, 64, device='cuda')
us = timeit(lambda: net.conv(ctx, y1, wpl, B, 256, 256, 64, 3, bias=bl, epi=L.EPI_LAST, y=out, lr=lr, scale=4), 10)
res["last_us"] = round(us, 2); res["last_GBs"] = round(y1.numel() * 2 / us / 1e3, 1)
hrt = torch.rand(B, 3, 256, 256, device='cuda'); dol = torch.empty(B, 256, 256, 16, device='cuda', dtype=dt)
lpl = torch.empty(B * 256, 1, device='cuda')
us = timeit(lambda: net.conv(ctx, y1, wpl, B, 256, 256, 64, 3, bias=bl, epi=L.EPI_LAST, y=out, lr=lr, scale=4,
                             hr=hrt, dout=dol, l1_scale=1e-6, loss_part=lpl), 10)
res["last_train_us"] = round(us, 2)
# dgrad rcab with prelu_bwd
wd = pack(w, 2); dz = torch.empty_like(x)
us = timeit(lambda: net.conv(ctx, x, wd, B, 64, 64, 64, 64, epi=L.EPI_PRELU_BWD, alpha=al, pre_in=x, y=dz, part=part))
res["rcab_dgrad_us"] = round(us, 2)
# dgrad of conv1 + the identity-skip gradient (one residual, no bias)
us = timeit(lambda: net.conv(ctx, x, wd, B, 64, 64, 64, 64, res=(dz,), y=y))
res["rcab_dgrad_res_us"] = round(us, 2)
# upsample dgrad 256->64 unshuffle (streamed kernel)
du = torch.randn(B, 128, 128, 256, device='cuda', dtype=dt); wud = pack(w1, 2)
dprev = torch.empty(B, 64, 64, 256, device='cuda', dtype=dt); v = torch.randn(B, 128, 128, 64, device='cuda', dtype=dt)
partu = torch.empty(B * 64, 64, device='cuda')
us = timeit(lambda: net.conv(ctx, du, wud, B, 128, 128, 256, 64, epi=L.EPI_PRELU_BWD | L.EPI_UNSHUFFLE, alpha=al, pre_in=v, y=dprev, part=partu), 10)
res["up1_dgrad_us"] = round(us, 2)
# wgrad rcab
dw = torch.empty(64, 64, 3, 3, device='cuda'); db = torch.empty(64, device='cuda')
rctx = Ctx(dt, 'cuda', record=True)
net.wgrad(rctx, x, x, B, 64, 64, 64, 64, dw, db)
us = timeit(lambda: rctx.run())
res["rcab_wgrad_us"] = round(us, 2); res["rcab_wgrad_tflops"] = round(flop / us / 1e6, 1)
print(json.dumps(res))
# wgrad upsample stage 1 (Cin 64, Cout 256 @128x128)
dw1 = torch.empty(256, 64, 3, 3, device='cuda'); db1 = torch.empty(256, device='cuda')
rctx1 = Ctx(dt, 'cuda', record=True)
net.wgrad(rctx1, x1, du, B, 128, 128, 64, 256, dw1, db1)
us = timeit(lambda: rctx1.run(), 10)
res2 = {"up1_wgrad_us": round(us, 2), "up1_wgrad_tflops": round(2 * B * 128 * 128 * 256 * 576 / us / 1e6, 1)}
print(json.dumps(res2))
