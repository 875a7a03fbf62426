"""conv_last (csrc/conv_last.hip) timing at B=32 256x256, inference and training epilogues."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch
from src.hip import lib as L, net
from src.hip.program import Ctx, ptr

B = 32
ctx = Ctx(torch.bfloat16, 'cuda')
x = torch.randn(B, 256, 256, 64, device='cuda', dtype=torch.bfloat16)
wl = torch.randn(3, 64, 3, 3, device='cuda') * 0.01; bl = torch.zeros(3, device='cuda')
wp = torch.empty(ctx.lib.fen_packed_elems(0, 3, 64), device='cuda', dtype=torch.bfloat16)
ctx.emit('p', ctx.lib.fen_pack_conv_w, ctx.code, 0, 3, 64, ptr(wl), ptr(wp))
out = torch.empty(B, 3, 256, 256, device='cuda'); lr = torch.rand(B, 3, 64, 64, device='cuda')
hr = torch.rand(B, 3, 256, 256, device='cuda'); do = torch.empty(B, 256, 256, 16, device='cuda', dtype=torch.bfloat16)
lp = torch.empty(B * 256, 1, device='cuda')


def timeit(f, n=20):
    """Device time per launch: n launches captured in one hipGraph, replayed (no host gaps)."""
    for _ in range(2): f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n): f()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


res = {"lib": os.path.basename(os.environ.get("FEN_HIP_LIB", "default"))}
us = timeit(lambda: net.conv(ctx, x, wp, B, 256, 256, 64, 3, bias=bl, epi=L.EPI_LAST, y=out, lr=lr, scale=4, clamp=1))
res["last_us"] = round(us, 2); res["GBs"] = round(x.numel() * 2 / us / 1e3, 1)
us = timeit(lambda: net.conv(ctx, x, wp, B, 256, 256, 64, 3, bias=bl, epi=L.EPI_LAST, y=out, lr=lr, scale=4,
                             hr=hr, dout=do, l1_scale=1e-6, loss_part=lp))
res["last_train_us"] = round(us, 2)
print(json.dumps(res))
# conv_first 3 -> 64 at 64x64 (the LR input, fp32 NCHW -> bf16 NHWC)
xl = torch.rand(B, 3, 64, 64, device='cuda'); wf = torch.randn(64, 3, 3, 3, device='cuda') * 0.2
bf = torch.zeros(64, device='cuda'); yf = torch.empty(B, 64, 64, 64, device='cuda', dtype=torch.bfloat16)
us = timeit(lambda: ctx.emit('cf', ctx.lib.fen_conv_first_fwd, ctx.code, B, 3, 64, 64, 64, ptr(xl), ptr(wf), ptr(bf), ptr(yf)))
print(json.dumps({"conv_first_us": round(us, 2), "GBs": round((xl.numel() * 4 + yf.numel() * 2) / us / 1e3, 1)}))
# SE backward pool: part = per-chunk sums of dy * t (B=32, 64x64x64)
ta = torch.randn(B, 64, 64, 64, device='cuda', dtype=torch.bfloat16); tb = torch.randn_like(ta)
pp = torch.empty(B * ctx.lib.fen_pool_parts(4096), 64, device='cuda')
us = timeit(lambda: ctx.emit('pd', ctx.lib.fen_pool_dot, ctx.code, B, 4096, 64, ptr(ta), ptr(tb), ptr(pp)))
print(json.dumps({"pool_dot_us": round(us, 2), "GBs": round(2 * ta.numel() * 2 / us / 1e3, 1)}))
# conv_last data gradient fused with the last upsampler stage's PReLU backward + PixelShuffle
# inverse (B=32, dout 256x256x16 -> du 128x128x256; pre 256x256x64)
pre = torch.randn(B, 256, 256, 64, device='cuda', dtype=torch.bfloat16); al = torch.full((64,), 0.25, device='cuda')
du = torch.empty(B, 128, 128, 256, device='cuda', dtype=torch.bfloat16); do.normal_()
dal = torch.empty(ctx.lib.fen_conv_last_dgrad_part_rows(B, 256, 256), 64, device='cuda')
us = timeit(lambda: ctx.emit('cld', ctx.lib.fen_conv_last_dgrad, ctx.code, B, 256, 256, 64, 3, ptr(do), ptr(wl), ptr(pre), None,
                             ptr(al), ptr(du), ptr(dal)))
print(json.dumps({"conv_last_dgrad_us": round(us, 2), "GBs": round((pre.numel() * 2 + du.numel() * 2 + do.numel() * 2) / us / 1e3, 1),
                  "du_sum": float(du.float().abs().sum())}))
