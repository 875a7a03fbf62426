"""VGG19 (to conv3_4) conv shapes through fen_conv3x3 at the perceptual loss's sizes: the
forward on 2B = 64 images (pred + target) and the dgrad on B = 32; TFLOP/s per layer."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch
from src.hip import lib as L, net
from src.hip.program import Ctx, ptr

dt = torch.bfloat16
ctx = Ctx(dt, 'cuda')


def pack(w, mode):
    n = ctx.lib.fen_packed_elems(mode, w.shape[0], w.shape[1]); buf = torch.empty(n, dtype=dt, device='cuda')
    ctx.emit('p', ctx.lib.fen_pack_conv_w, ctx.code, mode, w.shape[0], w.shape[1], ptr(w), ptr(buf)); return buf


def timeit(fn, reps=10):
    for _ in range(2): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


res = {}
for name, N, hw, cin, cout in [("c1_2", 64, 256, 64, 64), ("c2_1", 64, 128, 64, 128), ("c2_2", 64, 128, 128, 128),
                               ("c3_1", 64, 64, 128, 256), ("c3_2", 64, 64, 256, 256)]:
    x = torch.randn(N, hw, hw, cin, device='cuda', dtype=dt)
    w = torch.randn(cout, cin, 3, 3, device='cuda') * 0.05; b = torch.zeros(cout, device='cuda')
    y = torch.empty(N, hw, hw, cout, device='cuda', dtype=dt)
    wp = pack(w, 0)
    yp = torch.empty(N, hw // 2, hw // 2, cout, device='cuda', dtype=dt) if name in ("c1_2", "c2_2") else None
    us = timeit(lambda: net.conv(ctx, x, wp, N, hw, hw, cin, cout, bias=b, epi=L.EPI_PRELU, alpha=torch.zeros(cout, device='cuda'), y=y,
                                 y_pool=yp, y_images=N // 2 if yp is not None else 0))
    fl = 2 * N * hw * hw * cin * cout * 9
    res[name] = [round(us, 1), round(fl / us / 1e6, 1)]
    if cin >= 128:     # its data gradient at B = 32 through the ReLU mask (mode-2 weights: Cout <-> Cin)
        n2 = N // 2
        d = torch.randn(n2, hw, hw, cout, device='cuda', dtype=dt)
        pre = torch.randn(n2, hw, hw, cin, device='cuda', dtype=dt)
        dz = torch.empty(n2, hw, hw, cin, device='cuda', dtype=dt)
        part = torch.empty(n2 * ((hw + 15) // 16) ** 2, cin, device='cuda')
        wp2 = pack(w, 2)
        if cin % 128 == 0:
            us = timeit(lambda: net.conv(ctx, d, wp2, n2, hw, hw, cout, cin, epi=L.EPI_RELU_BWD, pre_in=pre, y=dz))
            res[name + "_dg"] = [round(us, 1), round(fl / 2 / us / 1e6, 1)]
print(json.dumps(res))
