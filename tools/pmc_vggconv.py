"""One VGG19 conv shape through fen_conv3x3 (bf16), repeated -- for rocprofv3 counter passes of
the streamed conv kernel.  SHAPE=c3_2 (N=64, 64x64, 256->256, bias+ReLU) by default; others as in
bench_vgg_conv.py; DGRAD=1: the data-gradient form (N=32, ReLU-backward epilogue)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch
from src.hip import lib as L, net
from src.hip.program import Ctx, ptr
SHAPES = {"c2_2": (64, 128, 128, 128), "c3_1": (64, 64, 128, 256), "c3_2": (64, 64, 256, 256)}
N, hw, cin, cout = SHAPES[os.environ.get("SHAPE", "c3_2")]
dt = torch.bfloat16
ctx = Ctx(dt, 'cuda')
dg = os.environ.get("DGRAD") == "1"
if dg:
    N //= 2
x = torch.randn(N, hw, hw, cin, device='cuda', dtype=dt)
w = torch.randn(cout, cin, 3, 3, device='cuda') * 0.05
b = torch.zeros(cout, device='cuda')
y = torch.empty(N, hw, hw, cout, device='cuda', dtype=dt)
n = ctx.lib.fen_packed_elems(0, cout, cin)
wp = torch.empty(n, dtype=dt, device='cuda')
L.check(ctx.lib.fen_pack_conv_w(ctx.code, 0, cout, cin, ptr(w), ptr(wp), torch.cuda.current_stream().cuda_stream), "pack")
pre = torch.randn(N, hw, hw, cout, device='cuda', dtype=dt)
part = torch.empty(N * ((hw + 15) // 16) ** 2, cout, device='cuda')
for _ in range(int(os.environ.get("REPS", "10"))):
    if dg:
        net.conv(ctx, x, wp, N, hw, hw, cin, cout, epi=L.EPI_RELU_BWD, pre_in=pre, y=y)
    else:
        net.conv(ctx, x, wp, N, hw, hw, cin, cout, bias=b, epi=L.EPI_PRELU, alpha=torch.zeros(cout, device='cuda'), y=y)
torch.cuda.synchronize()
print("done")
