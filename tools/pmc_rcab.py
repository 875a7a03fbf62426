"""Launch the bench's dominant kernel (RCAB conv1: 64->64 3x3 + bias + PReLU, bf16,
B=32, 64x64, inference epilogue) REPS times, plainly (no graph), for rocprofv3 --pmc
passes.  Usage: rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- \
    python tools/pmc_rcab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402

from src.hip import lib as L, net  # noqa: E402
from src.hip.program import Ctx, ptr  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
B, H, W, C = 32, 64, 64, 64
torch.manual_seed(0)
ctx = Ctx(torch.bfloat16, "cuda")
x = torch.randn(B, H, W, C, device="cuda", dtype=torch.bfloat16)
w = torch.randn(C, C, 3, 3, device="cuda") * 0.05
n = ctx.lib.fen_packed_elems(0, C, C)
wp = torch.empty(n, dtype=torch.bfloat16, device="cuda")
ctx.emit("pack", ctx.lib.fen_pack_conv_w, ctx.code, 0, C, C, ptr(w), ptr(wp))
bias = torch.zeros(C, device="cuda")
alpha = torch.full((C,), 0.25, device="cuda")
y = torch.empty_like(x)
for _ in range(REPS):
    net.conv(ctx, x, wp, B, H, W, C, C, bias=bias, epi=L.EPI_PRELU, alpha=alpha, y=y)
torch.cuda.synchronize()
print("algorithmic_bytes_per_launch", x.numel() * 2 + y.numel() * 2 + n * 2 + 2 * C * 4)
