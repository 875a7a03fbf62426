"""Launch the bench's dominant kernel REPS times, plainly (no graph), for rocprofv3 --pmc
passes: the fused RCAB block (fen_rcab_fused, inference form: conv1 + PReLU + conv2 + SE
gate + residual, bf16, B=32, 64x64x64).  Prints the algorithmic bytes per launch.
Usage: rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python tools/pmc_rcab.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402

from src.hip import lib as L  # noqa: E402
from src.hip.net import Weights  # noqa: E402
from src.hip.program import ptr  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
B, H, W, C, CR = 32, 64, 64, 64, 4
torch.manual_seed(0)
p = {"conv1.weight": torch.randn(C, C, 3, 3) * 0.06, "conv1.bias": torch.zeros(C), "prelu.weight": torch.full((C,), .25),
     "conv2.weight": torch.randn(C, C, 3, 3) * 0.06, "conv2.bias": torch.zeros(C),
     "fc1": torch.randn(CR, C) * .3, "fc2": torch.randn(C, CR) * .3}
pd = {k: v.cuda() for k, v in p.items()}
Wt = Weights(pd, torch.bfloat16, "cuda")
x = torch.randn(B, H, W, C, device="cuda", dtype=torch.bfloat16)
y = torch.empty_like(x)
s = torch.empty(B, C, device="cuda")
lib = L.load()
ws = L.RcabWorkspace(B, H, W)
d = L.RcabDesc()
d.dtype, d.B, d.H, d.W, d.C, d.Cr = L.BF16, B, H, W, C, CR
d.x, d.w1, d.b1, d.alpha = ptr(x), ptr(Wt.packed("conv1", 0)), ptr(pd["conv1.bias"]), ptr(pd["prelu.weight"])
d.w2, d.b2, d.fc1, d.fc2 = ptr(Wt.packed("conv2", 0)), ptr(pd["conv2.bias"]), ptr(pd["fc1"]), ptr(pd["fc2"])
d.res_scale, d.inv_hw = 0.2, 1.0 / (H * W)
d.y, d.s, d.ws = ptr(y), ptr(s), ws.ptr
stream = torch.cuda.current_stream().cuda_stream
for _ in range(REPS):
    L.check(lib.fen_rcab_fused(ctypes.byref(d), stream), "rcab")
torch.cuda.synchronize()
assert lib.fen_rcab_workspace_status(ws.ptr, B, H, W) == 0
# x in, y out, both packed filters (2 x 9 x 64 x 64 bf16), biases / alpha / fc weights, s out
alg = 2 * x.numel() * 2 + 2 * 9 * C * C * 2 + 3 * C * 4 + 2 * CR * C * 4 + B * C * 4
print("algorithmic_bytes_per_launch", alg)
