"""Launch the bench's dominant kernel REPS times, plainly (no graph), for rocprofv3 --pmc
passes: one RCAB of the chain on fen_rcab_deferred (deferred input: the previous RCAB's gate
and residual applied to the input halo, conv1 + PReLU + conv2 + tile sums), inference form,
B=32, 64x64x64, fp16 (PREC=bf16 for bf16).  Prints the algorithmic bytes per launch.
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
dt = torch.bfloat16 if os.environ.get("PREC", "fp16") == "bf16" else torch.float16
B, H, W, C, CR = 32, 64, 64, 64, 16
T = (H // 16) * (W // 16)
torch.manual_seed(0)
p = {"conv1.weight": torch.randn(C, C, 3, 3) * 0.06, "conv1.bias": torch.zeros(C), "prelu.weight": torch.full((C,), .25),
     "conv2.weight": torch.randn(C, C, 3, 3) * 0.06, "conv2.bias": torch.zeros(C),
     "fc1": torch.randn(CR, C) * .3, "fc2": torch.randn(C, CR) * .3}
pd = {k: v.cuda() for k, v in p.items()}
Wt = Weights(pd, dt, "cuda")
x = torch.randn(B, H, W, C, device="cuda").to(dt)
tp = torch.randn(B, H, W, C, device="cuda").to(dt)
pp = torch.randn(B * T, C, device="cuda")
xo, t = torch.empty_like(x), torch.empty_like(x)
part = torch.empty(B * T, C, device="cuda")
lib = L.load()
d = L.RcabDeferredDesc()
d.dtype, d.B, d.H, d.W, d.C, d.Cr = L.dtype_code(dt), B, H, W, C, CR
d.x, d.tp, d.pp, d.pfc1, d.pfc2, d.xo = ptr(x), ptr(tp), ptr(pp), ptr(pd["fc1"]), ptr(pd["fc2"]), ptr(xo)
d.w1, d.b1, d.alpha = ptr(Wt.packed("conv1", 0)), ptr(pd["conv1.bias"]), ptr(pd["prelu.weight"])
d.w2, d.b2 = ptr(Wt.packed("conv2", 0)), ptr(pd["conv2.bias"])
d.res_scale, d.inv_hw = 0.2, 1.0 / (H * W)
d.t, d.part = ptr(t), ptr(part)
stream = torch.cuda.current_stream().cuda_stream
for _ in range(REPS):
    L.check(lib.fen_rcab_deferred(ctypes.byref(d), stream), "rcab_deferred")
torch.cuda.synchronize()
# x_{j-1} and t_{j-1} in, x_j and t_j out (16-bit NHWC), both packed filters, the previous
# RCAB's tile partials + SE weights in, this RCAB's partials out, biases / alpha
alg = 4 * x.numel() * 2 + 2 * 9 * C * C * 2 + 2 * B * T * C * 4 + 2 * CR * C * 4 + 3 * C * 4
print("algorithmic_bytes_per_launch", alg)
