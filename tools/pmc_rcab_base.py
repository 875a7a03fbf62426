"""A/B helper (not a product tool): tools/pmc_rcab.py as of the base commit, bound to that commit's
descriptor, for FEN_HIP_LIB=<base library>."""

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
from ctypes import Structure, c_float, c_int, c_void_p  # noqa: E402


class OldDesc(Structure):   # fen_rcab_deferred_desc as of the base commit
    _fields_ = [
        ("dtype", c_int), ("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("Cr", c_int),
        ("x", c_void_p), ("tp", c_void_p), ("pp", c_void_p), ("pfc1", c_void_p), ("pfc2", c_void_p),
        ("res_scale", c_float), ("inv_hw", c_float), ("ps", c_void_p), ("pmean", c_void_p), ("phid", c_void_p),
        ("xo", c_void_p), ("w1", c_void_p), ("b1", c_void_p), ("alpha", c_void_p), ("w2", c_void_p),
        ("b2", c_void_p), ("t", c_void_p), ("part", c_void_p), ("z1", c_void_p), ("a1", c_void_p),
        ("stamps", c_void_p),
    ]


L.load()
lib = ctypes.CDLL(L.LIB_PATH)
d = OldDesc()
d.dtype, d.B, d.H, d.W, d.C, d.Cr = L.dtype_code(dt), B, H, W, C, CR
d.x, d.tp, d.pp, d.pfc1, d.pfc2, d.xo = ptr(x), ptr(tp), ptr(pp), ptr(pd["fc1"]), ptr(pd["fc2"]), ptr(xo)
d.w1, d.b1, d.alpha = ptr(Wt.packed("conv1", 0)), ptr(pd["conv1.bias"]), ptr(pd["prelu.weight"])
d.w2, d.b2 = ptr(Wt.packed("conv2", 0)), ptr(pd["conv2.bias"])
d.res_scale, d.inv_hw = 0.2, 1.0 / (H * W)
d.t, d.part = ptr(t), ptr(part)
stream = torch.cuda.current_stream().cuda_stream
for _ in range(REPS):
    L.check(lib.fen_rcab_deferred(ctypes.byref(d), c_void_p(stream)), "rcab_deferred")
torch.cuda.synchronize()
# x_{j-1} and t_{j-1} in, x_j and t_j out (16-bit NHWC), both packed filters, the previous
# RCAB's tile partials + SE weights in, this RCAB's partials out, biases / alpha
alg = 4 * x.numel() * 2 + 2 * 9 * C * C * 2 + 2 * B * T * C * 4 + 2 * CR * C * 4 + 3 * C * 4
print("algorithmic_bytes_per_launch", alg)
