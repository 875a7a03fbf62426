"""Phase timeline of the persistent conv kernel from in-kernel stamps (diagnostic build).

  make -C face-super-resolution_amd/csrc stamp
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so python tools/stamp_conv.py

Launches the RCAB conv1 (64->64 + bias + PReLU, bf16, B=32, 64x64) a few times and prints,
per phase, the median over blocks of the time since the kernel's earliest block start
(s_memrealtime, 100 MHz) and the median per-block duration in shader cycles (s_memtime).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402

from src.hip import lib as L, net  # noqa: E402
from src.hip.program import Ctx, ptr  # noqa: E402

B, H, W, C = int(os.environ.get("B", "32")), 64, 64, 64
torch.manual_seed(0)
ctx = Ctx(torch.bfloat16, "cuda")
x = torch.randn(B, H, W, C, device="cuda", dtype=torch.bfloat16)
w = torch.randn(C, C, 3, 3, device="cuda") * 0.05
wp = torch.empty(ctx.lib.fen_packed_elems(0, C, C), dtype=torch.bfloat16, device="cuda")
ctx.emit("pack", ctx.lib.fen_pack_conv_w, ctx.code, 0, C, C, ptr(w), ptr(wp))
bias = torch.zeros(C, device="cuda")
alpha = torch.full((C,), 0.25, device="cuda")
y = torch.empty_like(x)
nblk = 4096
st = torch.zeros(nblk * 32, dtype=torch.int64, device="cuda")
epi = int(os.environ.get("EPI", str(L.EPI_PRELU)))
for _ in range(int(os.environ.get("REPS", "30"))):
    st.zero_()
    net.conv(ctx, x, wp, B, H, W, C, C, bias=bias, epi=epi, alpha=alpha, y=y, loss_part=st)
torch.cuda.synchronize()
a = st.view(nblk, 16, 2).cpu().numpy().astype(np.int64)
used = a[:, 0, 0] != 0
a = a[used]
rt, mt = a[:, :, 0], a[:, :, 1]
t0 = rt[:, 0].min()
out = {"blocks": int(used.sum())}
names = ["start", "prologue"] + [f"t{k}_{p}" for k in range(5) for p in ("mfma", "epi", "bar")]
for i, nm in enumerate(names[:16]):
    valid = rt[:, i] != 0
    if not valid.any():
        continue
    out[nm + "_us"] = round(float(np.median(rt[valid, i] - t0)) / 100.0, 2)
    if i:
        prev = i - 1
        v2 = valid & (mt[:, prev] != 0)
        out[nm + "_cyc"] = int(np.median(mt[v2, i] - mt[v2, prev]))
out["end_max_us"] = round(float((rt.max() - t0)) / 100.0, 2)
out["start_spread_us"] = round(float(rt[:, 0].max() - t0) / 100.0, 2)
print(json.dumps(out))
