"""Phase timeline of the persistent conv kernel from in-kernel stamps (diagnostic build).

  make -C face-super-resolution_amd/csrc stamp
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so python tools/stamp_conv.py

Launches the RCAB conv1 (64->64 + bias + PReLU, bf16, B=32, 64x64) a few times and prints,
per phase, the median over blocks of the time since the kernel's earliest block start
(s_memrealtime, 100 MHz) and the median per-block duration in shader cycles (s_memtime).
UP=1: the inference upsampler's stage 1 instead (64 -> 256 + bias + PReLU + PixelShuffle,
fp16, 128x128 -> 256x256, packed mode 1).
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

UP = os.environ.get("UP", "0") == "1"
B, C = int(os.environ.get("B", "32")), 64
H = W = 128 if UP else 64
CO, MODE = (4 * C, 1) if UP else (C, 0)
DT = torch.float16 if UP else torch.bfloat16
torch.manual_seed(0)
ctx = Ctx(DT, "cuda")
x = torch.randn(B, H, W, C, device="cuda", dtype=DT)
w = torch.randn(CO, C, 3, 3, device="cuda") * 0.05
wp = torch.empty(ctx.lib.fen_packed_elems(MODE, CO, C), dtype=DT, device="cuda")
ctx.emit("pack", ctx.lib.fen_pack_conv_w, ctx.code, MODE, CO, C, ptr(w), ptr(wp))
bias = torch.zeros(CO, device="cuda")
alpha = torch.full((C,), 0.25, device="cuda")
y = torch.empty(B, 2 * H, 2 * W, C, device="cuda", dtype=DT) if UP else torch.empty_like(x)
nblk = 1024
st = torch.zeros(nblk * 8 * 32, dtype=torch.int64, device="cuda")
epi = int(os.environ.get("EPI", str(L.EPI_PRELU | (L.EPI_SHUFFLE if UP else 0))))
for _ in range(int(os.environ.get("REPS", "30"))):
    st.zero_()
    net.conv(ctx, x, wp, B, H, W, C, CO, bias=bias, epi=epi, alpha=alpha, y=y, loss_part=st,
             debug=int(os.environ.get("DEBUG", "0")))
torch.cuda.synchronize()
a = st.view(nblk, 8, 16, 2).cpu().numpy().astype(np.int64)
used = a[:, 0, 0, 0] != 0
a = a[used]                      # [blk, wave, stamp, (rt, mt)]
nw = int((a[0, :, 0, 0] != 0).sum())
a = a[:, :nw]
rt = a[..., 0]
t0 = rt[:, :, 0].min()
# slot -> label: 0 start, 1 end of start-up, 2+3k / 3+3k / 4+3k: tile k after MFMAs / after
# epilogue / after the closing barrier; 13, 14: q-kernel start-up (DMA issued, DMA landed)
labels = {0: "start", 1: "startup"}
if os.environ.get("FEN_CONV_VARIANT", "0") == "5":   # single-group kernel: 3 stamps per tile
    for k in range(4):
        labels.update({2 + 3 * k: f"t{k}_mfma", 3 + 3 * k: f"t{k}_epi", 4 + 3 * k: f"t{k}_bar"})
else:                                                # ping-pong kernel: 2 stamps per phase
    for k in range(7):
        labels.update({2 + 2 * k: f"ph{k}_work", 3 + 2 * k: f"ph{k}_bar"})
out = {"blocks": int(used.sum()), "waves": nw}
for i in sorted(labels):
    valid = (rt[:, :, i] != 0).all(axis=1)
    if not valid.any():
        continue
    r = (rt[valid, :, i] - t0) / 100.0          # us since the first start, per wave
    if os.environ.get("FEN_CONV_VARIANT", "0") == "5" or nw < 8:
        out[labels[i]] = [round(float(np.median(r.min(1))), 2), round(float(np.median(r.max(1))), 2)]
    else:   # [group A min, max, group B min, max]
        out[labels[i]] = [round(float(np.median(r[:, :4].min(1))), 2), round(float(np.median(r[:, :4].max(1))), 2),
                          round(float(np.median(r[:, 4:].min(1))), 2), round(float(np.median(r[:, 4:].max(1))), 2)]
mt = a[..., 1]
valid = (rt[:, :, 1] != 0).all(axis=1) & (rt[:, :, 2] != 0).all(axis=1)
dm = (mt[valid, :, 2] - mt[valid, :, 1]).astype(np.float64)
dr = (rt[valid, :, 2] - rt[valid, :, 1]).astype(np.float64)
out["t0_mfma_GHz"] = round(float(np.median(dm / np.maximum(dr, 1))) * 0.1, 3)
out["end_max_us"] = round(float((rt.max() - t0)) / 100.0, 2)
print(json.dumps(out))
