"""Phase timeline of the fused RCAB kernel (diagnostic build with -DFEN_STAMPS).
  make -C face-super-resolution_amd/csrc stamp
  FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_stamp.so python tools/stamp_rcab.py
Prints, per stamp slot, [median over blocks of the earliest wave, of the latest wave] in us
since the kernel's first stamp."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import numpy as np
import torch
from src.hip import lib as L
from src.hip.net import Weights
from src.hip.program import Ctx, ptr

B = int(os.environ.get("B", "32")); H = W = 64
torch.manual_seed(0)
p = {"conv1.weight": torch.randn(64, 64, 3, 3) * 0.06, "conv1.bias": torch.zeros(64), "prelu.weight": torch.full((64,), .25),
     "conv2.weight": torch.randn(64, 64, 3, 3) * 0.06, "conv2.bias": torch.zeros(64),
     "fc1": torch.randn(16, 64) * .3, "fc2": torch.randn(64, 16) * .3}
pd = {k: v.cuda() for k, v in p.items()}
ctx = Ctx(torch.bfloat16, 'cuda')
Wt = Weights(pd, torch.bfloat16, 'cuda')
x = torch.randn(B, H, W, 64, device='cuda', dtype=torch.bfloat16)
y = torch.empty_like(x)
s = torch.empty(B, 64, device='cuda')
lib = L.load()
ws = L.RcabWorkspace(B, H, W)
st = torch.zeros(256 * 8 * 48, dtype=torch.int64, device='cuda')
d = L.RcabDesc()
d.dtype, d.B, d.H, d.W, d.C, d.Cr = L.BF16, B, H, W, 64, 16
d.x, d.w1, d.b1, d.alpha = ptr(x), ptr(Wt.packed("conv1", 0)), ptr(pd["conv1.bias"]), ptr(pd["prelu.weight"])
d.w2, d.b2, d.fc1, d.fc2 = ptr(Wt.packed("conv2", 0)), ptr(pd["conv2.bias"]), ptr(pd["fc1"]), ptr(pd["fc2"])
d.res_scale, d.inv_hw = 0.2, 1.0 / (H * W)
d.y, d.s, d.ws, d.stamps = ptr(y), ptr(s), ws.ptr, ptr(st)
for _ in range(int(os.environ.get("REPS", "20"))):
    st.zero_()
    L.check(lib.fen_rcab_fused(ctypes.byref(d), torch.cuda.current_stream().cuda_stream), "rcab")
torch.cuda.synchronize()
assert lib.fen_rcab_workspace_status(ws.ptr, B, H, W) == 0
a = st.view(256, 8, 48).cpu().numpy().astype(np.int64)
used = a[:, 0, 0] != 0
a = a[used]
t0 = a[:, :, 0][a[:, :, 0] > 0].min()
out = {"blocks": int(used.sum())}
for i in range(48):
    v = a[:, :, i].astype(np.float64)
    ok = (v > 0).any(axis=1)              # slots only some waves stamp (e.g. wave 0's gate)
    if not ok.any():
        continue
    v = np.where(v > 0, (v - t0) / 100.0, np.nan)[ok]
    out[str(i)] = [round(float(np.median(np.nanmin(v, 1))), 2), round(float(np.median(np.nanmax(v, 1))), 2)]
print(json.dumps(out))
# per-wave medians (over blocks) of chosen intervals: slot pairs (start, end)
per = {}
for nm, (s0, s1) in {"apply": (38, 39), "conv2_p3": (40, 42), "conv1_p1": (45, 46), "epi1+gate": (15, 8)}.items():
    v0, v1 = a[:, :, s0].astype(np.float64), a[:, :, s1].astype(np.float64)
    ok = (v0 > 0) & (v1 > 0)
    d = np.where(ok, (v1 - v0) / 100.0, np.nan)
    per[nm] = [round(float(np.nanmedian(d[:, w])), 2) if ok[:, w].any() else None for w in range(8)]
print(json.dumps({"per_wave_us": per}))
