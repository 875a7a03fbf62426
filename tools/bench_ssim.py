"""fen_ssim (stage-2 form: fwd + gradient accumulated into an NHWC16 bf16 buffer) at B=32,
3x256x256 fp32: us per launch and GB/s against the 8 TB/s HBM roofline; mode 0 = the map and
tile sums only, 2 = the one-launch gradient form, 2ex = fen_ssim_ex's two launches."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch
from src.hip import lib as L
from src.hip.program import ptr
from src.losses.ssim import _window1d
B, C, H, W = int(os.environ.get("B", "32")), 3, 256, 256
lib = L.load()
p = torch.rand(B, C, H, W, device="cuda"); t = torch.rand(B, C, H, W, device="cuda")
buf = torch.zeros(B, H, W, 16, device="cuda", dtype=torch.bfloat16)
part = torch.empty(lib.fen_ssim_parts(B, C, H, W) * B, device="cuda")
win = _window1d(11, 1.5).cuda()
s = torch.cuda.current_stream().cuda_stream
work = torch.empty(lib.fen_ssim_work_floats(B, C, H, W), device="cuda")
res = {}
for mode in (0, 2, "2ex"):
    if mode == "2ex":      # fen_ssim_ex: the two-launch form
        f = lambda: L.check(lib.fen_ssim_ex(L.BF16, B, C, H, W, ptr(p), ptr(t), ptr(win), 11, 1e-4, 9e-4, ptr(part),
                                            ptr(buf), -1e-6, 2, ptr(work), s), "ssim_ex")
    else:
        f = lambda: L.check(lib.fen_ssim(L.BF16, B, C, H, W, ptr(p), ptr(t), ptr(win), 11, 1e-4, 9e-4, ptr(part),
                                         ptr(buf), -1e-6, mode, s), "ssim")
    for _ in range(5): f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): f()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    nbytes = 2 * B * C * H * W * 4 + (2 * B * H * W * 16 * 2 if mode else 0)
    res[f"mode{mode}_frac"] = round(nbytes / us / 1e3 / 8000.0, 4)
    res[f"mode{mode}_us"] = round(us, 2)
    res[f"mode{mode}_GBs"] = round(nbytes / us / 1e3, 1)
print(json.dumps(res))
