"""The stage-2 SSIM launch alone (fen_ssim, grad_mode 2: map + tile sums + gradient added to the
NHWC16 bf16 dL/dsr), B=32, 3 x 256 x 256, REPS back-to-back launches, for rocprofv3 passes and
A/B timing (HIP events, printed as us per launch).  MODE=ex: fen_ssim_ex's two launches (the
map kernel writing a / b / c to a workspace, then k_ssim_g2)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402

from src.hip import lib as L  # noqa: E402
from src.losses.ssim import _window1d  # noqa: E402

REPS = int(os.environ.get("REPS", "50"))
B, C, H, W = 32, 3, 256, 256
lib = L.load()
g = torch.Generator().manual_seed(0)
pred = torch.rand(B, C, H, W, generator=g).cuda()
target = (pred.cpu() + 0.1 * torch.randn(B, C, H, W, generator=g)).clamp(0, 1).cuda()
win = _window1d(11, 1.5).cuda()
part = torch.zeros(int(lib.fen_ssim_parts(B, C, H, W)) * B, device="cuda")
grad = torch.zeros(B, H, W, 16, dtype=torch.bfloat16, device="cuda")
s = torch.cuda.current_stream().cuda_stream
EX = os.environ.get("MODE", "") == "ex"
work = torch.empty(int(lib.fen_ssim_work_floats(B, C, H, W)), device="cuda") if EX else None


def launch():
    if EX:
        L.check(lib.fen_ssim_ex(1, B, C, H, W, pred.data_ptr(), target.data_ptr(), win.data_ptr(), 11, 1e-4, 9e-4,
                                part.data_ptr(), grad.data_ptr(), -1e-6, 2, work.data_ptr(), s), "ssim_ex")
        return
    L.check(lib.fen_ssim(1, B, C, H, W, pred.data_ptr(), target.data_ptr(), win.data_ptr(), 11, 1e-4, 9e-4,
                         part.data_ptr(), grad.data_ptr(), -1e-6, 2, s), "ssim")


for _ in range(3):
    launch()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    launch()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / REPS
nbytes = 2 * B * C * H * W * 4 + 2 * B * H * W * 16 * 2
print(f"ssim us {us:.2f}  frac {nbytes / us / 1e3 / 8000:.4f}  sum {float(part.sum()):.6e}")
