"""The bench's stage-1 training step run EAGERLY (no graph) REPS times, for rocprofv3 --pmc
passes over its two strip kernels: the training form of fen_group_strip (a ResidualGroup's
forward writing the backward's operands) and fen_group_strip_bwd (its backward).  bf16, B=32,
64x64 -> 256x256, 6x10 RCAB, L1.  Prints each kernel's algorithmic bytes per launch (every tensor
read or written once; 16.8 MB per [32,64,64,64] bf16 activation):
  training forward: x in; y, x_last and per RCAB z1, a1, t (+ x_j for j >= 1) out; 21 filters
  backward:         dy, per RCAB z1 and t in; dx, per RCAB dt and dz1 out; 21 filters
(SE vectors and partials, < 0.1 MB, left out).
Usage: rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python tools/pmc_train.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402
from src.hip.engine import FENEngine  # noqa: E402

REPS = int(os.environ.get("REPS", "6"))
B, H, W, C, NB = 32, 64, 64, 64, 10
hr, _ = bench_batch(B, 0)
eng = FENEngine(build_model("bf16"), batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda")
eng.hr.copy_(hr)
for _ in range(REPS):
    eng.step()
torch.cuda.synchronize()
act = B * H * W * C * 2
filt = (2 * NB + 1) * 9 * C * C * 2
print("algorithmic_bytes_fwd_train", (1 + 2 + 3 * NB + (NB - 1)) * act + filt)
print("algorithmic_bytes_bwd", (1 + 2 * NB + 1 + 2 * NB) * act + filt)
