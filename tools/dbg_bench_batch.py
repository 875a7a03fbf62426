"""Check bench.bench_batch: the GPU bicubic /4 of the smooth HR batch vs the oracle's."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
from oracle import fen_oracle as O  # noqa: E402
hr, x = bench.bench_batch(4, 0)
torch.cuda.synchronize()
ref = O.lr_from_hr(hr.cpu())
print("hr", hr.shape, float(hr.mean()), "x", x.shape, float(x.mean()), float(x.std()), "ref", float(ref.mean()),
      "maxdiff", float((x.cpu() - ref).abs().max()))
