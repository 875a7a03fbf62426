"""The bench's stage-1 training step alone (bf16, B=32, 64->256, 6x10 RCAB; L1, backward, clip,
AdamW; graph-replayed; PERCEPTUAL=1 adds the VGG19 conv3_4 term), STEPS replays after 3 warm-ups: ms per step on stdout.  Run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel breakdown of one step (divide by the
launch count of STEPS + 3 + 1 replays)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402
from src.hip.engine import FENEngine  # noqa: E402

STEPS = int(os.environ.get("STEPS", "20"))
B = 32
hr, _ = bench_batch(B, 0)
spec = None
if os.environ.get("PERCEPTUAL", "0") == "1":            # the bench's train_perceptual leg
    import warnings
    from src.losses import PerceptualLoss
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec = PerceptualLoss(layers=["conv3_4"]).to("cuda").fused_spec(1.0)
eng = FENEngine(build_model("bf16"), batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda",
                perceptual=spec)
eng.hr.copy_(hr)
eng.capture()
for _ in range(3):
    eng.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(STEPS):
    eng.replay()
torch.cuda.synchronize()
print(f"train step ms {1000 * (time.perf_counter() - t0) / STEPS:.3f} loss {float(eng.total_loss() if spec else eng.loss):.5f}", flush=True)
