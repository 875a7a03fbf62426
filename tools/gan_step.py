"""bench.py's stage-3 GAN iteration alone (B=16, module autograd path), STEPS iterations after
2 warm-ups: ms per iteration on stdout.  Under rocprofv3 --kernel-trace --stats the summed
kernel time per iteration shows how much of it is GPU work vs host launch overhead."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

r = bench.time_gan_step(int(os.environ.get("STEPS", "5")))
print("gan ms per iteration", r["ms_per_step"], flush=True)
