"""BASELINE configs[4] alone (the bench's stress_c128_x8 leg: 128 ch, 10x20 RCAB, x8, 128x128 ->
1024x1024, B=4, fp16 inference, graph-replayed): ms per step on stdout.  Run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel breakdown."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)

from bench import time_stress  # noqa: E402

print(time_stress(steps=int(os.environ.get("STEPS", "3"))), flush=True)
