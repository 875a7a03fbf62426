"""Do host<->device copies overlap the graph replay?  Times the inference replay alone, a 25-MB
pinned D2H alone (copy stream), and both issued together, N times each (B=32, fp16)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402
from src.hip.engine import FENEngine  # noqa: E402

N = 20
eng = FENEngine(build_model("fp16"), batch=32, lr_hw=(64, 64), dtype=torch.float16, train=False, device="cuda")
hr, x = bench_batch(32, 0)
eng.x.copy_(x)
eng.capture()
cs = torch.cuda.Stream()
hout = torch.empty(eng.out.shape, dtype=eng.out.dtype).pin_memory()
dout = torch.empty_like(eng.out)


def t(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / N


def rep():
    for _ in range(N):
        eng.replay()


def d2h():
    with torch.cuda.stream(cs):
        for _ in range(N):
            hout.copy_(dout, non_blocking=True)


def both():
    d2h()
    rep()


print(f"replay {t(rep):.3f} ms  d2h {t(d2h):.3f} ms  both {t(both):.3f} ms (per iteration)")
