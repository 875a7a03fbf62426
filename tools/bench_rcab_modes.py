"""A/B of the RCAB chain implementations inside the B=32 inference engine (same box, same
process): FEN_RCAB modes 'deferred' / 'perop' -- whole-forward ms and the dominant launch's
average duration."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
from src.hip import net  # noqa: E402
from src.hip.engine import FENEngine  # noqa: E402

prec = os.environ.get("PREC", "fp16")
hr, x = bench.bench_batch(32, 0)
for mode in os.environ.get("MODES", "deferred,perop").split(","):
    net.RCAB_MODE = mode
    for rep in range(2):
        m = bench.build_model(prec)
        e = FENEngine(m, batch=32, lr_hw=(64, 64), dtype=bench.DTYPES[prec], train=False)
        e.x.copy_(x)
        e.capture()
        t = bench.timed(e.replay, 50, 10, 1)
        km, kl, kf = bench.time_dominant_kernel(e)
        print(f"{mode:9s} {prec}: {1000 * t / 50:.4f} ms/step  {32 * 50 / t:.0f} img/s   dominant {km * 1000:.2f} us "
              f"({kf / km / 1e9:.0f} TFLOP/s, frac {kf / km / 1e9 / 2500:.3f})  [{kl[:40]}]", flush=True)
        del e, m
        torch.cuda.empty_cache()
