"""Per-launch times of the bench's inference program (fp16, B=32, 6x10, 64 -> 256): every
recorded C-ABI launch of the engine replayed on its own, 5 warm-ups + REPS back to back,
HIP events on the launch stream.  Inference launches are pure (no accumulation), so repeating
one in place is safe.  Prints name, shape, us and the achieved TFLOP/s of the convs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402
from src.hip.engine import FENEngine  # noqa: E402
from src.hip.program import current_stream_handle  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
PREC = os.environ.get("PREC", "fp16")


def main():
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[PREC]
    eng = FENEngine(build_model(PREC), batch=32, lr_hw=(64, 64), dtype=dt, train=False, device="cuda")
    _, x = bench_batch(32, 0)
    eng.x.copy_(x)
    eng.forward()
    torch.cuda.synchronize()
    s = current_stream_handle()
    total = 0.0
    seen = {}
    for i, (name, fn, args) in enumerate(eng.ctx.ops):
        if fn is None:
            continue
        desc = args[0]._obj if hasattr(args[0], "_obj") else None
        key = name
        shape, flop = "", 0.0
        if desc is not None and hasattr(desc, "Cin"):
            shape = f"{desc.Cin}->{desc.Cout} {desc.H}x{desc.W} epi={desc.epi}"
            flop = 2.0 * desc.B * desc.H * desc.W * desc.Cin * desc.Cout * 9
        elif desc is not None and hasattr(desc, "nb"):
            shape = f"nb={desc.nb} {desc.H}x{desc.W}"
            flop = (2 * desc.nb + 1) * 2.0 * desc.B * desc.H * desc.W * 64 * 576
        key = (name, shape)
        if key in seen and name == "group_strip":      # the 6 group launches are alike: time one
            total += seen[key]
            continue
        for _ in range(5):
            fn(*args, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            fn(*args, s)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / REPS
        seen[key] = us
        total += us
        tf = f"{flop / us / 1e6:8.1f} TFLOP/s" if flop else ""
        print(f"{i:3d} {name:18s} {shape:28s} {us:9.2f} us {tf}", flush=True)
    print(f"sum of launches {total:.1f} us per forward", flush=True)


if __name__ == "__main__":
    main()
