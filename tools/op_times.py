"""Per-launch times of the bench's inference program (fp16, B=32, 6x10, 64 -> 256) or, with
TRAIN=1, of its stage-1 training step (bf16; forward + backward + update programs): every
recorded C-ABI launch of the engine replayed on its own, 5 warm-ups + REPS back to back,
HIP events on the launch stream.  Repeating a launch in place is safe for timing (a training
launch that accumulates just accumulates more).  Prints name, shape, us and the achieved
TFLOP/s of the convs (dgrads / wgrads counted at their forward FLOPs)."""
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
TRAIN = os.environ.get("TRAIN", "0") == "1"


def main():
    prec = "bf16" if TRAIN else PREC
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[prec]
    eng = FENEngine(build_model(prec), batch=32, lr_hw=(64, 64), dtype=dt, train=TRAIN, device="cuda")
    hr, x = bench_batch(32, 0)
    if TRAIN:
        eng.hr.copy_(hr)
        eng.step()
    else:
        eng.x.copy_(x)
        eng.forward()
    torch.cuda.synchronize()
    ops = list(eng.ctx.ops) + (list(eng.upd.ops) if TRAIN else [])
    s = current_stream_handle()
    total = 0.0
    seen = {}
    for i, (name, fn, args) in enumerate(ops):
        if fn is None:
            continue
        desc = args[0]._obj if hasattr(args[0], "_obj") else None
        key = name
        shape, flop = "", 0.0
        if desc is not None and hasattr(desc, "cout_valid"):
            shape = f"wgrad {desc.Cin}->{desc.Cout} {desc.H}x{desc.W}"
            flop = 2.0 * desc.B * desc.H * desc.W * desc.Cin * desc.Cout * 9
        elif desc is not None and hasattr(desc, "Cin"):
            shape = f"{desc.Cin}->{desc.Cout} {desc.H}x{desc.W} epi={desc.epi}"
            flop = 2.0 * desc.B * desc.H * desc.W * desc.Cin * desc.Cout * 9
        elif desc is not None and hasattr(desc, "nb"):
            shape = f"nb={desc.nb} {desc.H}x{desc.W}"
            flop = (2 * desc.nb + 1) * 2.0 * desc.B * desc.H * desc.W * 64 * 576
        key = (name, shape)
        if key in seen and name.startswith("group_strip"):   # the 6 group launches are alike: time one
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
    print(f"sum of launches {total:.1f} us per {'training step' if TRAIN else 'forward'}", flush=True)


if __name__ == "__main__":
    main()
