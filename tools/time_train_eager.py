"""Time the stage-1 training step eager (engine.step(), the N>1 path: no graph) against the
graph replay, at world 1; with --allreduce, also a bare async all_reduce of the flat arena
under the initialised process group (torchrun)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd")); sys.path.insert(0, ROOT)
import torch
import torch.distributed as dist
from bench import build_model

world = int(os.environ.get("WORLD_SIZE", "1"))
if world > 1:
    dist.init_process_group(os.environ.get("FEN_BENCH_BACKEND", "gloo"))
torch.cuda.set_device(0)
from src.hip.engine import FENEngine
B = 32
eng = FENEngine(build_model("bf16"), batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda")
eng.hr.copy_(torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1)).cuda())


def t(fn, n=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / n


print("eager step ms", round(t(eng.step), 3), "world", world, flush=True)


def phases(n=5):
    """host-side time of each phase of engine.step(): enqueueing the recorded program (marks
    included), joining the buckets, enqueueing the update, then draining the stream."""
    acc = [0.0] * 4
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.ctx.run()
        t1 = time.perf_counter()
        eng.exchange.wait()
        t2 = time.perf_counter()
        eng.upd.run()
        eng.Wt.pack()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        for i, d in enumerate((t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            acc[i] += 1000 * d / n
    print("phases ms: enqueue %.3f  wait %.3f  update %.3f  drain %.3f  (ops %d)"
          % (*acc, len(eng.ctx.ops)), flush=True)


phases()
if world == 1:
    eng.capture()
    print("graph replay ms", round(t(eng.replay), 3), flush=True)
else:
    from src.training import dp as DP
    orig = DP.BucketExchange.launch
    DP.BucketExchange.launch = lambda self, tag: None
    print("eager step, exchange off, ms", round(t(eng.step), 3), flush=True)
    DP.BucketExchange.launch = orig
    import torch.distributed as dist_
    flat = eng.flat_g
    print("bare all_reduce of arena ms", round(t(lambda: dist.all_reduce(flat)), 3), flat.numel(), flush=True)
    dist.destroy_process_group()
