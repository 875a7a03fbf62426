"""What the DP step's gradient exchange costs the full-chip persistent grids, on ONE GPU.

The stage-1 training step (bench config: bf16, B=32, 6x10, 64 -> 256, graph-replayed) timed:
  none      no exchange (the N=1 step);
  rccl1     a forced one-rank RCCL exchange (dp.BucketExchange(force=True) on a one-rank nccl
            group: the real RCCL kernels, on their side stream, at each bucket's mark; a
            one-rank all-reduce moves no xGMI bytes, so this is RCCL's launch + kernel floor);
  spinK     a CU-occupancy stand-in for an 8-GPU ring all-reduce: at each bucket's mark a side
            stream (forked like BucketExchange's) runs K workgroups of 256 threads that hold their
            CUs for the bucket's modelled ring time, 2 (N-1)/N bytes / BUSBW + LAT (N = 8);
  spinK_end the same stand-in issued after the backward, serial with the update (no overlap).
Implied 8-GPU weak-scaling efficiency of the step = t(none) / t(stand-in), compute unchanged.
Environment: BUSBW (GB/s, default 150), LAT (us, default 20), BLOCKS (comma list, default 16,64),
STEPS (default 20).  Needs tools/spin/libspin.so (hipcc -shared tools/spin/spin.hip)."""
import ctypes
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402
from src.hip.engine import FENEngine  # noqa: E402

STEPS = int(os.environ.get("STEPS", "20"))
BUSBW = float(os.environ.get("BUSBW", "150"))
LAT = float(os.environ.get("LAT", "20"))
BLOCKS = [int(b) for b in os.environ.get("BLOCKS", "16,64").split(",")]
NRANK = 8
spin = ctypes.CDLL(os.path.join(ROOT, "tools", "spin", "libspin.so"))
spin.spin_launch.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_void_p]


def ring_us(nbytes):
    return 2.0 * (NRANK - 1) / NRANK * nbytes / (BUSBW * 1e3) + LAT


class SpinExchange:
    """BucketExchange's stream pattern with the collective replaced by the stand-in kernel."""
    world = 1

    def __init__(self, flat, plan, blocks, at_end=False):
        self.plan, self.blocks, self.at_end = plan, blocks, at_end
        self.us = {tag: ring_us((hi - lo) * 4) for tag, lo, hi in plan}
        self.stream = torch.cuda.Stream()
        self.forked = False

    def _issue(self, tags):
        self.stream.wait_stream(torch.cuda.current_stream())
        for t in tags:
            spin.spin_launch(self.blocks, self.us[t], ctypes.c_void_p(self.stream.cuda_stream))
        self.forked = True

    def launch(self, tag):
        if not self.at_end:
            self._issue([tag])

    def wait(self):
        if self.at_end:
            self._issue([t for t, _, _ in self.plan])
        if self.forked:
            torch.cuda.current_stream().wait_stream(self.stream)
            self.forked = False


def time_engine(exchange=None):
    hr, _ = bench_batch(32, 0)
    kw = {} if exchange is None else {"exchange": exchange}
    eng = FENEngine(build_model("bf16"), batch=32, lr_hw=(64, 64), dtype=torch.bfloat16, train=True,
                    device="cuda", **kw)
    eng.hr.copy_(hr)
    eng.capture()
    for _ in range(3):
        eng.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        eng.replay()
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / STEPS
    plan = eng.exchange.plan if hasattr(eng.exchange, "plan") else None
    del eng
    torch.cuda.empty_cache()
    return ms, plan


def main():
    out = {"busbw_GBs": BUSBW, "lat_us": LAT, "nranks_modelled": NRANK, "steps": STEPS}
    t_none, _ = time_engine()
    out["none_ms"] = round(t_none, 4)
    print(f"none {t_none:.3f} ms", file=sys.stderr, flush=True)
    for K in BLOCKS:
        for at_end in (False, True):
            holder = {}

            def fac(flat, plan, K=K, at_end=at_end):
                holder["x"] = SpinExchange(flat, plan, K, at_end)
                return holder["x"]
            t, plan = time_engine(fac)
            key = f"spin{K}" + ("_end" if at_end else "")
            out[key + "_ms"] = round(t, 4)
            out[key + "_eff"] = round(t_none / t, 4)
            out["modelled_ring_us_per_step"] = round(sum(holder["x"].us.values()), 1)
            out["buckets"] = {tg: round(u, 1) for tg, u in holder["x"].us.items()}
            print(f"{key} {t:.3f} ms eff {t_none / t:.4f}", file=sys.stderr, flush=True)
    # the real RCCL kernels on a one-rank group (forced exchange)
    from src.training.dp import BucketExchange, init_rccl
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    init_rccl(torch.device("cuda", 0), rank=0, world_size=1)
    t, _ = time_engine(lambda flat, plan: BucketExchange(flat, plan, force=True))
    out["rccl1_ms"] = round(t, 4)
    out["rccl1_eff"] = round(t_none / t, 4)
    print(f"rccl1 {t:.3f} ms", file=sys.stderr, flush=True)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
