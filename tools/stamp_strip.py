"""Phase timeline of k_group_strip from its diagnostic stamp build (s_memrealtime, 100 MHz).

    make -C face-super-resolution_amd/csrc gsstamp
    FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so python tools/stamp_strip.py

Runs the inference engine (fp16, B=32, 64x64) a few times and reads the last group launch's
stamps from the workspace tail: every wave of every block, 100 u16 slots (10 ns ticks from the
block's start).  Per RCAB j the slots 2+9j .. 10+9j are: step start (gate barrier passed), conv1
phase 1 start (combine done), phase 1 done, conv1 done, conv2 phase 1 start (a1 epilogue done),
its phase 1 done, phase 2 start (pool partial published), conv2 done, gate barrier reached.
Prints the medians over blocks and RCABs 1..9 of each segment, per wave (us).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402

NSTAMP = 100
SEG = ["combine", "conv1 p1", "halo+c1 p2-3", "a1 epilogue", "conv2 p1", "pool partial", "conv2 p2-3",
       "epi2+gate", "B_G wait"]


def main():
    from src.hip.engine import FENEngine
    B = 32
    m = build_model("fp16")
    eng = FENEngine(m, batch=B, lr_hw=(64, 64), dtype=torch.float16, train=False, device="cuda")
    _, x = bench_batch(B, 0)
    eng.x.copy_(x)
    for _ in range(int(os.environ.get("REPS", "1500"))):   # >= 2 s back to back: the clock under load
        eng.forward()
    torch.cuda.synchronize()
    buf = eng.ctx._shared["pz:group_strip/32x64"]
    nblk = B * 8
    n = nblk * 8 * NSTAMP * 2
    total = int(eng.ctx.lib.fen_group_strip_work_bytes(B, 64))
    st = buf[total - n:total].cpu().numpy().view(np.uint16).astype(np.float64).reshape(nblk, 8, NSTAMP) / 100.0
    med = np.median
    print(f"launch: first conv ready {med(st[:, :, 1]):.2f} us; end {med(st[:, 0, NSTAMP - 1]):.2f} us "
          f"(max {st[:, 0, NSTAMP - 1].max():.2f})")
    ghz = st[:, 1, NSTAMP - 1] * 100 * 16 / np.maximum(st[:, 0, NSTAMP - 1] * 1000, 1)
    print(f"in-kernel shader clock (s_memtime / s_memrealtime over each block's life): median {med(ghz):.3f} GHz")
    rows = []
    for j in range(1, 10):
        b = 2 + 9 * j
        nxt = 2 + 9 * (j + 1)
        seg = [st[:, :, b + k + 1] - st[:, :, b + k] for k in range(8)] + [st[:, :, nxt] - st[:, :, b + 8]]
        rows.append(np.stack(seg))                      # [9 seg][blocks][8 waves]
    r = np.stack(rows)                                  # [rcab][seg][blocks][waves]
    print("segment        " + " ".join(f"  w{w}  " for w in range(8)) + "   (median over blocks, RCABs 1..9; us)")
    for k, name in enumerate(SEG):
        print(f"{name:14s} " + " ".join(f"{med(r[:, k, :, w]):6.2f}" for w in range(8)))
    tot = st[:, :, 2 + 9 * 10] - st[:, :, 2 + 9 * 1]
    print(f"RCAB 1..9 total per RCAB: {med(tot) / 9:.2f} us")
    g = 2 + 9 * 10
    print(f"group end: combine {med(st[:, :, g + 1] - st[:, :, g]):.2f}  conv {med(st[:, :, g + 3] - st[:, :, g + 1]):.2f}  "
          f"out {med(st[:, 0, NSTAMP - 1] - st[:, 0, g + 3]):.2f}")


if __name__ == "__main__":
    main()
