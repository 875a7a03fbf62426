"""Phase timeline of k_group_strip_bwd from the diagnostic stamp build (s_memrealtime, 100 MHz).

    make -C face-super-resolution_amd/csrc gsstamp
    FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so python tools/stamp_strip_bwd.py

Runs the bench's stage-1 training step (bf16, B=32, 64x64 -> 256x256, 6x10) a few times and
reads the last group backward's stamps from its workspace tail: every wave of every block, 104
u16 slots (10 ns ticks from the block's start).  Per RCAB step k (1..10) the slots 2+9k ..
10+9k are: step start (B_Z passed), conv2^T phase 1 start (dt' written; wave 1: + the SE
backward and the kh = 1 correction), its phase 1 done, B_X passed (dt' halo built), conv2^T done
(+ dt saved), B_T passed (the kh = 0 / 2 correction terms), dz1 epilogue done and stored,
conv1^T phase 1 done, conv1^T done (B_Y, incl. the dz1 halo); the next step's start closes the
d epilogue + row sums + B_Z.  Prints per-wave medians over blocks and RCAB steps 2..9 (us)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402

NSTAMP = 104
SEG = ["combine", "c2T p1", "halo+B_X", "SE(w1)+c2T p2-3", "corr(w1)+B_T", "dz1+dt out+B_E", "c1T p1",
       "B_Y+c1T p2-3", "d epi+sums+B_Z"]


def main():
    from src.hip.engine import FENEngine
    B = 32
    eng = FENEngine(build_model("bf16"), batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda")
    hr, _ = bench_batch(B, 0)
    eng.hr.copy_(hr)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    buf = eng.ctx._shared["pz:group_strip_bwd/32x64"]
    nblk = B * 8
    n = nblk * 8 * NSTAMP * 2
    total = int(eng.ctx.lib.fen_group_strip_bwd_work_bytes(B, 64))
    st = buf[total - n:total].cpu().numpy().view(np.uint16).astype(np.float64).reshape(nblk, 8, NSTAMP) / 100.0
    med = np.median
    print(f"launch end {med(st[:, 0, NSTAMP - 1]):.2f} us (max {st[:, 0, NSTAMP - 1].max():.2f}); "
          f"group conv^T step {med(st[:, :, 11] - st[:, :, 2]):.2f} us")
    rows = []
    for k in range(2, 10):
        b = 2 + 9 * k
        seg = [st[:, :, b + i + 1] - st[:, :, b + i] for i in range(9)]
        rows.append(np.stack(seg))
    r = np.stack(rows)
    print("segment        " + " ".join(f"  w{w}  " for w in range(8)) + "   (median over blocks, steps 2..9; us)")
    for i, name in enumerate(SEG):
        print(f"{name:14s} " + " ".join(f"{med(r[:, i, :, w]):6.2f}" for w in range(8)))
    tot = st[:, :, 2 + 9 * 10] - st[:, :, 2 + 9 * 2]
    print(f"RCAB steps 2..9 per step: {med(tot) / 8:.2f} us")


if __name__ == "__main__":
    main()
