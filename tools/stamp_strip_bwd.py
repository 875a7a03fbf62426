"""Phase timeline of k_group_strip_bwd from the diagnostic stamp build (s_memrealtime, 100 MHz).

    make -C face-super-resolution_amd/csrc gsstamp
    FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so python tools/stamp_strip_bwd.py

Runs the bench's stage-1 training step (bf16, B=32, 64x64 -> 256x256, 6x10) a few times and
reads the last group backward's stamps from its workspace tail: every wave of every block, 136
u16 slots (10 ns ticks from the block's start).  Per RCAB step k (1..10) the slots 2+12k ..
13+12k are: step start (B_G passed), dt written (conv2^T phase 1 start), its phase 1 done, B_X
passed (dt halo built), conv2^T done, dz1 epilogue computed, B_E passed, conv1^T phase 1 start
(dz1 row written / stored), its phase 1 done, conv1^T done (incl. the dz1 halo), d epilogue +
row sums done, SE backward done (B_G reached).  Prints per-wave medians over blocks and
RCAB steps 2..9 (us)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402

NSTAMP = 136
SEG = ["dt combine", "c2T p1", "halo+B_X", "c2T p2-3", "dz1 epi", "B_E wait", "dz1 out", "c1T p1", "B_Y+c1T p2-3",
       "d epi+sums", "B_Z+SE bwd", "B_G wait"]


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
          f"group conv^T step {med(st[:, :, 14] - st[:, :, 2]):.2f} us")
    rows = []
    for k in range(2, 10):
        b = 2 + 12 * k
        seg = [st[:, :, b + i + 1] - st[:, :, b + i] for i in range(11)] + [st[:, :, b + 12] - st[:, :, b + 11]]
        rows.append(np.stack(seg))
    r = np.stack(rows)
    print("segment        " + " ".join(f"  w{w}  " for w in range(8)) + "   (median over blocks, steps 2..9; us)")
    for i, name in enumerate(SEG):
        print(f"{name:14s} " + " ".join(f"{med(r[:, i, :, w]):6.2f}" for w in range(8)))
    tot = st[:, :, 2 + 12 * 10] - st[:, :, 2 + 12 * 2]
    print(f"RCAB steps 2..9 per step: {med(tot) / 8:.2f} us")


if __name__ == "__main__":
    main()
