"""Phase timeline of k_group_strip from the diagnostic stamp build (s_memrealtime, 100 MHz).

    make -C face-super-resolution_amd/csrc gsstamp
    FEN_HIP_LIB=face-super-resolution_amd/csrc/build_stamp/libfen_hip_gsstamp.so python tools/stamp_strip.py

Runs the inference engine (fp16, B=32, 64x64) a few times and reads the last group launch's
stamps from the workspace tail: waves 0 and 1 of every block, 96 slots.  Per RCAB j the slots are
2+8j sync wait start, 3+8j sync done, 4+8j conv start (gate + combine done), 5+8j conv1 done,
6+8j conv2 start (a1 epilogue done), 7+8j conv2 before phase 3 (a1 halo fetched), 8+8j conv2
done, 9+8j signalled.  Prints medians over blocks (us) of each interval.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import bench_batch, build_model  # noqa: E402

NSTAMP = 96


def main():
    from src.hip.engine import FENEngine
    B = 32
    m = build_model("fp16")
    eng = FENEngine(m, batch=B, lr_hw=(64, 64), dtype=torch.float16, train=False, device="cuda")
    _, x = bench_batch(B, 0)
    eng.x.copy_(x)
    for _ in range(5):
        eng.forward()
    torch.cuda.synchronize()
    buf = eng.ctx._shared["pz:group_strip/32x64"]
    nblk = B * 8
    n = nblk * 2 * NSTAMP * 4
    total = int(eng.ctx.lib.fen_group_strip_work_bytes(B, 64))
    st = buf[total - n:total].cpu().view(torch.int32).numpy().astype(np.int64).reshape(nblk, 2, NSTAMP)
    st = st & 0xffffffff
    t0 = st[:, :, 0].min()
    rel = (st - t0) / 100.0          # us
    nb = 10

    def med(a):
        return float(np.median(a))

    w = rel[:, 0, :]
    print(f"launch span (wave 0): start {med(w[:, 0]):.2f} .. end {med(w[:, NSTAMP - 1]):.2f} us "
          f"(max end {w[:, NSTAMP - 1].max():.2f})")
    print(f"startup (ticket -> first conv ready): {med(w[:, 1] - w[:, 0]):.2f}")
    names = ["sync wait", "gate+combine", "conv1", "a1 epilogue", "conv2 p1-2", "conv2 p3", "epilogue+signal"]
    rows = []
    for j in range(nb):
        b = 2 + 8 * j
        if j == 0:
            vals = [0.0, med(w[:, b + 2] - w[:, 1])]
        else:
            vals = [med(w[:, b + 1] - w[:, b]), med(w[:, b + 2] - w[:, b + 1])]
        vals += [med(w[:, b + 3] - w[:, b + 2]), med(w[:, b + 4] - w[:, b + 3]), med(w[:, b + 5] - w[:, b + 4]),
                 med(w[:, b + 6] - w[:, b + 5]), med(w[:, b + 7] - w[:, b + 6])]
        rows.append(vals)
        print(f"RCAB {j}: " + "  ".join(f"{n_}={v:.2f}" for n_, v in zip(names, vals)) +
              f"  total={med(w[:, b + 7] - (w[:, b] if j else w[:, 1])):.2f}")
    r = np.array(rows[1:])
    print("mean over RCAB 1..9: " + "  ".join(f"{n_}={v:.2f}" for n_, v in zip(names, r.mean(0))))
    g = 2 + 8 * nb
    print(f"group end: sync {med(w[:, g + 1] - w[:, g]):.2f}  gate+combine {med(w[:, g + 2] - w[:, g + 1]):.2f}  "
          f"conv {med(w[:, g + 3] - w[:, g + 2]):.2f}  epilogue {med(w[:, NSTAMP - 1] - w[:, g + 3]):.2f}")
    # skew: spread of the sync-done time across the blocks of one image
    sk = []
    for j in range(1, nb):
        v = w[:, 3 + 8 * j].reshape(B, 8)
        sk.append(float(np.median(v.max(1) - v.min(1))))
    print("sync-done spread within an image (median over images): " + " ".join(f"{v:.2f}" for v in sk))
    w1 = rel[:, 1, :]
    print(f"wave 1 (gate wave) gate+combine mean: "
          f"{np.mean([med(w1[:, 4 + 8 * j] - w1[:, 3 + 8 * j]) for j in range(1, nb)]):.2f}")


if __name__ == "__main__":
    main()
