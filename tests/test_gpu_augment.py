"""Device HR batch preparation (csrc/augment.hip, src/data/device_loader.py) against the
oracle's restatement of the reference transform (transforms.py:173-279 + to_tensor).
Flip / rot90 / crop / scaling are bit-exact; with colour jitter the contrast mean (numpy's
float32 pairwise mean vs an exact integer sum here) may move a uint8 truncation by one level
on a few pixels.  The HSV step is PARITY UNPINNED vs cv2 (absent offline): both sides run the
restated OpenCV 8-bit algorithm."""
import numpy as np
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"

_PARAM = np.dtype([("flip", "<i4"), ("jitter", "<i4"), ("brightness", "<f4"), ("contrast", "<f4"),
                   ("saturation", "<f4"), ("rot", "<i4")])


def _run_kernel(crops, recs):
    from src.hip import lib as L
    from src.hip.program import ptr
    B, P = crops.shape[0], crops.shape[1]
    src = torch.from_numpy(crops).to(DEV)
    prm = torch.from_numpy(np.frombuffer(recs.tobytes(), dtype=np.uint8).copy()).to(DEV)
    sums = torch.empty(B, dtype=torch.int64, device=DEV)
    out = torch.empty(B, 3, P, P, device=DEV)
    lib = L.load()
    L.check(lib.fen_augment_u8(B, P, ptr(src), ptr(prm), ptr(sums), ptr(out),
                               torch.cuda.current_stream().cuda_stream), "augment")
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _compare(got, crops, recs, jitter_frac=0.005):
    for j in range(crops.shape[0]):
        r = recs[j]
        ref = O.transform_hr(crops[j], int(r["flip"]), int(r["rot"]), int(r["jitter"]), float(r["brightness"]),
                             float(r["contrast"]), float(r["saturation"]))
        d = np.abs(got[j] - ref) * 255
        if not r["jitter"]:
            assert d.max() == 0, (j, d.max())
        else:
            assert d.max() <= 1.0 + 1e-3 and (d > 1e-3).mean() <= jitter_frac, (j, d.max(), (d > 1e-3).mean())


def test_augment_kernel_vs_oracle():
    rng = np.random.default_rng(21)
    B, P = 8, 64
    crops = rng.integers(0, 256, (B, P, P, 3), dtype=np.uint8)
    crops[3] = 128                                        # flat image (HSV s = 0)
    recs = np.zeros(B, _PARAM)
    for j in range(B):
        recs[j]["flip"] = j & 1
        recs[j]["rot"] = (j // 2) % 4
        recs[j]["jitter"] = int(j >= 4)
        recs[j]["brightness"] = 0.9 + 0.05 * j
        recs[j]["contrast"] = 1.1 - 0.04 * j
        recs[j]["saturation"] = [1.0, 1.0, 0.7, 1.3, 1.0, 0.0, 2.0, 1.0][j]
    _compare(_run_kernel(crops, recs), crops, recs)


def test_device_loader_end_to_end():
    """Crop / flip / jitter draws replayed from the same seed; batches land in one reused
    output buffer (the engine's HR buffer in training)."""
    from src.data.device_loader import DeviceHRLoader
    rng = np.random.default_rng(5)
    imgs = [rng.integers(0, 256, (80 + 2 * (i % 3), 72 + 4 * (i % 2), 3), dtype=np.uint8) for i in range(10)]
    kw = dict(batch_size=4, hr_patch_size=64, horizontal_flip=0.5, random_rotate90=0.2, color_jitter_prob=0.5,
              brightness=0.1, contrast=0.1, saturation=0.2, seed=11, shuffle=False)
    ld = DeviceHRLoader(imgs, **kw)
    replay = DeviceHRLoader(imgs, **kw)                   # same RNG stream, host side only
    out = torch.empty(4, 3, 64, 64, device=DEV)
    seen = 0
    for bi, batch in enumerate(ld.batches(out=out)):
        assert batch["hr"].data_ptr() == out.data_ptr()
        torch.cuda.synchronize()
        got = batch["hr"].cpu().numpy()
        crops = np.zeros((4, 64, 64, 3), np.uint8)
        recs = np.zeros(4, _PARAM)
        for j in range(4):
            img = imgs[bi * 4 + j]
            top, left, recs[j] = replay._draw(img)
            crops[j] = img[top:top + 64, left:left + 64]
        _compare(got, crops, recs, jitter_frac=0.01)
        seen += 1
    assert seen == len(ld) == 2
