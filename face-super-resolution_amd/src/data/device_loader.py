"""Pinned-host -> HBM HR batches with the reference's train-mode transform on the GPU
(reference src/data/dataset.py:241-352, transforms.py:173-279,
scripts/train.py:174-198 for the defaults).

Per batch the host only draws the per-sample parameters (crop origin, flip, rot90, colour
jitter factors -- in the reference's np.random call order) and gathers the uint8 HWC crops
into one of two pinned staging buffers; a side stream copies it to HBM asynchronously and
fen_augment_u8 (csrc/augment.hip) applies flip -> rot90 -> jitter -> /255 -> NCHW fp32,
writing straight into `out` (e.g. a training engine's HR buffer).  The copy of batch k+1
overlaps the compute stream's work on batch k; a staging buffer is refilled only after the
copy that read it has completed.  There is no CPU fallback.

Images: any sequence whose items are HxWx3 uint8 RGB arrays (FFHQ PNGs decoded elsewhere,
.npy files, ...).  256x256x3 uint8 = 196 KB per image, so B = 32 moves 6.3 MB per step.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ..hip import lib as L
from ..hip.program import ptr

_PARAM = np.dtype([("flip", "<i4"), ("jitter", "<i4"), ("brightness", "<f4"), ("contrast", "<f4"),
                   ("saturation", "<f4"), ("rot", "<i4")])


class DeviceHRLoader:
    def __init__(self, images: Sequence[np.ndarray], batch_size: int, hr_patch_size: int = 128,
                 horizontal_flip: float = 0.5, random_rotate90: float = 0.0, color_jitter_prob: float = 0.3,
                 brightness: float = 0.1, contrast: float = 0.1, saturation: float = 0.0, seed: int = 0,
                 shuffle: bool = True, drop_last: bool = True, device="cuda", train: bool = True):
        if hr_patch_size % 2:
            raise ValueError("hr_patch_size must be even")
        self.images, self.B, self.P = images, batch_size, hr_patch_size
        self.dataset = images           # the reference's `len(loader.dataset)` (scripts/train.py:200)
        self.flip_p, self.rot_p, self.color_p = horizontal_flip, random_rotate90, color_jitter_prob
        self.bri, self.con, self.sat = brightness, contrast, saturation
        self.rng = np.random.default_rng(seed)
        self.shuffle, self.drop_last, self.train = shuffle, drop_last, train
        self.device = torch.device(device)
        B, P = batch_size, hr_patch_size
        self.lib = L.load()
        self.stage = [torch.empty(B, P, P, 3, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.pstage = [torch.empty(B * _PARAM.itemsize, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.dev = [torch.empty(B, P, P, 3, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.dparams = [torch.empty(B * _PARAM.itemsize, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.sums = torch.empty(B, dtype=torch.int64, device=self.device)
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.copied = [None, None]          # event: the copy out of stage[k] finished

    def __len__(self):
        n = len(self.images)
        return n // self.B if self.drop_last else (n + self.B - 1) // self.B

    def _draw(self, img: np.ndarray):
        """One sample's parameters, in the reference's np.random order (transforms.py:188-226)."""
        h, w = img.shape[:2]
        P, r = self.P, self.rng
        top = left = 0
        if not self.train:
            return 0, 0, np.zeros(1, _PARAM)[0]
        if h > P and w > P:
            top = int(r.integers(0, h - P + 1))
            left = int(r.integers(0, w - P + 1))
        rec = np.zeros(1, _PARAM)[0]
        rec["flip"] = int(r.random() < self.flip_p)
        if r.random() < self.rot_p:
            rec["rot"] = int(r.integers(1, 4))
        if r.random() < self.color_p:
            rec["jitter"] = 1
            rec["brightness"] = r.uniform(1.0 - self.bri, 1.0 + self.bri)
            rec["contrast"] = r.uniform(1.0 - self.con, 1.0 + self.con)
            rec["saturation"] = r.uniform(1.0 - self.sat, 1.0 + self.sat)
        return top, left, rec

    def _fill(self, k: int, idx) -> None:
        if self.copied[k] is not None:
            self.copied[k].synchronize()    # the copy that last read stage[k] is done
        stage = self.stage[k].numpy()
        recs = np.zeros(self.B, _PARAM)
        for j, i in enumerate(idx):
            img = self.images[int(i)]
            if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
                raise ValueError("images must be HxWx3 uint8")
            if img.shape[0] < self.P or img.shape[1] < self.P:
                raise ValueError(f"image {int(i)} is smaller than the {self.P}px patch")
            top, left, recs[j] = self._draw(img)
            stage[j] = img[top:top + self.P, left:left + self.P]
        self.pstage[k].numpy()[:] = np.frombuffer(recs.tobytes(), dtype=np.uint8)

    def batches(self, out: Optional[torch.Tensor] = None):
        """Yields NCHW fp32 [B,3,P,P] batches on the device (`out` reused when given)."""
        n = len(self.images)
        order = self.rng.permutation(n) if self.shuffle else np.arange(n)
        nb = len(self)
        cur = torch.cuda.current_stream(self.device)
        for bi in range(nb):
            k = bi & 1
            idx = order[bi * self.B:(bi + 1) * self.B]
            if len(idx) < self.B:
                idx = np.concatenate([idx, order[: self.B - len(idx)]])
            self._fill(k, idx)
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_stream(cur)       # dev[k] no longer read by batch k-2's kernel
                self.dev[k].copy_(self.stage[k], non_blocking=True)
                self.dparams[k].copy_(self.pstage[k], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            self.copied[k] = ev
            cur.wait_event(ev)
            dst = out if out is not None else torch.empty(self.B, 3, self.P, self.P, device=self.device)
            L.check(self.lib.fen_augment_u8(self.B, self.P, ptr(self.dev[k]), ptr(self.dparams[k]), ptr(self.sums),
                                            ptr(dst), cur.cuda_stream), "augment")
            yield {"hr": dst}

    def __iter__(self):
        return self.batches()


__all__ = ["DeviceHRLoader"]
