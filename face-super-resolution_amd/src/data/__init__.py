"""HR-image sources for the trainer.  Each batch is {'hr': [B,3,H,W] fp32 in [0,1]}; LR is
synthesised on the GPU by the trainer, as the reference does (trainer.py:416).

* DeviceHRLoader (device_loader.py): uint8 HWC images -> pinned
  staging -> async copy -> the reference's train-mode transform (crop, flip, rot90, colour
  jitter, /255) on the GPU (csrc/augment.hip).  get_device_loader() builds one over a
  directory of HxWx3 uint8 .npy files with the reference's augmentation defaults
  (scripts/train.py:174-198).
* SyntheticHRDataset: seeded U[0,1) images (benchmarks, smoke runs).
* NpyHRDataset: a directory of .npy files holding HxWx3 uint8 or [0,1] float arrays.
get_dataloader() keeps the reference's signature (dataset.py:321-352) and, under
torch.distributed, shards with a DistributedSampler.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset


class SyntheticHRDataset(Dataset):
    def __init__(self, n: int = 256, hr_size: int = 256, seed: int = 0):
        self.n, self.hr, self.seed = n, hr_size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return {"hr": torch.rand(3, self.hr, self.hr, generator=g)}


class NpyHRDataset(Dataset):
    def __init__(self, root: str, hr_patch_size: int = 256, horizontal_flip: float = 0.0, seed: int = 0):
        self.files = sorted(os.path.join(root, f) for f in os.listdir(root) if f.endswith(".npy"))
        if not self.files:
            raise FileNotFoundError(f"no .npy images under {root}")
        self.size, self.flip = hr_patch_size, horizontal_flip
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return len(self.files)

    def __getitem__(self, i):
        a = np.load(self.files[i], allow_pickle=False)
        t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).float()
        if a.dtype == np.uint8:
            t = t / 255.0
        t = t[:, : self.size, : self.size]
        if self.flip and self.rng.random() < self.flip:
            t = t.flip(-1)
        return {"hr": t}


def get_dataloader(data_root: Optional[str], mode: str = "train", batch_size: int = 16, num_workers: int = 4,
                   hr_patch_size: int = 256, horizontal_flip: float = 0.5, synthetic: int = 0, seed: int = 0,
                   **unused) -> DataLoader:
    if not synthetic and (not data_root or not os.path.isdir(data_root)):
        raise FileNotFoundError(f"data root {data_root!r} not found (synthetic=N, the CLI's --synthetic N, "
                                "trains on N seeded synthetic images instead)")
    if synthetic:
        ds = SyntheticHRDataset(synthetic, hr_patch_size, seed + (0 if mode == "train" else 1))
    else:
        ds = NpyHRDataset(os.path.join(data_root, mode) if os.path.isdir(os.path.join(data_root, mode)) else data_root,
                          hr_patch_size, horizontal_flip if mode == "train" else 0.0, seed)
    sampler = None
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        sampler = torch.utils.data.DistributedSampler(ds, shuffle=(mode == "train"), drop_last=True)
    return DataLoader(ds, batch_size=batch_size, shuffle=(mode == "train" and sampler is None), sampler=sampler,
                      num_workers=num_workers, pin_memory=True, drop_last=(mode == "train"))


class _NpyImages:
    """Lazy uint8 HxWx3 images from .npy files (np.load, allow_pickle=False)."""

    def __init__(self, files):
        self.files = files

    def __len__(self):
        return len(self.files)

    def __getitem__(self, i):
        a = np.load(self.files[i], allow_pickle=False)
        if a.dtype != np.uint8:
            raise ValueError(f"{self.files[i]}: the device pipeline takes uint8 images")
        return a


def get_device_loader(data_root: str, mode: str = "train", batch_size: int = 16, hr_patch_size: int = 128,
                      horizontal_flip: float = 0.5, random_rotate90: float = 0.0, color_jitter_prob: float = 0.3,
                      brightness: float = 0.1, contrast: float = 0.1, saturation: float = 0.0, seed: int = 0,
                      device="cuda", **unused):
    """The GPU data path over a directory of uint8 .npy images (train: the reference's
    transform; other modes: centre-free top-left crop, no augmentation, in order)."""
    from .device_loader import DeviceHRLoader
    root = os.path.join(data_root, mode) if os.path.isdir(os.path.join(data_root, mode)) else data_root
    files = sorted(os.path.join(root, f) for f in os.listdir(root) if f.endswith(".npy"))
    if not files:
        raise FileNotFoundError(f"no .npy images under {root}")
    train = mode == "train"
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        r, w = torch.distributed.get_rank(), torch.distributed.get_world_size()
        files = files[r::w]
    return DeviceHRLoader(_NpyImages(files), batch_size, hr_patch_size, horizontal_flip, random_rotate90,
                          color_jitter_prob, brightness, contrast, saturation, seed=seed, shuffle=train,
                          drop_last=train, device=device, train=train)


__all__ = ["SyntheticHRDataset", "NpyHRDataset", "get_dataloader", "get_device_loader"]
