"""Minimal HR-image sources for the trainer (the reference's FFHQ/HDF5 loader, src/data, is
outside this build's scope).  Each item is {'hr': [3,H,W] fp32 in
[0,1]}; LR is synthesised on the GPU by the trainer, as the reference does (trainer.py:416).

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
    if synthetic or not data_root or not os.path.isdir(data_root):
        ds = SyntheticHRDataset(synthetic or 256, hr_patch_size, seed + (0 if mode == "train" else 1))
    else:
        ds = NpyHRDataset(os.path.join(data_root, mode) if os.path.isdir(os.path.join(data_root, mode)) else data_root,
                          hr_patch_size, horizontal_flip if mode == "train" else 0.0, seed)
    sampler = None
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        sampler = torch.utils.data.DistributedSampler(ds, shuffle=(mode == "train"), drop_last=True)
    return DataLoader(ds, batch_size=batch_size, shuffle=(mode == "train" and sampler is None), sampler=sampler,
                      num_workers=num_workers, pin_memory=True, drop_last=(mode == "train"))


__all__ = ["SyntheticHRDataset", "NpyHRDataset", "get_dataloader"]
