"""HR-image sources for the trainer.  Each batch is {'hr': [B,3,H,W] fp32 in [0,1]}; LR is
synthesised on the GPU by the trainer, as the reference does (trainer.py:416: the dataset's
'lr' is never used).

get_dataloader() keeps the reference's signature and keywords (dataset.py:88-104,321-352, as
scripts/train.py:174-198 calls it) and applies its train-mode transform (transforms.py:173-216:
random crop -> horizontal flip -> rot90 -> colour jitter; val / test: the full image):

* uint8 images (a directory of HxWx3 uint8 .npy files, or --synthetic N seeded uint8
  images) on a GPU -> DeviceHRLoader (device_loader.py): the host draws
  each sample's parameters in the reference's np.random order and gathers the uint8 crops into
  pinned staging; flip / rot90 / colour jitter / /255 run on the GPU (csrc/augment.hip).
* otherwise (float .npy images, or no GPU) -> a torch DataLoader over NpyHRDataset /
  SyntheticHRDataset with crop / flip / rot90 on the host.  Colour jitter is defined on uint8
  images (the reference's cv2 HSV round trip) and runs only on the GPU path: with
  color_jitter_prob > 0 these sources raise instead of dropping it.

Keywords the path cannot honour raise (return_filename=True, an .h5 data root); `hue` is
accepted and, as in the reference (transforms.py:228-257 never reads it), has no effect.

Under torch.distributed every rank reads its own shard of the images -- files or synthetic
indices alike -- with DistributedSampler's counts (`rank_shard`): train drops the remainder so
every rank has n // world images (and, with drop_last batching, the same number of steps: a
rank with one more step would pair its gradient all-reduce with another rank's end-of-epoch
reduction); other modes take the exact disjoint split rank::world (validation metrics are
reduced as sums and counts, so no image may be counted twice).  Per-sample augmentation
draws are seeded by (seed, rank) so the ranks' draws are independent.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset


def _crop_flip_rot(rng: np.random.Generator, h: int, w: int, P: int, flip: float, rot: float):
    """The geometric draws of PairedTransform.__call__ (transforms.py:188-216), in its order:
    crop origin (only when the image is larger than the patch), flip, rot90 and its k."""
    top = left = 0
    if h > P and w > P:
        top = int(rng.integers(0, h - P + 1))
        left = int(rng.integers(0, w - P + 1))
    f = rng.random() < flip
    k = int(rng.integers(1, 4)) if rng.random() < rot else 0
    return top, left, f, k


def _geom(t: torch.Tensor, top: int, left: int, P: int, flip: bool, k: int) -> torch.Tensor:
    """[3,H,W] -> the P x P crop, flipped left-right, rotated k x 90 degrees counter-clockwise
    (np.rot90 on HWC = torch.rot90 over (H, W))."""
    t = t[:, top:top + P, left:left + P]
    if flip:
        t = t.flip(-1)
    if k:
        t = torch.rot90(t, k, dims=(1, 2))
    return t.contiguous()


class SyntheticHRDataset(Dataset):
    """n seeded U[0,1) images (no augmentation: the pixels are i.i.d. already)."""

    def __init__(self, n: int = 256, hr_size: int = 256, seed: int = 0):
        self.n, self.hr, self.seed = n, hr_size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return {"hr": torch.rand(3, self.hr, self.hr, generator=g)}


class NpyHRDataset(Dataset):
    """A directory of .npy files holding HxWx3 uint8 or [0,1] float arrays.  Train mode: a
    random hr_patch_size crop, flip and rot90 with the reference's probabilities; other modes
    (train=False): the full image."""

    def __init__(self, root: str, hr_patch_size: int = 256, horizontal_flip: float = 0.0, seed: int = 0,
                 random_rotate90: float = 0.0, train: bool = True, files=None):
        self.files = files if files is not None else sorted(
            os.path.join(root, f) for f in os.listdir(root) if f.endswith(".npy"))
        if not self.files:
            raise FileNotFoundError(f"no .npy images under {root}")
        self.size, self.flip, self.rot, self.train = hr_patch_size, horizontal_flip, random_rotate90, train
        self.seed, self.epoch = seed, 0

    def __len__(self):
        return len(self.files)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __getitem__(self, i):
        # one generator per (seed, epoch, sample): DataLoader workers each hold a copy of the
        # dataset, so a shared generator would repeat the same draws in every worker and epoch
        self.rng = np.random.default_rng((self.seed, self.epoch, int(i)))
        a = np.load(self.files[i], allow_pickle=False)
        t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).float()
        if a.dtype == np.uint8:
            t = t / 255.0
        if not self.train:
            return {"hr": t}
        h, w = a.shape[:2]
        if h < self.size or w < self.size:
            raise ValueError(f"{self.files[i]}: {h}x{w} is smaller than the {self.size}px patch")
        top, left, f, k = _crop_flip_rot(self.rng, h, w, self.size, self.flip, self.rot)
        return {"hr": _geom(t, top, left, self.size, f, k)}


class SyntheticU8Images:
    """n seeded HxWx3 uint8 images (the CLI's --synthetic N on the GPU data path); `index`
    (optional) maps this view's positions to image ids (a rank's shard)."""

    def __init__(self, n: int, size: int, seed: int = 0, index=None):
        self.n, self.size, self.seed = n, size, seed
        self.index = list(index) if index is not None else None

    def __len__(self):
        return len(self.index) if self.index is not None else self.n

    def __getitem__(self, i):
        i = self.index[int(i)] if self.index is not None else int(i)
        r = np.random.default_rng(self.seed * 1_000_003 + int(i))
        return r.integers(0, 256, (self.size, self.size, 3), dtype=np.uint8)


def rank_shard(n: int, train: bool, rank: Optional[int] = None, world: Optional[int] = None):
    """This rank's item indices out of n, DistributedSampler-style (no shuffle: the loaders
    shuffle within the shard): indices rank, rank + world, ...; train keeps n // world of them
    (equal step counts on every rank: a rank with one more step would pair its gradient
    all-reduce with another rank's end-of-epoch reduction).  Other modes take the exact
    disjoint split (rank::world): validation has no per-batch collective, its metrics are
    reduced as sums and counts, so unequal shard lengths are fine and no image is counted
    twice (the global val loss / PSNR / SSIM equal the one-rank values).  Without
    torch.distributed: all of range(n)."""
    if rank is None or world is None:
        if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
            return list(range(n))
        rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
    if world <= 1:
        return list(range(n))
    if not train:
        return list(range(rank, n, world))
    m = n // world
    if m == 0:
        raise ValueError(f"{n} images cannot give each of {world} ranks one")
    return [rank + world * j for j in range(m)]


def _rank() -> int:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank()
    return 0


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


def _files(data_root: str, mode: str):
    if data_root.endswith(".h5"):
        raise NotImplementedError("HDF5 data roots (dataset.py:154-175) are not read here: convert the images to "
                                  "HxWx3 uint8 .npy files")
    root = os.path.join(data_root, mode) if os.path.isdir(os.path.join(data_root, mode)) else data_root
    files = sorted(os.path.join(root, f) for f in os.listdir(root) if f.endswith(".npy"))
    if not files:
        raise FileNotFoundError(f"no .npy images under {root}")
    return [files[i] for i in rank_shard(len(files), mode == "train")]


def get_dataloader(data_root: Optional[str], mode: str = "train", batch_size: int = 16, num_workers: int = 4,
                   hr_patch_size: int = 128, horizontal_flip: float = 0.5, random_rotate90: float = 0.0,
                   color_jitter_prob: float = 0.3, brightness: float = 0.1, contrast: float = 0.1,
                   saturation: float = 0.1, hue: float = 0.05, synthetic: int = 0, seed: int = 0,
                   device=None, scale_factor: int = 4, use_cache: bool = True, cache_size: int = 100,
                   return_filename: bool = False, generate_lr_on_the_fly: bool = True):
    """The reference's get_dataloader(data_root, mode, batch_size, num_workers, **FFHQDataset
    kwargs) (dataset.py:321-352), defaults as FFHQDataset's (dataset.py:88-104).  `synthetic` N
    (the CLI's --synthetic) replaces the data directory by N seeded images; `device` (default:
    cuda when available) selects the GPU data path for uint8 sources.  scale_factor,
    use_cache / cache_size and generate_lr_on_the_fly only concern the reference's LR images,
    which training discards (LR comes from HR on the device)."""
    if return_filename:
        raise NotImplementedError("return_filename=True: batches carry only 'hr' here")
    if not synthetic and (not data_root or not os.path.isdir(data_root)):
        if data_root and data_root.endswith(".h5"):
            _files(data_root, mode)
        raise FileNotFoundError(f"data root {data_root!r} not found (synthetic=N, the CLI's --synthetic N, "
                                "trains on N seeded synthetic images instead)")
    train = mode == "train"
    dev = torch.device(device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
    jitter = color_jitter_prob if train else 0.0
    rseed = seed + 1_000_033 * _rank()          # independent augmentation draws per rank
    if synthetic:
        u8 = SyntheticU8Images(synthetic, hr_patch_size, seed + (0 if train else 1), rank_shard(synthetic, train))
    else:
        files = _files(data_root, mode)
        u8 = _NpyImages(files) if np.load(files[0], mmap_mode="r", allow_pickle=False).dtype == np.uint8 else None
    if dev.type == "cuda" and u8 is not None:
        from .device_loader import DeviceHRLoader
        P = hr_patch_size if train else int(u8[0].shape[0])
        return DeviceHRLoader(u8, batch_size, P, horizontal_flip, random_rotate90, jitter, brightness, contrast,
                              saturation, seed=rseed, shuffle=train, drop_last=train, device=dev, train=train)
    if jitter > 0:
        raise ValueError(f"color_jitter_prob={color_jitter_prob}: colour jitter (transforms.py:228-257, a uint8 HSV "
                         "round trip) runs on the GPU data path only -- uint8 images on a GPU device; set "
                         "augmentation.color_jitter.probability: 0 for this source")
    if synthetic:
        ds = SyntheticHRDataset(synthetic, hr_patch_size, seed + (0 if train else 1))
        idx = rank_shard(synthetic, train)
        if len(idx) != synthetic:
            ds = torch.utils.data.Subset(ds, idx)
    else:
        ds = NpyHRDataset(None, hr_patch_size, horizontal_flip if train else 0.0, rseed,
                          random_rotate90 if train else 0.0, train=train, files=files)
    return DataLoader(ds, batch_size=batch_size, shuffle=train, num_workers=num_workers, pin_memory=dev.type == "cuda",
                      drop_last=train)


def get_device_loader(data_root: str, mode: str = "train", batch_size: int = 16, hr_patch_size: int = 128,
                      horizontal_flip: float = 0.5, random_rotate90: float = 0.0, color_jitter_prob: float = 0.3,
                      brightness: float = 0.1, contrast: float = 0.1, saturation: float = 0.0, seed: int = 0,
                      device="cuda", **unused):
    """The GPU data path over a directory of uint8 .npy images (train: the reference's
    transform; other modes: top-left crop, no augmentation, in order)."""
    from .device_loader import DeviceHRLoader
    train = mode == "train"
    return DeviceHRLoader(_NpyImages(_files(data_root, mode)), batch_size, hr_patch_size, horizontal_flip,
                          random_rotate90, color_jitter_prob, brightness, contrast, saturation,
                          seed=seed + 1_000_033 * _rank(),
                          shuffle=train, drop_last=train, device=device, train=train)


__all__ = ["SyntheticHRDataset", "SyntheticU8Images", "NpyHRDataset", "get_dataloader", "get_device_loader",
           "rank_shard"]
