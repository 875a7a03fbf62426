"""Deterministic smooth synthetic HR images (test infrastructure).

PSNR parity is measured against an HR image, and U[0,1) noise makes that
meaningless (every SR output is ~8 dB from noise).  These images are sums of seeded 2-D
sinusoids (up to ~20 cycles per 256 px, below the 64-px LR's Nyquist limit of 32), Gaussian
blobs and a fine texture band (24-90 cycles, lost at LR), clipped to [0, 1] and quantised to uint8 levels like a decoded image, so
that the 4x bicubic path lands at a face-like ~30 dB.  Generated with numpy float64 from a
seed; the golden fixture (g9) stores the uint8 HR itself, so parity does not depend on
libm agreeing across machines.
"""
import numpy as np
import torch


def smooth_images_u8(B: int, H: int, W: int, seed: int) -> np.ndarray:
    """uint8 [B, 3, H, W]."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(H) / H, np.arange(W) / W, indexing="ij")
    out = np.empty((B, 3, H, W), dtype=np.uint8)
    for b in range(B):
        base = np.zeros((H, W))
        for _ in range(12):                         # shared structure (all channels)
            f = rng.uniform(0.5, 20.0)
            th = rng.uniform(0, 2 * np.pi)
            a = rng.uniform(0.02, 0.09) * (8.0 / (f + 4.0))
            base += a * np.sin(2 * np.pi * f * (np.cos(th) * xx + np.sin(th) * yy) + rng.uniform(0, 2 * np.pi))
        for _ in range(4):                          # blobs
            cy, cx = rng.uniform(0.1, 0.9, 2)
            s = rng.uniform(0.05, 0.25)
            base += rng.uniform(-0.25, 0.25) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        tex = np.zeros((H, W))                      # fine texture (hair / skin detail): lost at LR
        for _ in range(24):
            f = rng.uniform(24.0, 90.0)
            th = rng.uniform(0, 2 * np.pi)
            tex += rng.uniform(0.004, 0.012) * np.sin(2 * np.pi * f * (np.cos(th) * xx + np.sin(th) * yy)
                                                      + rng.uniform(0, 2 * np.pi))
        base += tex
        for c in range(3):
            img = 0.5 + base * rng.uniform(0.8, 1.2) + rng.uniform(-0.1, 0.1)
            for _ in range(3):                      # per-channel colour variation
                f = rng.uniform(0.5, 8.0)
                th = rng.uniform(0, 2 * np.pi)
                img += rng.uniform(0.01, 0.05) * np.sin(2 * np.pi * f * (np.cos(th) * xx + np.sin(th) * yy)
                                                        + rng.uniform(0, 2 * np.pi))
            out[b, c] = np.clip(np.rint(np.clip(img, 0.0, 1.0) * 255.0), 0, 255).astype(np.uint8)
    return out


def smooth_images(B: int, H: int, W: int, seed: int) -> torch.Tensor:
    """float32 [B, 3, H, W] in [0, 1] (uint8 levels / 255)."""
    return torch.from_numpy(smooth_images_u8(B, H, W, seed).astype(np.float32) / np.float32(255.0))
