"""SSIM golden vectors (test infrastructure; runs ONLY in the survey container).

Loads the reference's src/losses/ssim_loss.py by file path (the package __init__ needs
torchvision, which is absent; the module itself imports only torch) and records
g7_ssim.npz:
  pred, target            B=2, C=3, 48x40 in [0,1] (non-square on purpose)
  ssim_mean, ssim_per_img ssim(size_average=True / False), window 11, sigma 1.5
  loss, dpred             SSIMLoss()(pred, target) = 1 - ssim and its gradient w.r.t. pred
  ssim_same               ssim(pred, pred) (= 1)
  msssim                  ms_ssim on a 2x3x64x64 pair (pred64, target64)
  window                  the 11x11 Gaussian window (channel 0)
Nothing from the reference travels except these numbers.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ssim.py
"""
import importlib.util
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = os.environ.get("FEN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

spec = importlib.util.spec_from_file_location("ref_ssim", os.path.join(REF, "src", "losses", "ssim_loss.py"))
ref = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ref)

g = torch.Generator().manual_seed(77)
pred = torch.rand(2, 3, 48, 40, generator=g)
# a target correlated with pred, so SSIM is neither ~0 nor ~1
target = (0.7 * pred + 0.3 * torch.rand(2, 3, 48, 40, generator=g)).clamp(0, 1)
pr = pred.clone().requires_grad_(True)
loss = ref.SSIMLoss()(pr, target)
loss.backward()
p64 = torch.rand(2, 3, 64, 64, generator=g)
t64 = (0.8 * p64 + 0.2 * torch.rand(2, 3, 64, 64, generator=g)).clamp(0, 1)
out = dict(
    pred=pred.numpy(), target=target.numpy(),
    ssim_mean=np.float64(ref.ssim(pred, target).item()),
    ssim_per_img=ref.ssim(pred, target, size_average=False).numpy(),
    loss=np.float64(loss.item()), dpred=pr.grad.numpy(),
    ssim_same=np.float64(ref.ssim(pred, pred).item()),
    pred64=p64.numpy(), target64=t64.numpy(), msssim=np.float64(ref.ms_ssim(p64, t64).item()),
    window=ref.create_gaussian_window(11, 1.5, 1)[0, 0].numpy(),
)
np.savez_compressed(os.path.join(OUT, "g7_ssim.npz"), **out)
print({k: (v.shape if hasattr(v, "shape") else v) for k, v in out.items()})
