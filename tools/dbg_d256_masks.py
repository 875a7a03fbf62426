"""Why the D256 discriminator gradients looked ill-conditioned: torch fp32
on CPU vs float64, on the same inputs (g10's HR batch and the fp32 oracle generator's fake),
(a) plainly and (b) with float64 forced onto the fp32 run's LeakyReLU branches
(oracle.disc_forward masks).  Prints per layer how many LeakyReLU elements sit on the other
branch in float64, and per parameter the relative L2 gradient error of (a) and (b).
CPU only:  python tools/dbg_d256_masks.py > profiles/r06_d256_masks.txt"""
import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import numpy as np, torch, torch.nn as nn
from oracle import fen_oracle as O
from src.models import VGGStyleDiscriminator

g1 = dict(np.load(os.path.join(ROOT, "tests/golden/g1_config1.npz")))
g10 = dict(np.load(os.path.join(ROOT, "tests/golden/g10_train64.npz")))
hr = torch.from_numpy(g10["hr_u8"].astype(np.float32) / np.float32(255.0))
sd = {k[2:]: torch.from_numpy(v) for k, v in g1.items() if k.startswith("p/")}
with torch.no_grad():
    fake = O.forward(sd, O.lr_from_hr(hr), O.NetShape(64, 1, 2, 4, 4, 0.2), training=True)
torch.manual_seed(3)                                   # the D256 test's discriminator
P = {k: v for k, v in VGGStyleDiscriminator(input_size=256).state_dict().items()
     if "running" not in k and "num_batches" not in k}
bce = nn.BCEWithLogitsLoss()


def grads(dt, masks=(None, None), rec=(None, None)):
    L = {k: v.to(dt).clone().requires_grad_(True) for k, v in P.items()}
    n = hr.shape[0]
    ((bce(O.disc_forward(L, hr.to(dt), masks[0], rec[0]), torch.ones(n, 1, dtype=dt))
      + bce(O.disc_forward(L, fake.to(dt), masks[1], rec[1]), torch.zeros(n, 1, dtype=dt))) / 2).backward()
    return {k: v.grad.double() for k, v in L.items()}


m32 = ([], [])
g32 = grads(torch.float32, rec=m32)
m64 = ([], [])
g64 = grads(torch.float64, rec=m64)
g64m = grads(torch.float64, masks=m32)
print("LeakyReLU elements whose branch differs between fp32 and float64 (real / fake):")
for i in range(11):
    name = f"features.{i}" if i < 10 else "classifier.2"
    print(f"  {name:14s} {int((m32[0][i] != m64[0][i]).sum()):3d} / {int((m32[1][i] != m64[1][i]).sum()):3d}"
          f"  of {m32[0][i].numel()}")
print(f"{'param':28s} {'fp32 vs float64':>16s} {'fp32 vs float64 on fp32 branches':>34s}")
for k in g32:
    e1 = float((g32[k] - g64[k]).norm() / g64[k].norm())
    e2 = float((g32[k] - g64m[k]).norm() / g64m[k].norm())
    print(f"{k:28s} {e1:16.2e} {e2:34.2e}")
