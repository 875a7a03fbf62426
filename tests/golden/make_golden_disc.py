"""Discriminator golden vectors (test infrastructure; runs ONLY in the survey container).

Loads the reference's src/models/discriminator.py by file path (it imports only torch) and
records g8_disc.npz for VGGStyleDiscriminator(input_size=64) (classifier 2048 -> 1024 -> 1):
  stat_names/stat_sum/stat_sumsq  init statistics after torch.manual_seed(0)
  (the weights are the seed-0 init itself: the statistics pin it, so they are not stored)
  x, r                            input B=4 3x64x64 in [0,1], random output weights R
  out_train                       train-mode output (batch statistics)
  gx                              gradient of sum(out_train * R) w.r.t. the input
  g/<param>                       that gradient w.r.t. parameters of <= 70k elements
  gn/<param>, gp/<param>          every parameter gradient's norm and its dot with seeded
                                  noise (torch.Generator().manual_seed(7), randn of its shape)
  bn_after/<key>                  running_mean / running_var after that forward
  out_eval                        eval-mode output afterwards (running statistics)
  gan_vanilla_real/fake, gan_lsgan_real  GANLoss values on out_train
  f64/...                         the same train-mode forward / gradients with the reference run
                                  in float64 (the yardstick for fp32 rounding)
Nothing from the reference travels except these numbers.
Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_disc.py
"""
import importlib.util
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = os.environ.get("FEN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
spec = importlib.util.spec_from_file_location("ref_disc", os.path.join(REF, "src", "models", "discriminator.py"))
ref = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ref)

torch.manual_seed(0)
d = ref.VGGStyleDiscriminator(input_size=64)
sd = d.state_dict()
out = {"stat_names": np.array(list(sd.keys())),
       "stat_sum": np.array([float(v.double().sum()) for v in sd.values()]),
       "stat_sumsq": np.array([float((v.double() ** 2).sum()) for v in sd.values()])}
g = torch.Generator().manual_seed(5)
x = torch.rand(4, 3, 64, 64, generator=g)
r = torch.randn(4, 1, generator=g)
xr = x.clone().requires_grad_(True)
d.train()
o = d(xr)
(o * r).sum().backward()
out.update(x=x.numpy(), r=r.numpy(), out_train=o.detach().numpy(), gx=xr.grad.numpy())
for k, p in d.named_parameters():
    gr = p.grad.double()
    if p.numel() <= 70000:
        out["g/" + k] = p.grad.numpy()
    out["gn/" + k] = np.float64(gr.norm())
    out["gp/" + k] = np.float64((gr * torch.randn(p.shape, generator=torch.Generator().manual_seed(7)).double()).sum())
for k, v in d.state_dict().items():
    if "running" in k:
        out["bn_after/" + k] = v.numpy()
d.eval()
with torch.no_grad():
    out["out_eval"] = d(x).numpy()
# the reference in float64 from the same initial state
torch.manual_seed(0)
d64 = ref.VGGStyleDiscriminator(input_size=64).double().train()
x64 = x.double().requires_grad_(True)
o64 = d64(x64)
(o64 * r.double()).sum().backward()
out["f64/out_train"] = o64.detach().numpy()
out["f64/gx"] = x64.grad.numpy()
for k, p in d64.named_parameters():
    gr = p.grad
    out["f64/gn/" + k] = np.float64(gr.norm())
    out["f64/gp/" + k] = np.float64((gr * torch.randn(p.shape, generator=torch.Generator().manual_seed(7)).double()).sum())
gl = ref.GANLoss("vanilla")
out["gan_vanilla_real"] = np.float64(gl(o.detach(), True))
out["gan_vanilla_fake"] = np.float64(gl(o.detach(), False))
out["gan_lsgan_real"] = np.float64(ref.GANLoss("lsgan")(o.detach(), True))
np.savez_compressed(os.path.join(OUT, "g8_disc.npz"), **out)
print(len(out), "arrays", o.detach().numpy().ravel())
