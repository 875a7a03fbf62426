"""Split the D256 gradient error of test_gpu_bench_legs.py::test_gan_leg_d256_matches_cpu_replay:
the discriminator's own kernels vs the fake image it is given.  The reference is torch float64
on CPU (real = g10's HR, fake = the float64 oracle generator's output).  Each fp32 candidate
(torch CPU, HIP) is run on (a) the same fake image rounded to fp32 and (b) its own fp32
generator's fake image; per parameter the relative L2 error against float64 is printed."""
import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import numpy as np, torch, torch.nn as nn
from oracle import fen_oracle as O
from src.models import FaceEnhanceNet, VGGStyleDiscriminator
from src.training.trainer import bicubic_down4

g1 = dict(np.load(os.path.join(ROOT, "tests/golden/g1_config1.npz")))
g10 = dict(np.load(os.path.join(ROOT, "tests/golden/g10_train64.npz")))
hr = torch.from_numpy(g10["hr_u8"].astype(np.float32) / np.float32(255.0))
sd = {k[2:]: torch.from_numpy(v) for k, v in g1.items() if k.startswith("p/")}
shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
torch.manual_seed(3)
D0 = copy.deepcopy(VGGStyleDiscriminator(input_size=256).state_dict())
bce = nn.BCEWithLogitsLoss()
one, zero = torch.ones(2, 1), torch.zeros(2, 1)
with torch.no_grad():
    sr64 = O.forward({k: v.double() for k, v in sd.items()}, O.lr_from_hr(hr.double()), shape, training=True)
    sr32 = O.forward(sd, O.lr_from_hr(hr), shape, training=True)
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       res_scale=0.2, precision="fp32")
    m.load_state_dict(sd)
    m = m.cuda().train()          # train mode: no clamp, as the trainer's D step sees it
    srh = m(bicubic_down4(hr.cuda())).cpu()
print("fake image vs float64: oracle fp32 %.2e, HIP fp32 %.2e (max abs)" %
      (float((sr32.double() - sr64).abs().max()), float((srh.double() - sr64).abs().max())))


def dstep(dtype, device, fake, prec=None, branch="both"):
    D = VGGStyleDiscriminator(input_size=256, **({"precision": prec} if prec else {}))
    D.load_state_dict(D0)
    D = D.to(device=device, dtype=dtype if device == "cpu" else torch.float32).train()
    f = (lambda t: D.classifier(D.features(t))) if device == "cpu" else D
    h, fk = hr.to(device, dtype), fake.to(device, dtype)
    o, z = one.to(device, dtype), zero.to(device, dtype)
    if branch == "both":
        loss = (bce(f(h), o) + bce(f(fk), z)) / 2
    elif branch == "real":
        loss = bce(f(h), o) / 2
    else:
        loss = bce(f(fk), z) / 2
    loss.backward()
    return {k: p.grad.detach().cpu().double() for k, p in D.named_parameters()}


ref = dstep(torch.float64, "cpu", sr64)
ref_r = dstep(torch.float64, "cpu", sr64, branch="real")
ref_f = dstep(torch.float64, "cpu", sr64, branch="fake")
hip_r = dstep(torch.float32, "cuda", sr64.float(), "fp32", branch="real")
hip_f = dstep(torch.float32, "cuda", sr64.float(), "fp32", branch="fake")
t32_r = dstep(torch.float32, "cpu", sr64.float(), branch="real")
print("%-34s%12s%14s%14s%14s%14s" % ("param", "kappa", "hip real", "hip fake", "torch real", "torch fake"))
for k in ref:
    kap = float((ref_r[k].norm() + ref_f[k].norm()) / max(float(ref[k].norm()), 1e-30))
    rel = lambda g, r: float((g[k] - r[k]).norm() / max(float(r[k].norm()), 1e-30))  # noqa: E731
    print("%-34s%12.1f%14.2e%14.2e%14.2e%14.2e" % (k, kap, rel(hip_r, ref_r), rel(hip_f, ref_f), rel(t32_r, ref_r),
                                                 float("nan")))
runs = {
    "torch32 same fake": dstep(torch.float32, "cpu", sr64.float()),
    "torch32 own fake": dstep(torch.float32, "cpu", sr32),
    "hip32 same fake": dstep(torch.float32, "cuda", sr64.float(), "fp32"),
    "hip32 own fake": dstep(torch.float32, "cuda", srh, "fp32"),
    "hip32 oracle-fp32 fake": dstep(torch.float32, "cuda", sr32, "fp32"),
}
keys = list(ref)
print("%-34s" % "param" + "".join("%24s" % n for n in runs))
for k in keys:
    r = ref[k]
    print("%-34s" % k + "".join("%24.2e" % float((g[k] - r).norm() / max(float(r.norm()), 1e-30))
                                 for g in runs.values()))

print("branch-scaled error |g - g64| / (|g64 real| + |g64 fake|):")
print("%-34s" % "param" + "".join("%24s" % n for n in runs))
for k in keys:
    sc = float(ref_r[k].norm() + ref_f[k].norm())
    print("%-34s" % k + "".join("%24.2e" % float((g[k] - ref[k]).norm() / sc) for g in runs.values()))
