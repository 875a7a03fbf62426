"""Isolate discriminator-gradient differences: D(hr) only, and the D step (real + fake)."""
import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import numpy as np, torch, torch.nn as nn
from oracle import fen_oracle as O
from src.models import VGGStyleDiscriminator
g1 = dict(np.load(os.path.join(ROOT, "tests/golden/g1_config1.npz")))
hr = torch.from_numpy(g1["hr"])
torch.manual_seed(3)
Dc = VGGStyleDiscriminator(input_size=128)
D0 = copy.deepcopy(Dc.state_dict())
Dc = Dc.double()
bce = nn.BCEWithLogitsLoss()
def rels(Dg):
    out = {}
    dcp = dict(Dc.named_parameters())
    for k, p in Dg.named_parameters():
        r = dcp[k].grad.double()
        out[k] = float((p.grad.cpu().double() - r).norm() / r.norm())
    return out
for case in ("real_only", "real_sum", "real_bce"):
    Dc.zero_grad()
    Dg = VGGStyleDiscriminator(input_size=128, precision="fp32"); Dg.load_state_dict(D0); Dg = Dg.cuda().train()
    Dc.load_state_dict({k: v.double() if v.dtype.is_floating_point else v for k, v in D0.items()})
    Dc.train()
    oc = Dc.classifier(Dc.features(hr.double()))
    og = Dg(hr.cuda())
    if case == "real_only":
        (oc * torch.tensor([[0.3], [-0.7]], dtype=torch.float64)).sum().backward()
        (og * torch.tensor([[0.3], [-0.7]], device="cuda")).sum().backward()
    elif case == "real_sum":
        oc.sum().backward(); og.sum().backward()
    else:
        bce(oc, torch.ones(2, 1, dtype=torch.float64)).backward(); bce(og, torch.ones(2, 1, device="cuda")).backward()
    r = rels(Dg)
    worst = sorted(r.items(), key=lambda kv: -kv[1])[:4]
    print(case, "out", (og.detach().cpu().double() - oc.detach()).abs().max().item(), worst)

# the D step on identical inputs (hr, and the f64 generator output as fake), then the G-step
# contribution at the updated parameters
shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
sd = {k[2:]: torch.from_numpy(v).double() for k, v in g1.items() if k.startswith("p/")}
with torch.no_grad():
    sr_d = O.forward(sd, O.lr_from_hr(hr.double()), shape, training=True)
Dc.load_state_dict({k: v.double() if v.dtype.is_floating_point else v for k, v in D0.items()}); Dc.train(); Dc.zero_grad()
Dg = VGGStyleDiscriminator(input_size=128, precision="fp32"); Dg.load_state_dict(D0); Dg = Dg.cuda().train()
one, zero = torch.ones(2, 1, dtype=torch.float64), torch.zeros(2, 1, dtype=torch.float64)
((bce(Dc.classifier(Dc.features(hr.double())), one) + bce(Dc.classifier(Dc.features(sr_d)), zero)) / 2).backward()
((bce(Dg(hr.cuda()), one.float().cuda()) + bce(Dg(sr_d.float().cuda()), zero.float().cuda())) / 2).backward()
r = rels(Dg)
print("D step", sorted(r.items(), key=lambda kv: -kv[1])[:4])

# generator gradient of the adversarial term alone, and D's input gradient, vs float64
from src.models import FaceEnhanceNet
m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                   res_scale=0.2, precision="fp32")
m.load_state_dict({k: v.float() for k, v in sd.items()})
m = m.cuda().train()
Dg = VGGStyleDiscriminator(input_size=128, precision="fp32"); Dg.load_state_dict(D0); Dg = Dg.cuda().train()
Dc.load_state_dict({k: v.double() if v.dtype.is_floating_point else v for k, v in D0.items()}); Dc.train(); Dc.zero_grad()
from src.training.trainer import bicubic_down4
lr_g = bicubic_down4(hr.cuda())
sr = m(lr_g)
srr = sr.detach().clone().requires_grad_(True)
bce(Dg(srr), torch.ones(2, 1, device="cuda")).backward()
leaves = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
src = O.forward(leaves, O.lr_from_hr(hr.double()), shape, training=True)
src_l = src.detach().clone().requires_grad_(True)
bce(Dc.classifier(Dc.features(src_l)), one).backward()
print("dD/dsr rel", float((srr.grad.cpu().double() - src_l.grad).norm() / src_l.grad.norm()))
sr.backward(srr.grad)
src.backward(src_l.grad)
errs = {k: float((p.grad.cpu().double() - leaves[k].grad).norm() / leaves[k].grad.norm()) for k, p in m.named_parameters()}
print("G adv grads", sorted(errs.items(), key=lambda kv: -kv[1])[:5])
