"""One stage-3 GAN iteration of the Trainer (reference trainer.py:424-485) on the HIP path --
generator through FaceEnhanceNet's HIP autograd, discriminator through the HIP
VGGStyleDiscriminator -- against a plain-torch CPU replay of the same iteration (oracle
generator, the discriminator's own nn.Sequential tree run natively on the CPU, torch AdamW
for D, clip + AdamW for G), the HIP path in fp32 against the replay in float64.  Compared: the loss, the discriminator's
gradients and running statistics, both networks' parameters after their updates."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_gan_step_matches_cpu_replay(golden):
    from src.models import FaceEnhanceNet, GANLoss, VGGStyleDiscriminator
    from src.training import Trainer, TrainerConfig
    g1 = golden("g1_config1.npz")
    sd = {k[2:]: torch.from_numpy(v) for k, v in g1.items() if k.startswith("p/")}
    hr = torch.from_numpy(g1["hr"])                              # [2,3,128,128]
    # the CPU replay runs in float64: the yardstick for the fp32 HIP path
    sd64 = {k: v.double() for k, v in sd.items()}
    hr64 = hr.double()
    # lr_d below fp32 resolution of D's weights: AdamW's first step moves every element by
    # ~lr sign(g), and a near-zero gradient whose sign differs between the two runs would
    # then feed a different D into the G step (measured: 3% on conv_first.weight's gradient
    # at lr_d = 2e-4; the adversarial gradient alone matches float64 to 0.3%, tools/dbg_gan.py)
    gw, lr_g, lr_d, clip = 0.05, 1e-4, 1e-7, 0.5
    # --- CPU replay ---
    torch.manual_seed(3)
    Dc = VGGStyleDiscriminator(input_size=128)
    D0 = copy.deepcopy(Dc.state_dict())
    Dc = Dc.double()
    dfwd = lambda t: Dc.classifier(Dc.features(t))               # noqa: E731  (native torch on CPU)
    bce = nn.BCEWithLogitsLoss()
    shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
    lr = O.lr_from_hr(hr64)
    optd = torch.optim.AdamW(Dc.parameters(), lr=lr_d, weight_decay=0.0)
    Dc.train()
    optd.zero_grad()
    with torch.no_grad():
        sr_d = O.forward(sd64, lr, shape, training=True)
    one, zero = torch.ones(2, 1, dtype=torch.float64), torch.zeros(2, 1, dtype=torch.float64)
    d_loss = (bce(dfwd(hr64), one) + bce(dfwd(sr_d), zero)) / 2
    d_loss.backward()
    ref_dgrad = {k: p.grad.detach().clone() for k, p in Dc.named_parameters()}
    optd.step()
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in sd64.items()}
    sr = O.forward(leaves, lr, shape, training=True)
    g_loss = (sr - hr64).abs().mean() + gw * bce(dfwd(sr), one)
    g_loss.backward()
    grads = {k: v.grad.detach() for k, v in leaves.items()}
    c = O.clip_coef(grads, clip)
    grads = {k: t * c for k, t in grads.items()}
    newp = {k: t.detach().clone() for k, t in sd64.items()}
    O.adamw_step(newp, grads, {k: torch.zeros_like(t) for k, t in newp.items()},
                 {k: torch.zeros_like(t) for k, t in newp.items()}, 1, lr_g, wd=0.0)
    # --- HIP trainer ---
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       res_scale=0.2, precision="fp32")
    m.load_state_dict(sd)
    Dg = VGGStyleDiscriminator(input_size=128, precision="fp32")
    Dg.load_state_dict(D0)
    cfg = TrainerConfig(learning_rate=lr_g, weight_decay=0.0, gradient_clip=clip, gan_weight=gw,
                        d_learning_rate=lr_d, d_weight_decay=0.0, use_wandb=False, scheduler_type="none",
                        checkpoint_dir="/tmp/fen_gan_ckpt")
    tr = Trainer(m, [], None, loss_fn=nn.L1Loss(), config=cfg, discriminator=Dg, gan_loss=GANLoss("vanilla"))
    snap, orig_step = {}, tr.optimizer_d.step

    def step_with_snapshot(*a, **kw):                   # the D-step gradients, before the update
        for k, p in Dg.named_parameters():
            snap[k] = p.grad.detach().clone()
        return orig_step(*a, **kw)

    tr.optimizer_d.step = step_with_snapshot
    loss = tr._gan_step(hr.to(DEV))
    torch.cuda.synchronize()
    assert abs(float(loss) - float(g_loss.detach())) <= 1e-4 * float(g_loss.detach())
    # D: its gradients at its update -- the real and fake branches cancel heavily in the first
    # conv's weight gradient (measured 4e-4 rel with identical inputs, tools/dbg_gan.py; 2.6e-3
    # when the fake image is the fp32 generator's output, ~1e-6 from the float64 one) -- and
    # running statistics (3 forwards);
    # parameters after AdamW's first step move by ~lr * sign(g), so an element whose gradient is
    # ~0 may flip under rounding: bound the flipped fraction and the size of any difference
    for k in snap:
        ref = ref_dgrad[k].double()
        e = float((snap[k].cpu().double() - ref).norm() / max(ref.norm(), 1e-30))
        assert e <= 5e-3, (k, e)
    for k, v in Dg.state_dict().items():
        ref = Dc.state_dict()[k]
        if "running" in k:
            # the third update runs at the AdamW-updated weights (the sign-flip caveat below)
            assert float((v.cpu().double() - ref.double()).abs().max()) <= 2e-4 * max(1.0, float(ref.abs().max())), k
        elif not ref.dtype.is_floating_point:
            assert int(v) == int(ref) == 3, k
        else:
            d = (v.cpu().double() - ref.double()).abs()
            assert float(d.max()) <= 2.1 * lr_d and float((d > 1e-6).double().mean()) <= 1e-2, k
    # G: its gradient (content + gan_weight x adversarial through D) before clipping, then the
    # parameters after clip + AdamW (the same first-step sign-flip caveat as D)
    raw = {k: v.grad.detach() for k, v in leaves.items()}
    for k, p in m.named_parameters():
        e = float((p.grad.cpu().double() - raw[k]).norm() / max(raw[k].norm(), 1e-30))
        assert e <= 5e-3, (k, e)
    for k, v in m.state_dict().items():
        d = (v.cpu().double() - newp[k].double()).abs()
        assert float(d.max()) <= 2.1 * lr_g and float((d > 2e-5).double().mean()) <= 5e-2, (k, float(d.max()))
