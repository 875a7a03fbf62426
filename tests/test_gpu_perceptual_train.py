"""The stage-1 training step with the perceptual term (stage1_psnr_config.yaml:40-50:
L1 x 1.0 + VGG19 conv3_4 perceptual x 1.0) on the fused engine and through the module API,
against autograd through the CPU oracle.  PARITY UNPINNED for the VGG weights (random, in
the torchvision layout; no ImageNet weights offline) -- the generator side is the config-1
golden's reference weights."""
import numpy as np
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _sd(g, prefix="p/"):
    return {k[len(prefix):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(prefix)}


@pytest.fixture(scope="module")
def g1(golden):
    return golden("g1_config1.npz")


def _vgg(seed=3):
    return {k: v for k, v in O.vgg19_init(seed=seed).items() if int(k.split(".")[1]) <= 16}


def _ref_grads(p, hr, vgg, pw):
    shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    out = O.forward(leaves, O.lr_from_hr(hr), shape, training=True)
    loss = (out - hr).abs().mean() + pw * O.perceptual_loss(vgg, out, hr, [16], None, "l1")
    loss.backward()
    return float(loss), {k: v.grad.detach() for k, v in leaves.items()}


def test_engine_step_with_perceptual_fp32(g1):
    """FENEngine(perceptual=...) forward + backward in fp32: the generator's parameter
    gradients and the total loss match autograd of L1 + perceptual through the oracle."""
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       res_scale=0.2, precision="fp32")
    m.load_state_dict(_sd(g1))
    p = {k: v.clone() for k, v in m.state_dict().items()}
    hr = torch.from_numpy(g1["hr"])
    vgg = _vgg()
    pw = 0.7
    eng = FENEngine(m, batch=2, lr_hw=(32, 32), dtype=torch.float32, train=True,
                    perceptual=dict(weight=pw, layers=["conv3_4"], params={k: v.to(DEV) for k, v in vgg.items()}))
    eng.hr.copy_(hr.to(DEV))
    eng.ctx.run()                                  # LR synthesis, forward, losses, backward
    torch.cuda.synchronize()
    ref_loss, ref_g = _ref_grads(p, hr, vgg, pw)
    assert abs(float(eng.total_loss()) - ref_loss) <= 1e-5 * ref_loss
    bad = {}
    for k, g in eng.grads.items():
        e = float((g.cpu().double() - ref_g[k].double()).norm() / max(ref_g[k].double().norm(), 1e-30))
        if not e <= 1e-4:
            bad[k] = e
    assert not bad, bad


def test_engine_step_with_perceptual_bf16_runs(g1):
    """bf16 engine step with the perceptual term: finite loss close to the fp32 one and the
    perceptual gradient moves the generator (grads differ from the L1-only step)."""
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    hr = torch.from_numpy(g1["hr"]).to(DEV)
    vgg = {k: v.to(DEV) for k, v in _vgg().items()}
    res = {}
    for tag, perc in (("l1", None), ("lp", dict(weight=1.0, layers=["conv3_4"], params=vgg))):
        m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, precision="bf16")
        m.load_state_dict(_sd(g1))
        eng = FENEngine(m, batch=2, lr_hw=(32, 32), dtype=torch.bfloat16, train=True, perceptual=perc)
        eng.hr.copy_(hr)
        eng.ctx.run()
        torch.cuda.synchronize()
        res[tag] = (float(eng.total_loss()), eng.flat_g.clone())
    _, ref_g = _ref_grads(_sd(g1), hr.cpu(), {k: v.cpu() for k, v in vgg.items()}, 1.0)
    assert np.isfinite(res["lp"][0]) and res["lp"][0] > res["l1"][0]
    g = res["lp"][1]
    flat_ref = torch.cat([ref_g[k].reshape(-1) for k in _sd(g1)]).to(DEV).float()
    cos = float((g * flat_ref).sum() / (g.norm() * flat_ref.norm()))
    assert cos >= 0.97, cos


def test_perceptual_module_autograd():
    """PerceptualLoss (module API, fp32 compute) forward value and d(pred) vs the oracle;
    a VGG19 state dict in torchvision layout is accepted via vgg_weights=."""
    from src.losses import PerceptualLoss
    torch.manual_seed(12)
    vgg = _vgg(seed=5)
    crit = PerceptualLoss(layers=["conv3_4"], criterion="l2", vgg_weights=vgg, precision="fp32").to(DEV)
    pred = torch.rand(2, 3, 32, 32)
    target = torch.rand(2, 3, 32, 32)
    pr = pred.clone().to(DEV).requires_grad_(True)
    loss = crit(pr, target.to(DEV))
    (2.0 * loss).backward()
    prc = pred.clone().requires_grad_(True)
    ref = O.perceptual_loss(vgg, prc, target, [16], None, "l2")
    (2.0 * ref).backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * float(ref)
    e = float((pr.grad.cpu() - prc.grad).norm() / prc.grad.norm())
    assert e <= 1e-4, e
    feats = crit.feature_extractor(pr.detach())
    assert feats["conv3_4"].shape == (2, 256, 8, 8)
