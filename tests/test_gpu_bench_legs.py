"""Parity of the bench's stage-1 perceptual and stage-3 GAN legs at the bench's own sizes.

bench.py's `train_perceptual` leg is the stage-1 recipe (stage1_psnr_config.yaml:40-50: L1 x 1 +
VGG19 conv3_4 perceptual x 1) on the full network (6x10 RCAB, 64x64 -> 256x256) at B=32, and
`train_gan` one stage-3 Trainer iteration (trainer.py:424-485: L1 x 0.01 + perceptual x 1 +
adversarial x 0.005 through VGGStyleDiscriminator(input_size=256)) at B=16.  Checked here:

  * perceptual, fp32: the engine step's loss and generator gradients against autograd through
    the CPU oracle (reference weights of tests/golden/g10_train64.npz, its 2 smooth HR images,
    VGG19 to conv3_4 at 256x256), at B=2 and at B=32 (the 2 images tiled 16x: the mean loss's
    gradient is the B=2 one) -- and at B=32 every copy's dL/dsr is bit-identical to its
    original's (a batch-position-dependent kernel would show here);
  * perceptual, bf16 at B=32 (the bench's dtype): loss and gradient against the same fp32
    oracle at the bf16 bounds of test_gpu_perceptual_train.py, copies bit-identical;
  * GAN, fp32, D input 256, B=2: one iteration against a float64 CPU replay (the reference
    discriminator tree run natively on the CPU, oracle generator, oracle perceptual term), as
    test_gpu_gan_step.py does at 128;
  * GAN, bf16, the bench's exact configuration (6x10 generator, D input 256, B=16): the
    captured iteration (Trainer._gan_iteration) bit-identical to the eager one over 5
    iterations.

VGG19 weights: random (torchvision layout, oracle.vgg19_init) -- PARITY UNPINNED for the VGG
weights themselves (no torchvision / ImageNet weights offline); the generator side is pinned by
the reference's own golden."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import fen_oracle as O
from src_models_seed import full_ctor, seeded_model

pytestmark = pytest.mark.gpu
DEV = "cuda"
FULL = O.NetShape(64, 6, 10, 4, 4, 0.2)


@pytest.fixture(scope="module")
def g10(golden):
    return golden("g10_train64.npz")


def _hr(g):
    return torch.from_numpy(g["hr_u8"].astype(np.float32) / np.float32(255.0))    # [2,3,256,256]


def _vgg(seed=3):
    return {k: v for k, v in O.vgg19_init(seed=seed).items() if int(k.split(".")[1]) <= 16}


@pytest.fixture(scope="module")
def perc_ref(g10):
    """Oracle autograd (fp32 CPU) of L1 + 1.0 x perceptual(conv3_4) at the north-star shape."""
    m = seeded_model(full_ctor("fp32"), g10)
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    hr, vgg = _hr(g10), _vgg()
    leaves = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    out = O.forward(leaves, O.lr_from_hr(hr), FULL, training=True)
    loss = (out - hr).abs().mean() + O.perceptual_loss(vgg, out, hr, [16], None, "l1")
    loss.backward()
    return float(loss.detach()), {k: v.grad.detach() for k, v in leaves.items()}


def _perc_engine(g10, B, dtype):
    from src.hip.engine import FENEngine
    m = seeded_model(full_ctor("fp32" if dtype == torch.float32 else "bf16"), g10)
    vgg = {k: v.to(DEV) for k, v in _vgg().items()}
    eng = FENEngine(m, batch=B, lr_hw=(64, 64), dtype=dtype, train=True, clip=0.5, lr=1e-4,
                    perceptual=dict(weight=1.0, layers=["conv3_4"], params=vgg))
    eng.hr.copy_(_hr(g10).repeat(B // 2, 1, 1, 1).to(DEV))
    eng.ctx.run()                       # LR synthesis, forward, L1 + perceptual, backward
    eng.exchange.wait()
    torch.cuda.synchronize()
    return m, eng


def _copies_identical(eng, B):
    d = eng.saved_tail["dout"]          # dL/dsr, NHWC16 (L1 + perceptual gradients)
    for i in range(2, B):
        assert torch.equal(d[i], d[i % 2]), i


@pytest.mark.parametrize("B", [2, 32])
def test_perceptual_leg_fp32(g10, perc_ref, B):
    ref_loss, ref_g = perc_ref
    m, eng = _perc_engine(g10, B, torch.float32)
    loss = float(eng.total_loss())
    assert abs(loss - ref_loss) <= 1e-5 * ref_loss, (loss, ref_loss)
    worst, bad = 0.0, {}
    num = den = 0.0
    for k, g in eng.grads.items():
        a, r = g.detach().cpu().double(), ref_g[k].double()
        e = float((a - r).norm() / max(float(r.norm()), 1e-30))
        num += float((a - r).norm()) ** 2
        den += float(r.norm()) ** 2
        worst = max(worst, e)
        if not e <= 5e-4:
            bad[k] = e
    whole = (num / den) ** 0.5
    print(f"B={B}: loss {loss:.6f} (ref {ref_loss:.6f}); gradient rel whole {whole:.2e}, worst tensor {worst:.2e}")
    assert whole <= 1e-4, whole
    assert not bad, dict(list(bad.items())[:10])
    if B > 2:
        _copies_identical(eng, B)


def test_perceptual_leg_bf16_batch32(g10, perc_ref):
    """The bench's configuration.  bf16 bounds as test_gpu_perceptual_train.py's: loss within
    3e-2 relative, the whole-network gradient's cosine to the fp32 oracle's >= 0.97 (L1's sign
    gradient flips wherever |sr - hr| is below bf16 resolution)."""
    ref_loss, ref_g = perc_ref
    m, eng = _perc_engine(g10, 32, torch.bfloat16)
    loss = float(eng.total_loss())
    assert np.isfinite(loss) and abs(loss - ref_loss) <= 3e-2 * ref_loss, (loss, ref_loss)
    g = torch.cat([eng.grads[k].detach().reshape(-1).double().cpu() for k in ref_g])
    r = torch.cat([ref_g[k].reshape(-1).double() for k in ref_g])
    cos = float((g * r).sum() / (g.norm() * r.norm()))
    print(f"bf16 B=32: loss {loss:.6f} (ref {ref_loss:.6f}), gradient cosine {cos:.5f}")
    assert cos >= 0.97, cos
    _copies_identical(eng, 32)


class _Content(nn.Module):
    """The bench's stage-3 content loss, 0.01 x L1 + 1.0 x perceptual(conv3_4) (stage3 config)."""

    def __init__(self, vgg, precision):
        super().__init__()
        from src.losses import PerceptualLoss
        self.perc = PerceptualLoss(layers=["conv3_4"], vgg_weights=vgg, precision=precision)

    def forward(self, sr, hr):
        return 0.01 * (sr - hr).abs().mean() + self.perc(sr, hr)


def _hip_d_masks(d0, x):
    """The LeakyReLU branches the HIP discriminator (fp32, train-mode BN, weights d0) takes on x:
    each feature block's output > 0 (_DFeatures keeps block j's output as block j+1's input; the
    last block's is its result) and the classifier's hidden pre-activation > 0, computed as the
    module's forward computes it."""
    from src.models import VGGStyleDiscriminator
    from src.models.discriminator import _DFeatures
    D = VGGStyleDiscriminator(input_size=256, precision="fp32")
    D.load_state_dict(d0)
    D = D.to(DEV).train()
    feats = _DFeatures.apply(x.to(DEV), D, 1, *D._feature_params())
    masks = [(s["a_in"] > 0).permute(0, 3, 1, 2).cpu() for s in feats.grad_fn.saved_blocks] + [(feats > 0).cpu()]
    masks.append((D.head_preactivation(feats.flatten(1)) > 0).cpu())
    return masks


def test_gan_leg_d256_matches_cpu_replay(golden, g10):
    """test_gpu_gan_step.py's float64 replay at the bench's discriminator size (input 256) and
    content loss; generator config-1 (the reference's golden weights) at 64 -> 256."""
    from src.models import FaceEnhanceNet, GANLoss, VGGStyleDiscriminator
    from src.training import Trainer, TrainerConfig
    g1 = golden("g1_config1.npz")
    sd = {k[2:]: torch.from_numpy(v) for k, v in g1.items() if k.startswith("p/")}
    hr = _hr(g10)
    vgg = _vgg()
    sd64, hr64 = {k: v.double() for k, v in sd.items()}, hr.double()
    vgg64 = {k: v.double() for k, v in vgg.items()}
    # lr_d below D's fp32 weight resolution: see test_gpu_gan_step.py (AdamW's first step ~ lr sign(g))
    gw, lr_g, lr_d, clip = 0.005, 1e-4, 1e-7, 0.5
    torch.manual_seed(3)
    Dc = VGGStyleDiscriminator(input_size=256)
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
    # yardstick for the D gradient: the float64 replay of the D step on the
    # SAME inputs the HIP D step sees (the real batch and the HIP generator's fake) with the HIP
    # discriminator's own LeakyReLU branches (oracle.disc_forward with masks) -- the derivative of
    # the piecewise-linear network on the piece the HIP run is on.  Without the masks, the 1-4
    # elements per layer whose pre-activation lies within fp32 rounding of 0 take the other branch
    # in float64, and each flip moves every gradient below it by a finite step (2e-3 .. 1e-2
    # relative, torch's own fp32 included: profiles/r06_d256_masks.txt); with them, torch fp32 is
    # within 2.5e-5 of float64 on every parameter, and the HIP discriminator is held to 1e-4.
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       res_scale=0.2, precision="fp32")
    m.load_state_dict(sd)
    from src.training.trainer import bicubic_down4
    with torch.no_grad():
        sr_d_hip = m.to(DEV).train()(bicubic_down4(hr.to(DEV))).cpu()   # what tr._gan_step's D sees
    masks_r, masks_f = _hip_d_masks(D0, hr), _hip_d_masks(D0, sr_d_hip)
    p64 = {k: v.double().requires_grad_(True) for k, v in D0.items() if "running" not in k and "num_batches" not in k}
    own_r, own_f = [], []
    ((bce(O.disc_forward(p64, hr64, masks=masks_r, record=own_r), one)
      + bce(O.disc_forward(p64, sr_d_hip.double(), masks=masks_f, record=own_f), zero)) / 2).backward()
    ref_dgrad_m = {k: v.grad.detach().clone() for k, v in p64.items()}
    flips = [int((a != b).sum()) + int((c != d).sum()) for a, b, c, d in zip(masks_r, own_r, masks_f, own_f)]
    print(f"LeakyReLU elements on the other branch in float64 (HIP masks imposed), per layer: {flips}")
    optd.step()
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in sd64.items()}
    sr = O.forward(leaves, lr, shape, training=True)
    content = 0.01 * (sr - hr64).abs().mean() + O.perceptual_loss(vgg64, sr, hr64, [16], None, "l1")
    g_loss = content + gw * bce(dfwd(sr), one)
    g_loss.backward()
    raw = {k: v.grad.detach() for k, v in leaves.items()}
    c = O.clip_coef(raw, clip)
    newp = {k: t.detach().clone() for k, t in sd64.items()}
    O.adamw_step(newp, {k: t * c for k, t in raw.items()}, {k: torch.zeros_like(t) for k, t in newp.items()},
                 {k: torch.zeros_like(t) for k, t in newp.items()}, 1, lr_g, wd=0.0)
    # --- HIP trainer (fp32) ---
    m.load_state_dict(sd)
    Dg = VGGStyleDiscriminator(input_size=256, precision="fp32")
    Dg.load_state_dict(D0)
    cfg = TrainerConfig(learning_rate=lr_g, weight_decay=0.0, gradient_clip=clip, gan_weight=gw,
                        d_learning_rate=lr_d, d_weight_decay=0.0, use_wandb=False, scheduler_type="none",
                        checkpoint_dir="/tmp/fen_gan256_ckpt")
    tr = Trainer(m, [], None, loss_fn=_Content(vgg, "fp32").to(DEV), config=cfg, discriminator=Dg,
                 gan_loss=GANLoss("vanilla"))
    snap, orig_step = {}, tr.optimizer_d.step

    def step_with_snapshot(*a, **kw):
        for k, p in Dg.named_parameters():
            snap[k] = p.grad.detach().clone()
        return orig_step(*a, **kw)

    tr.optimizer_d.step = step_with_snapshot
    loss = tr._gan_step(hr.to(DEV))
    torch.cuda.synchronize()
    print(f"GAN D256: loss {float(loss):.7f} vs float64 replay {float(g_loss.detach()):.7f}")
    assert abs(float(loss) - float(g_loss.detach())) <= 1e-4 * float(g_loss.detach())
    worst = 0.0
    for k in snap:
        ref = ref_dgrad_m[k]
        e = float((snap[k].cpu().double() - ref).norm() / max(ref.norm(), 1e-30))
        e0 = float((snap[k].cpu().double() - ref_dgrad[k]).norm() / max(ref_dgrad[k].norm(), 1e-30))
        worst = max(worst, e)
        print(f"  D {k}: rel {e:.2e} vs the mask-matched float64 replay ({e0:.2e} vs the plain one on the float64 fake)")
        assert e <= 1e-4, (k, e)
    print(f"D gradients: worst rel {worst:.2e} (bound 1e-4 on every parameter)")
    for k, v in Dg.state_dict().items():
        ref = Dc.state_dict()[k]
        if "running" in k:
            assert float((v.cpu().double() - ref.double()).abs().max()) <= 2e-4 * max(1.0, float(ref.abs().max())), k
        elif not ref.dtype.is_floating_point:
            assert int(v) == int(ref) == 3, k
        else:
            d = (v.cpu().double() - ref.double()).abs()
            assert float(d.max()) <= 2.1 * lr_d and float((d > 1e-6).double().mean()) <= 1e-2, k
    worst = 0.0
    for k, p in m.named_parameters():
        e = float((p.grad.cpu().double() - raw[k]).norm() / max(raw[k].norm(), 1e-30))
        worst = max(worst, e)
        assert e <= 5e-3, (k, e)
    print(f"G gradients: worst rel {worst:.2e}")
    for k, v in m.state_dict().items():
        d = (v.cpu().double() - newp[k].double()).abs()
        assert float(d.max()) <= 2.1 * lr_g and float((d > 2e-5).double().mean()) <= 5e-2, (k, float(d.max()))


def _bench_gan_trainer(capture, tmp, precision="bf16"):
    """bench.py:time_gan_step's configuration (B=16 below), capture on or off."""
    import warnings
    from src.losses import create_loss_function
    from src.models import FaceEnhanceNet, GANLoss, VGGStyleDiscriminator
    from src.training import Trainer, TrainerConfig
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        loss_fn = create_loss_function(l1_weight=0.01, perceptual_weight=1.0, ssim_weight=0.0,
                                       perceptual_layers=["conv3_4"])
    torch.manual_seed(42)
    G = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, precision=precision)
    torch.manual_seed(7)
    D = VGGStyleDiscriminator(input_size=256, precision=precision)
    cfg = TrainerConfig(learning_rate=1e-4, weight_decay=0.0, gradient_clip=0.5, gan_weight=0.005,
                        d_learning_rate=1e-4, use_wandb=False, scheduler_type="none", checkpoint_dir=str(tmp),
                        capture_gan_step=capture)
    tr = Trainer(G, [], None, loss_fn=loss_fn, config=cfg, discriminator=D, gan_loss=GANLoss("vanilla"))
    for g in tr.optimizer_d.param_groups:      # the same AdamW form on both sides
        g["capturable"] = True
    return tr


def test_gan_leg_bench_config_capture_matches_eager(tmp_path):
    eager, cap = _bench_gan_trainer(False, tmp_path / "e"), _bench_gan_trainer(True, tmp_path / "c")
    gen = torch.Generator().manual_seed(99)
    base = torch.rand(2, 3, 256, 256, generator=gen)
    for i in range(5):
        hr = (base.roll(i, dims=0) * (1.0 - 0.05 * i)).repeat(8, 1, 1, 1).to(DEV)     # B = 16
        le = float(eager._gan_iteration(hr))
        lc = float(cap._gan_iteration(hr))
        assert np.isfinite(le) and le == lc, (i, le, lc)
        assert torch.equal(eager.model._fen_flat, cap.model._fen_flat), i
        for a, b in zip(list(eager.discriminator.parameters()) + list(eager.discriminator.buffers()),
                        list(cap.discriminator.parameters()) + list(cap.discriminator.buffers())):
            assert torch.equal(a, b), i
    assert cap._gan_graph is not None and eager._gan_graph is None


def test_gan_leg_bench_config_bf16_vs_fp32(tmp_path):
    """The bench's stage-3 iteration (bf16, 6x10, D input 256, B=16) against the same iteration
    in fp32 -- two precisions of the kernels, not a self-comparison.  Same seeded G / D / VGG,
    same batch.  Yardstick for the discriminator's gradient: torch's own CPU discriminator, bf16
    against fp32, from the same initial D on the same inputs (the real batch and each
    precision's fake, i.e. the generator output that iteration's D step sees): the HIP bf16 D
    gradient may be off the HIP fp32 one by at most 1.5x what torch's bf16 is off torch's fp32
    (the D gradients are ill-conditioned below features.7 -- DESIGN.md section 5 -- so a fixed
    bound says little).  The HIP fp32 D gradient against torch fp32 on the identical fake:
    within 3e-2 (2x the worst fp32 spread measured at D input 256, profiles/r05_d256_conditioning.txt).
    The loss within 1 %.  The generator's gradient only as a sanity check (cosine >= 0.95): its bf16
    parity is held by test_gpu_train64.py (G10) and the perceptual leg above."""
    from src.models import VGGStyleDiscriminator
    from src.training.trainer import bicubic_down4
    res = {}
    gen = torch.Generator().manual_seed(99)
    hr = torch.rand(2, 3, 256, 256, generator=gen).repeat(8, 1, 1, 1).to(DEV)     # B = 16
    for prec in ("fp32", "bf16"):
        tr = _bench_gan_trainer(False, tmp_path / prec, precision=prec)
        d0 = {k: v.detach().cpu().clone() for k, v in tr.discriminator.state_dict().items()}
        with torch.no_grad():
            fake = tr.model(bicubic_down4(hr)).float().cpu()              # what the D step sees
        snap, orig_step = {}, tr.optimizer_d.step

        def step_with_snapshot(*a, _s=snap, _tr=tr, _o=orig_step, **kw):
            _s["d"] = torch.cat([p.grad.detach().float().flatten() for p in _tr.discriminator.parameters()])
            return _o(*a, **kw)

        tr.optimizer_d.step = step_with_snapshot
        loss = float(tr._gan_iteration(hr, update=False))     # G's gradients left in .grad
        torch.cuda.synchronize()
        g = torch.cat([p.grad.detach().float().flatten() for p in tr.model.parameters()])
        res[prec] = (loss, snap["d"].cpu().double(), g.cpu().double(), fake, d0)
        del tr
    (l32, d32, g32, f32, d0), (l16, d16, g16, f16, _) = res["fp32"], res["bf16"]
    bce = nn.BCEWithLogitsLoss()
    hr_c = hr.cpu()

    def torch_dgrad(fake, dtype):
        D = VGGStyleDiscriminator(input_size=256)
        D.load_state_dict(d0)
        D = D.to(dtype).train()
        n = hr_c.shape[0]
        lr_ = D.classifier(D.features(hr_c.to(dtype))).float()
        lf_ = D.classifier(D.features(fake.to(dtype))).float()
        ((bce(lr_, torch.ones(n, 1)) + bce(lf_, torch.zeros(n, 1))) / 2).backward()
        return torch.cat([p.grad.float().flatten() for p in D.parameters()]).double()

    t32, t16 = torch_dgrad(f32, torch.float32), torch_dgrad(f16, torch.bfloat16)
    rel = lambda a, b: float((a - b).norm() / b.norm())                      # noqa: E731
    cos = lambda a, b: float((a * b).sum() / (a.norm() * b.norm()))         # noqa: E731
    e_hip, e_torch, e_32 = rel(d16, d32), rel(t16, t32), rel(d32, t32)
    print(f"GAN bench config: loss bf16 {l16:.6f} fp32 {l32:.6f}; D grad bf16 vs fp32: HIP rel {e_hip:.3e} "
          f"(cos {cos(d16, d32):.5f}), torch CPU rel {e_torch:.3e} (cos {cos(t16, t32):.5f}); HIP fp32 vs torch "
          f"fp32 {e_32:.3e}; G grad rel {rel(g16, g32):.3e} cos {cos(g16, g32):.5f}")
    assert np.isfinite(l16) and abs(l16 - l32) <= 1e-2 * abs(l32), (l16, l32)
    assert e_32 <= 3e-2, e_32
    assert e_hip <= 1.5 * e_torch, (e_hip, e_torch)
    assert cos(g16, g32) >= 0.95, cos(g16, g32)
