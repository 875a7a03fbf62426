"""VGGStyleDiscriminator on the HIP path vs the reference's own outputs and gradients
(tests/golden/g8_disc.npz: input_size 64, seed-0 init, B = 4): train-mode forward (batch
statistics), d(sum out*R) w.r.t. the input and every parameter, running statistics after
the step, eval-mode forward (running statistics).  fp32 against the reference in float64;
bf16 no further from float64 than torch's own bf16 run of the same module tree (x1.25)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_discriminator_vs_reference(golden, precision):
    from src.models import VGGStyleDiscriminator
    g = golden("g8_disc.npz")
    torch.manual_seed(0)
    d = VGGStyleDiscriminator(input_size=64, precision=precision).to(DEV).train()
    x = torch.from_numpy(g["x"]).to(DEV).requires_grad_(True)
    r = torch.from_numpy(g["r"]).to(DEV)
    out = d(x)
    (out * r).sum().backward()
    torch.cuda.synchronize()
    fp32 = precision == "fp32"
    if not fp32:
        # bf16 yardstick: torch's own bf16 autograd of the same module tree on the CPU (the
        # nn.Sequential submodules run natively there), each error measured against float64
        torch.manual_seed(0)
        dt = VGGStyleDiscriminator(input_size=64).to(torch.bfloat16).train()
        xb = torch.from_numpy(g["x"]).to(torch.bfloat16).requires_grad_(True)
        ob = dt.classifier(dt.features(xb))
        (ob.float() * torch.from_numpy(g["r"])).sum().backward()
        yard = {"gx": _rel(xb.grad.float(), g["f64/gx"]), "out": _rel(ob.detach().float(), g["f64/out_train"])}
        for k, p in dt.named_parameters():
            yard[k] = abs(float(p.grad.double().norm()) - float(g["f64/gn/" + k])) / float(g["f64/gn/" + k])
    # fp32: against the reference run in float64, within max(2 x the reference's own fp32
    # error, 1e-4) -- ten BatchNorm backward layers (the last over 16 samples per channel)
    # amplify rounding order; bf16: 5e-2 on outputs, 1e-1 on gradients
    ref_o, ref_gx = g["f64/out_train"], g["f64/gx"]
    tol_o = max(2 * _rel(g["out_train"], g["f64/out_train"]), 1e-4) if fp32 else 1.25 * yard["out"] + 1e-2
    tol_gx = max(2 * _rel(g["gx"], g["f64/gx"]), 1e-4) if fp32 else 1.25 * yard["gx"] + 1e-2
    assert _rel(out.detach().cpu(), ref_o) <= tol_o
    assert _rel(x.grad.cpu(), ref_gx) <= tol_gx
    bad = {}
    for k, p in d.named_parameters():
        gr = p.grad.detach().double().cpu()
        gn = float(g["f64/gn/" + k])
        e = abs(float(gr.norm()) - gn) / max(gn, 1e-30)
        if fp32:
            noise = torch.randn(p.shape, generator=torch.Generator().manual_seed(7)).double()
            e = max(e, abs(float((gr * noise).sum()) - float(g["f64/gp/" + k])) / max(gn, 1e-30))
        tol = max(2 * abs(float(g["gn/" + k]) - gn) / max(gn, 1e-30), 1e-4) if fp32 else max(1.25 * yard[k], 5e-2)
        if not e <= tol:
            bad[k] = (e, tol)
    assert not bad, bad
    for k, v in d.state_dict().items():
        if "running" in k:
            assert _rel(v.cpu(), g["bn_after/" + k]) <= (1e-5 if precision == "fp32" else 2e-2), k
    d.eval()
    with torch.no_grad():
        oe = d(torch.from_numpy(g["x"]).to(DEV))
    assert _rel(oe.cpu(), g["out_eval"]) <= (1e-4 if fp32 else 5e-2)


@pytest.mark.parametrize("B,sigmoid", [(2, False), (16, False), (20, True)])
def test_classifier_head_vs_float64(B, sigmoid):
    """The HIP classifier head (fen_dhead_fwd / fen_dhead_bwd: Linear(32768, 1024) -> LeakyReLU(0.2)
    -> Linear(1024, 1) [-> sigmoid], discriminator.py:85-90,131-132) against torch float64 on the
    same fp32 operands, at the bench's D input (256: K = 512 x 8 x 8); B = 20 takes two sample
    chunks in the backward.  Score, input gradient and every parameter gradient within rel 1e-5;
    two runs bit-identical."""
    import torch.nn.functional as F
    from src.models.discriminator import _DHead
    K, N = 32768, 1024
    g = torch.Generator().manual_seed(11)
    h = (torch.randn(B, K, generator=g) * 0.5).to(DEV)
    w1 = (torch.randn(N, K, generator=g) * (2.0 / K) ** 0.5).to(DEV)
    b1 = (torch.randn(N, generator=g) * 0.1).to(DEV)
    w2 = (torch.randn(1, N, generator=g) * (2.0 / N) ** 0.5).to(DEV)
    b2 = (torch.randn(1, generator=g) * 0.1).to(DEV)
    r = torch.randn(B, 1, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        leaves = [t.clone().requires_grad_(True) for t in (h, w1, b1, w2, b2)]
        y = _DHead.apply(*leaves, sigmoid)
        (y * r).sum().backward()
        torch.cuda.synchronize()
        outs.append([y.detach()] + [t.grad for t in leaves])
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    l64 = [t.detach().double().cpu().requires_grad_(True) for t in (h, w1, b1, w2, b2)]
    y64 = F.linear(F.leaky_relu(F.linear(l64[0], l64[1], l64[2]), 0.2), l64[3], l64[4])
    if sigmoid:
        y64 = torch.sigmoid(y64)
    (y64 * r.double().cpu()).sum().backward()
    ref = [y64.detach()] + [t.grad for t in l64]
    for name, a, b in zip(("y", "dh", "dw1", "db1", "dw2", "db2"), outs[0], ref):
        e = _rel(a.cpu().numpy(), b.numpy())
        assert e <= 1e-5, (name, e)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_forward_pair_matches_two_calls(precision):
    """VGGStyleDiscriminator.forward_pair (the D step's real and fake batches as one pass,
    trainer.py:433-434): the same scores as two calls (per-batch BatchNorm statistics; bit for bit
    in fp32, where the kernels do not depend on the batch), the same running statistics and
    num_batches_tracked (updated real then fake), parameter gradients of the summed loss equal
    up to fp32 summation order (one weight-gradient launch over both batches vs two + add)."""
    import copy
    from src.models import VGGStyleDiscriminator
    torch.manual_seed(4)
    d1 = VGGStyleDiscriminator(input_size=64, precision=precision).to(DEV).train()
    d2 = copy.deepcopy(d1)
    g = torch.Generator().manual_seed(5)
    xr, xf = torch.rand(3, 3, 64, 64, generator=g).to(DEV), torch.rand(3, 3, 64, 64, generator=g).to(DEV)
    a1, b1 = d1(xr), d1(xf)
    a2, b2 = d2.forward_pair(xr, xf)
    ((a1 * 0.7).sum() - (b1 * 1.3).sum()).backward()
    ((a2 * 0.7).sum() - (b2 * 1.3).sum()).backward()
    torch.cuda.synchronize()
    if precision == "fp32":
        assert torch.equal(a1, a2) and torch.equal(b1, b2)
    else:
        assert float((a1 - a2).abs().max()) <= 2e-2 * float(a1.abs().max()) + 1e-3
    for (k, t1), t2 in zip(d1.state_dict().items(), d2.state_dict().values()):
        if "running" in k or "num_batches" in k:
            assert torch.allclose(t1.float(), t2.float(), rtol=1e-5, atol=1e-6), k
    tol = 1e-5 if precision == "fp32" else 3e-2
    for (k, p1), p2 in zip(d1.named_parameters(), d2.parameters()):
        e = float((p1.grad - p2.grad).norm() / max(float(p1.grad.norm()), 1e-30))
        assert e <= tol, (k, e)


@pytest.mark.parametrize("gan_type", ["vanilla", "lsgan", "wgan"])
@pytest.mark.parametrize("is_real", [True, False])
def test_gan_loss_hip(gan_type, is_real):
    """GANLoss on fen_gan_loss: the loss and d(loss)/d(scores) equal the reference criteria's
    (nn.BCEWithLogitsLoss / nn.MSELoss / the signed mean, torch on the same device) within fp32
    rounding, for large, small and zero scores."""
    from src.models import GANLoss
    x = torch.tensor([[-30.0], [-3.5], [-0.2], [0.0], [0.7], [4.0], [25.0]] * 3, device=DEV, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    gl = GANLoss(gan_type)
    loss = gl(x, is_real) * 1.7
    t = torch.full_like(xr, 1.0 if is_real else 0.0)
    if gan_type == "vanilla":
        ref = torch.nn.BCEWithLogitsLoss()(xr, t)
    elif gan_type == "lsgan":
        ref = torch.nn.MSELoss()(xr, t)
    else:
        ref = -xr.mean() if is_real else xr.mean()
    ref = ref * 1.7
    loss.backward()
    ref.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(ref)) <= 1e-6 * abs(float(ref)) + 1e-7
    assert torch.allclose(x.grad, xr.grad, rtol=1e-5, atol=1e-8)
