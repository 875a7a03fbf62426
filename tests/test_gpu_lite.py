"""FaceEnhanceNetLite (reference custom.py:322-333: 32 channels, reduction 2, 3 groups x 4
RCABs) trained on the HIP path: the 16-bit convs and weight gradients take its 32-channel
activations (a half 64-channel panel, the upper half zeros), so Lite runs the same engine and
module paths as the full net.  Inference parity vs the reference is test_gpu_module's g6_lite
case (fp32, bf16, fp16); here the training step against autograd through the CPU oracle on
the same seeded Lite weights."""
import pytest
import torch
import torch.nn.functional as F

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPE = O.NetShape(32, 3, 4, 2, 4, 0.2)
DT = {"fp32": torch.float32, "bf16": torch.bfloat16}


def _lite(precision):
    from src.models import FaceEnhanceNetLite
    torch.manual_seed(0)
    m = FaceEnhanceNetLite(precision=precision)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=g) * 3e-2)
    return m


def _hr():
    return torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(5))


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_lite_engine_step(precision):
    """One fused engine step (LR synthesis, fwd, L1, bwd, clip 0.5, AdamW lr 1e-3): fp32 ==
    the oracle's step (grads rel 1e-4, weights 2e-5); bf16: every gradient tensor within rel
    5e-2 of the oracle's (cosine of the whole gradient >= 0.999)."""
    from src.hip.engine import FENEngine
    m = _lite(precision)
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    hr = _hr()
    eng = FENEngine(m, batch=2, lr_hw=(16, 16), dtype=DT[precision], train=True, clip=0.5, lr=1e-3)
    eng.hr.copy_(hr.to(DEV))
    eng.ctx.run()
    torch.cuda.synchronize()
    ref_loss, ref_g = O.l1_grads(p, hr, SHAPE)
    assert abs(float(eng.loss) - ref_loss) <= (1e-5 if precision == "fp32" else 2e-3) * ref_loss
    tol = 1e-4 if precision == "fp32" else 5e-2
    bad = {k: _rel(eng.grads[k], g) for k, g in ref_g.items() if not _rel(eng.grads[k], g) <= tol}
    assert not bad, bad
    flat_ref = torch.cat([ref_g[k].reshape(-1) for k in ref_g]).double()
    flat = torch.cat([eng.grads[k].reshape(-1).cpu() for k in ref_g]).double()
    assert float((flat @ flat_ref) / (flat.norm() * flat_ref.norm())) >= 0.999
    if precision == "fp32":
        eng.exchange.wait()
        eng.upd.run()
        torch.cuda.synchronize()
        c = O.clip_coef(ref_g, 0.5)
        newp = {k: t.clone() for k, t in p.items()}
        O.adamw_step(newp, {k: t * c for k, t in ref_g.items()}, {k: torch.zeros_like(t) for k, t in p.items()},
                     {k: torch.zeros_like(t) for k, t in p.items()}, 1, 1e-3)
        for k, v in m.state_dict().items():
            assert float((v.cpu() - newp[k]).abs().max()) <= 2e-5, k


def test_lite_module_autograd_bf16():
    """The module path (autograd Functions over the same kernels) in bf16: loss and gradients
    of F.l1_loss(model(lr), hr) vs the oracle."""
    m = _lite("bf16").to(DEV).train()
    p = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    hr = _hr()
    lr = O.lr_from_hr(hr.double()).float()
    loss = F.l1_loss(m(lr.to(DEV)), hr.to(DEV))
    loss.backward()
    ref_loss, ref_g = O.l1_grads(p, hr, SHAPE)
    assert abs(float(loss) - ref_loss) <= 2e-3 * ref_loss
    bad = {k: _rel(q.grad, ref_g[k]) for k, q in m.named_parameters() if not _rel(q.grad, ref_g[k]) <= 5e-2}
    assert not bad, bad
