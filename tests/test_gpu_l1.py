"""The module path's L1 (src/losses L1Loss -> fen_l1_loss; combined.py:38-47, the Trainer's
F.l1_loss fallback) against torch's F.l1_loss: value and d(pred), including an element count
that is not a multiple of the block size and exact ties (sign 0), and a non-unit upstream
gradient read on the device."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape", [(2, 3, 64, 64), (3, 3, 37, 41)])
def test_l1_loss_matches_torch(shape):
    from src.losses import L1Loss
    g = torch.Generator().manual_seed(0)
    p = torch.rand(shape, generator=g).to(DEV)
    t = torch.rand(shape, generator=g).to(DEV)
    t.view(-1)[:50] = p.view(-1)[:50]                      # ties: zero gradient
    a = p.clone().requires_grad_(True)
    b = p.clone().requires_grad_(True)
    la = L1Loss()(a, t)
    lb = F.l1_loss(b, t)
    (3.0 * la).backward()
    (3.0 * lb).backward()
    torch.cuda.synchronize()
    assert abs(float(la) - float(lb)) <= 1e-6 * float(lb)
    assert torch.allclose(a.grad, b.grad, rtol=1e-6, atol=0)
    assert float(a.grad.view(-1)[:50].abs().max()) == 0.0
