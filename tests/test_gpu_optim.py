"""HipAdamW (src/training/optim.py: torch.optim.AdamW with its step on fen_adamw_multi) against
torch.optim.AdamW itself -- the discriminator's optimizer_d (reference trainer.py:230-250,
446-451).  Several steps with weight decay on tensors of mixed sizes (a tail of 1..3 elements,
one larger than a block), parameters without a gradient skipped; every tensor within fp32
rounding of torch's; state_dict interchangeable both ways; captured in a hipGraph it replays."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 3, 3), (1,), (7,), (1000, 33), (5, 5), (33,)]
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]


def _grads(ps, step):
    g = torch.Generator().manual_seed(100 + step)
    for i, p in enumerate(ps):
        p.grad = None if i == 2 and step % 2 else torch.randn(p.shape, generator=g).to(DEV)


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_hip_adamw_matches_torch(wd):
    from src.training.optim import HipAdamW
    a, b = _params(0), _params(0)
    oa = torch.optim.AdamW(a, lr=3e-3, weight_decay=wd, capturable=True)
    ob = HipAdamW(b, lr=3e-3, weight_decay=wd)
    for step in range(5):
        _grads(a, step)
        _grads(b, step)
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        assert torch.allclose(pa, pb, rtol=2e-6, atol=2e-7), float((pa - pb).abs().max())
        sa, sb = oa.state[pa], ob.state[pb]
        assert float(sa["step"]) == float(sb["step"])
        for k in ("exp_avg", "exp_avg_sq"):
            ta, tb = sa[k], sb[k]
            assert float((ta - tb).abs().max()) <= 1e-6 * float(ta.abs().max()), (k, float((ta - tb).abs().max()))
    # state_dict both ways: the next step from either optimizer's state agrees
    c = _params(0)
    oc = HipAdamW(c, lr=3e-3, weight_decay=wd)
    with torch.no_grad():
        for pc, pa in zip(c, a):
            pc.copy_(pa)
    # (a copy, as a checkpoint is: torch's load_state_dict keeps same-device tensors as they are,
    # so a live state_dict would alias oa's moments)
    oc.load_state_dict(copy.deepcopy(oa.state_dict()))
    _grads(a, 7)
    _grads(c, 7)
    oa.step()
    oc.step()
    torch.cuda.synchronize()
    for pa, pc in zip(a, c):
        assert torch.allclose(pa, pc, rtol=2e-6, atol=2e-7)
    assert set(oc.state_dict()["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


def test_hip_adamw_captured():
    from src.training.optim import HipAdamW
    a, b = _params(1), _params(1)
    oa, ob = HipAdamW(a, lr=1e-3), HipAdamW(b, lr=1e-3)
    for p, q in zip(a, b):
        p.grad = torch.ones_like(p)
        q.grad = torch.ones_like(q)
    oa.step()
    ob.step()                                   # lazy state before the capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g):
        ob.step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        oa.step()
        g.replay()
    torch.cuda.synchronize()
    for p, q in zip(a, b):
        assert torch.equal(p, q)
