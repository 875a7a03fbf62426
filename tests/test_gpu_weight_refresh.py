"""After an optimizer update done by the HIP kernels (FusedAdamW on the module path, the fused
engine's step / graph replay), the module forward must run on the UPDATED weights.  The
update kernels write the parameters through raw pointers, so the packed-weight caches keyed on
torch's version counters would otherwise keep serving the pre-update packs (reference: one
nn.Module whose forward always sees its current parameters, custom.py:147-190)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net(seed, precision="bf16"):
    from src.models import FaceEnhanceNet
    torch.manual_seed(seed)
    return FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, precision=precision).to(DEV)


def _fresh_forward(m, x, precision="bf16"):
    ref = _net(123, precision)
    ref.load_state_dict(m.state_dict())
    ref.eval()
    with torch.no_grad():
        return ref(x)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_module_forward_after_fused_adamw(precision):
    from src.hip.engine import flatten_params
    from src.training.optim import FusedAdamW
    m = _net(1, precision)
    flatten_params(m, DEV)                          # the arena FusedAdamW steps on (Trainer does this)
    m.eval()
    x = torch.rand(2, 3, 32, 32, device=DEV)
    with torch.no_grad():
        y0 = m(x)                                   # packs the weights
    flat = m._fen_flat
    g = torch.randn_like(flat) * 1e-2
    opt = FusedAdamW(list(m.parameters()), flat, g, lr=1e-2)
    opt.step()
    with torch.no_grad():
        y1 = m(x)
    ref = _fresh_forward(m, x, precision)
    assert not torch.equal(y1, y0)
    assert torch.equal(y1, ref)


def test_module_forward_after_engine_step_and_replay():
    from src.hip.engine import FENEngine
    m = _net(2)
    x = torch.rand(2, 3, 32, 32, device=DEV)
    m.eval()
    with torch.no_grad():
        y0 = m(x)
    eng = FENEngine(m, batch=2, lr_hw=(32, 32), dtype=torch.bfloat16, train=True, device=DEV, lr=1e-2)
    hr = torch.rand(2, 3, 128, 128, device=DEV)
    eng.step(hr)
    torch.cuda.synchronize()
    with torch.no_grad():
        y1 = m(x)
    assert not torch.equal(y1, y0)
    assert torch.equal(y1, _fresh_forward(m, x))
    eng.capture()
    eng.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        y2 = m(x)
    assert not torch.equal(y2, y1)
    assert torch.equal(y2, _fresh_forward(m, x))
