"""A strip kernel's timed-out hand-off wait is an error, not wrong numbers.

fen_group_strip / fen_group_strip_bwd (the ResidualGroup forward / backward, reference
blocks.py:135-189) bound every wait on a neighbouring strip; on expiry the launch carries on
with stale halo rows, and its last block reports FEN_STATUS_GS_* through the caller's status
word -- host-mapped pinned memory, so the product path reads it without a sync
(lib.check_strip_status).  The engine (forward / step / replay), the module path (every
ResidualGroup forward and backward) and the Trainer (after each step's loss sync) check it and
raise FenError; the word is then clear and the next launch is good.

The fault is injected with the descriptors' test-only `fault` field (net.GS_FAULT): the block
holding ticket 1 (image 0, strip 1) skips one hand-off flag, so strip 0's wait for it runs out
its bound (~1 s).  Shapes: LR 16x64 (two strips per image), one group of two RCABs."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(precision):
    from src.models import FaceEnhanceNet
    torch.manual_seed(0)
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, precision=precision)
    with torch.no_grad():
        m.conv_last.weight.normal_(0, 1e-2)
    return m.to(DEV)


def _lr(B=2):
    return torch.rand(B, 3, 16, 64, generator=torch.Generator().manual_seed(3)).to(DEV)


class _Fault:
    def __init__(self, bits):
        self.bits = bits

    def __enter__(self):
        from src.hip import net
        self.old, net.GS_FAULT = net.GS_FAULT, self.bits

    def __exit__(self, *a):
        from src.hip import net
        net.GS_FAULT = self.old


def _strip_used(m, x):
    from src.hip import lib as L
    return bool(L.load().fen_group_strip_supported(L.dtype_code(m.compute_dtype), x.shape[0], x.shape[2],
                                                   x.shape[3], 64, 16, 2))


def test_status_clear_without_fault():
    from src.hip import lib as L
    m = _model("fp16").eval()
    x = _lr()
    assert _strip_used(m, x)
    with torch.no_grad():
        m(x)
        m(x)
    torch.cuda.synchronize()
    L.check_strip_status()          # nothing reported


def test_forward_fault_raises_then_recovers():
    from src.hip import lib as L
    m = _model("fp16").eval()
    x = _lr()
    with torch.no_grad():
        good = m(x).clone()
        with _Fault(1):
            m(x)                    # one strip's wait expires inside this launch
        torch.cuda.synchronize()
        with pytest.raises(L.FenError, match="fen_group_strip"):
            m(x)                    # the next group forward sees the report
        L.check_strip_status()      # cleared by the raise
        again = m(x)
    torch.cuda.synchronize()
    L.check_strip_status()
    assert torch.equal(again, good)


def test_backward_fault_raises():
    from src.hip import lib as L
    m = _model("bf16").train()
    x = _lr()
    hr = torch.rand(2, 3, 64, 256, generator=torch.Generator().manual_seed(4)).to(DEV)
    with _Fault(2):                 # the backward launch only
        loss = torch.nn.functional.l1_loss(m(x), hr)
        loss.backward()
    torch.cuda.synchronize()
    with pytest.raises(L.FenError, match="fen_group_strip_bwd"):
        m(x)
    L.check_strip_status()


def test_engine_replay_fault_raises():
    """The graph-replayed engine: the fault is baked into the recorded launch; the replay
    after the faulty one raises (check on entry), as does check_status() once drained."""
    from src.hip import lib as L
    from src.hip.engine import FENEngine
    m = _model("fp16").eval()
    x = _lr()
    with _Fault(1):
        eng = FENEngine(m, batch=2, lr_hw=(16, 64), dtype=torch.float16, train=False, device=DEV)
    eng.x.copy_(x)
    eng.capture()                   # its warm-up body ran the faulty launch
    torch.cuda.synchronize()
    with pytest.raises(L.FenError):
        eng.check_status()
    eng.replay()                    # the entry check passes (cleared); this replay faults
    torch.cuda.synchronize()
    with pytest.raises(L.FenError):
        eng.replay()
    L.check_strip_status()
    eng2 = FENEngine(m, batch=2, lr_hw=(16, 64), dtype=torch.float16, train=False, device=DEV)
    eng2.x.copy_(x)
    eng2.capture()
    eng2.replay()
    torch.cuda.synchronize()
    eng2.check_status()             # a fault-free engine reports nothing
