"""The engine's data-parallel step (the reference's DDP generator step,
trainer.py:126-134 / 480-503) on one GPU, with a stand-in for the RCCL bucket exchange.

`PairExchange` plays a world of 2 whose other rank holds the same batch: `launch(tag)` enqueues
the SUM of the two identical shards (bucket *= 2) on a side stream -- as RCCL runs on its own
stream -- behind an event recorded on the compute stream at the mark and a ~1 ms spin, and
`wait()` joins the side stream into the compute stream.  Then:

  * 1/world pre-scale: the exchanged gradients equal the world-1 gradients (bit for bit:
    the scale 1/2 and the SUM x2 are exact in fp32 and bf16), and so do the updated weights;
  * mark order: every launch whose arguments point into a bucket's slice of the gradient
    arena precedes that bucket's mark (a mark issued early would exchange a half-written
    bucket and, with the side stream's delay, show up as a gradient mismatch too), the marks
    come in the backward's completion order (tail, rg{G-1}..rg0, head), once each;
  * the update waits for every bucket: the host calls wait() after the last launch and
    before the update program is enqueued, and the updated weights (read by AdamW after the
    side stream's delayed x2) match the world-1 step.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


class PairExchange:
    world = 2

    def __init__(self, flat, plan, log, delay_cycles=2_000_000):
        self.plan = plan
        self.views = {tag: flat[lo:hi] for tag, lo, hi in plan}
        self.side = torch.cuda.Stream()
        self.log, self.delay, self.done = log, delay_cycles, []

    def launch(self, tag):
        self.log.append(("launch", tag))
        ready = torch.cuda.Event()
        ready.record()                        # on the compute stream, after the enqueued wgrads
        self.side.wait_event(ready)
        with torch.cuda.stream(self.side):
            torch.cuda._sleep(self.delay)     # a slow collective: a missing join reads stale grads
            self.views[tag].mul_(2.0)         # SUM over two ranks holding identical shards
        done = torch.cuda.Event()
        done.record(self.side)
        self.done.append(done)

    def wait(self):
        self.log.append(("wait",))
        for e in self.done:
            torch.cuda.current_stream().wait_event(e)
        self.done = []


def _model(precision, seed=4):
    from src.models import FaceEnhanceNet
    torch.manual_seed(seed)
    m = FaceEnhanceNet(num_channels=64, num_groups=2, blocks_per_group=2, precision=precision)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():   # a conv_last that moves the output (the reference init is tiny)
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=g) * 2e-2)
    return m


def _addrs(a):
    """Every pointer-sized integer an op's arguments carry (descriptors walked field by field)."""
    if isinstance(a, bool):
        return []
    if isinstance(a, int):
        return [a]
    if isinstance(a, (list, tuple)):
        return [x for y in a for x in _addrs(y)]
    if hasattr(a, "_obj"):                    # ctypes.byref(...)
        return _addrs(a._obj)
    if isinstance(a, ctypes.c_void_p):
        return [a.value or 0]
    if isinstance(a, ctypes.Structure):
        return _addrs([getattr(a, f[0]) for f in a._fields_])
    if isinstance(a, ctypes.Array):
        return _addrs(list(a))
    return []


def _engine(precision, exchange=None, ssim=0.0):
    from src.hip.engine import FENEngine
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
    m = _model(precision)
    eng = FENEngine(m, batch=2, lr_hw=(32, 32), dtype=dt, train=True, clip=0.5, lr=1e-3,
                    ssim_weight=ssim, exchange=exchange)
    return m, eng


@pytest.mark.parametrize("precision,ssim", [("fp32", 0.0), ("bf16", 0.0), ("bf16", 0.2)])
def test_dp_step_matches_world1(precision, ssim):
    hr = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(7)).to(DEV)
    _, e1 = _engine(precision, ssim=ssim)
    log = []
    _, e2 = _engine(precision, exchange=lambda flat, plan: PairExchange(flat, plan, log), ssim=ssim)
    assert e1.world == 1 and e2.world == 2
    upd_run = e2.upd.run
    e2.upd.run = lambda *a: (log.append(("update",)), upd_run(*a))[1]
    tags = [t for t, _, _ in e2.exchange.plan]
    assert tags == ["tail", "rg1", "rg0", "head"]
    for step in range(2):
        log.clear()
        l1 = e1.step(hr)
        l2 = e2.step(hr)
        torch.cuda.synchronize()
        # the host order: every bucket launched once, in plan order, then the join, then the update
        assert log == [("launch", t) for t in tags] + [("wait",), ("update",)], log
        # each rank's own loss is its shard's (the same batch here)
        assert torch.equal(l1, l2)
        assert torch.equal(e2.flat_g, e1.flat_g), (step, float((e2.flat_g - e1.flat_g).abs().max()))
        assert torch.equal(e2.flat_p, e1.flat_p), step
        assert float(e2.grad_norm) == float(e1.grad_norm)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_dp_marks_follow_bucket_writers(precision):
    log = []
    _, eng = _engine(precision, exchange=lambda flat, plan: PairExchange(flat, plan, log), ssim=0.2)
    el = eng.flat_g.element_size()
    base = eng.flat_g.data_ptr()
    spans = {t: (base + lo * el, base + hi * el) for t, lo, hi in eng.exchange.plan}
    marks, last_writer = {}, {t: -1 for t in spans}
    forked = False                       # a strip-backward group's column sums on the side stream
    for i, (name, fn, args) in enumerate(eng.ctx.ops):
        if fn is None and name in ("cs_fork", "cs_join"):
            assert forked == (name == "cs_join"), (i, name)     # fork, join, fork, join ...
            forked = name == "cs_fork"
            continue
        if fn is None:
            assert not forked, (i, name)                        # joined before any bucket's exchange
            assert name.startswith("allreduce_"), name
            tag = name[len("allreduce_"):]
            assert tag not in marks, tag
            marks[tag] = i
            continue
        for a in _addrs(args):
            for t, (lo, hi) in spans.items():
                if lo <= a < hi:
                    last_writer[t] = i
    assert list(marks) == [t for t, _, _ in eng.exchange.plan]
    for t, i in marks.items():
        assert 0 <= last_writer[t] < i, (t, last_writer[t], i)
    # the forward's first launch precedes every mark (the exchange belongs to the backward)
    assert min(marks.values()) > 0
