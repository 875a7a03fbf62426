"""The engine's bucket exchange over RCCL itself (torch.distributed backend "nccl" = RCCL on
ROCm), on the one GPU of the test box: a one-rank process group, with every bucket's
all_reduce issued even at world size 1 (BucketExchange skips them there), so the RCCL
collectives run on their own stream beside the backward exactly as at N > 1, and the join
before the update is RCCL's work.wait().  A one-rank SUM is the identity, so two fused
steps must equal the exchange-free step bit for bit (gradients, weights, grad norm).  The
N > 1 numerics (1/world pre-scale, mark order, join) are covered by test_gpu_dp_engine.py
and tests/test_dp_cpu.py (gloo, world 2)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
from src.training.dp import init_rccl

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class RcclExchange:
    """dp.BucketExchange with the all-reduces forced at world size 1."""
    world = 1

    def __init__(self, flat, plan, log):
        self.plan = plan
        self.views = {tag: flat[lo:hi] for tag, lo, hi in plan}
        self.works, self.log = [], log

    def launch(self, tag):
        self.log.append(tag)
        self.works.append(dist.all_reduce(self.views[tag], op=dist.ReduceOp.SUM, async_op=True))

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_engine_step_over_rccl(precision):
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    from src.training.dp import broadcast_arena

    def model():
        torch.manual_seed(4)
        m = FaceEnhanceNet(num_channels=64, num_groups=2, blocks_per_group=2, precision=precision)
        with torch.no_grad():
            m.conv_last.weight.normal_(0, 1e-3, generator=torch.Generator().manual_seed(5))
        return m

    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
    hr = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(7)).to(DEV)
    e1 = FENEngine(model(), batch=2, lr_hw=(32, 32), dtype=dt, train=True, clip=0.5, lr=1e-3)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    init_rccl(torch.device("cuda", torch.cuda.current_device()), rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        log = []
        e2 = FENEngine(model(), batch=2, lr_hw=(32, 32), dtype=dt, train=True, clip=0.5, lr=1e-3,
                       exchange=lambda flat, plan: RcclExchange(flat, plan, log))
        broadcast_arena(e2.flat_p)                       # a no-op at one rank, as at N > 1 for rank 0
        for step in range(2):
            log.clear()
            l1 = e1.step(hr)
            l2 = e2.step(hr)
            torch.cuda.synchronize()
            assert log == [t for t, _, _ in e2.exchange.plan], log
            assert torch.equal(l1, l2)
            assert torch.equal(e2.flat_g, e1.flat_g), step
            assert torch.equal(e2.flat_p, e1.flat_p), step
    finally:
        dist.destroy_process_group()


def _init_one_rank():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    init_rccl(torch.device("cuda", torch.cuda.current_device()), rank=0, world_size=1)


def test_engine_captured_step_over_rccl():
    """The DP training step recorded in one hipGraph with its bucket all-reduces
    (dp.BucketExchange on the GPU is stream-ordered: each bucket's RCCL all_reduce on a side
    stream forked from the capture stream at the backward's mark, the side stream joined before
    clip + AdamW), on a one-rank RCCL group with the exchange forced: the capture's warm-up step
    and every replay equal the exchange-free eager step bit for bit."""
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    from src.training.dp import BucketExchange

    def model():
        torch.manual_seed(4)
        m = FaceEnhanceNet(num_channels=64, num_groups=2, blocks_per_group=2, precision="bf16")
        with torch.no_grad():
            m.conv_last.weight.normal_(0, 1e-3, generator=torch.Generator().manual_seed(5))
        return m

    hr = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(7)).to(DEV)
    kw = dict(batch=2, lr_hw=(32, 32), dtype=torch.bfloat16, train=True, clip=0.5, lr=1e-3)
    e1 = FENEngine(model(), **kw)
    _init_one_rank()
    try:
        e2 = FENEngine(model(), **kw, exchange=lambda flat, plan: BucketExchange(flat, plan, force=True))
        assert e2.exchange.active and e2.exchange.stream is not None and e2.exchange.capturable
        e2.hr.copy_(hr)
        e2.capture()                      # one eager step (exchanged), then the recorded step
        e1.step(hr)
        torch.cuda.synchronize()
        assert torch.equal(e2.flat_p, e1.flat_p)
        for i in range(3):
            e2.replay()
            l1 = e1.step(hr)
            torch.cuda.synchronize()
            assert torch.equal(e2.loss, l1), i
            assert torch.equal(e2.flat_g, e1.flat_g), i
            assert torch.equal(e2.flat_p, e1.flat_p), i
    finally:
        dist.destroy_process_group()


def test_gan_iteration_over_rccl(tmp_path):
    """The stage-3 GAN iteration with the module path's bucketed exchanges (dp.ParamGradExchange:
    the generator's tail / group / head buckets and the discriminator's two, each all-reduced
    from a post-accumulate hook on autograd's device thread as the backward completes it,
    stream-ordered), forced on a one-rank RCCL group, CAPTURED (the default at any world size
    since the exchange calls RCCL directly, dp.RcclComm): bit-identical to the exchange-free
    iteration (losses, generator arena, discriminator parameters and buffers) over 2 eager
    warm-ups, the capture and 9 replays; every bucket launch of the capturing iteration forked
    from a capturing stream (so the graph holds the all-reduces, not an eager side effect)."""
    from test_gpu_gan_capture import _state, _trainer
    eager = _trainer(False, tmp_path / "e")
    _init_one_rank()
    try:
        cap = _trainer(True, tmp_path / "c")
        cap._dp_force = True
        assert cap._capture_gan()
        gen = torch.Generator().manual_seed(5)
        for i in range(12):
            hr = torch.rand(2, 3, 128, 128, generator=gen).to(DEV)
            le = float(eager._gan_iteration(hr))
            lc = float(cap._gan_iteration(hr))
            assert le == lc, (i, le, lc)
            for a, b in zip(_state(eager), _state(cap)):
                assert torch.equal(a, b), i
        assert cap._gan_graph is not None
        assert cap._g_ex is not None and cap._d_ex is not None
        assert len(cap._g_ex.ranges) == 2 + 1 and len(cap._d_ex.ranges) == 2   # tail, rg0, head
        assert cap._g_ex.ex.comm is not None and cap._d_ex.ex.comm is not None     # direct RCCL
        g, d = list(cap._g_ex.ex.captured_launches), list(cap._d_ex.ex.captured_launches)
        # 2 eager iterations + the captured one went through Python; replays do not
        assert g == [False] * 6 + [True] * 3, g
        nd = cap.config.d_updates_per_g * 2
        assert d == [False] * (2 * nd) + [True] * nd, d
        cap._g_ex.ex.comm.check()
    finally:
        dist.destroy_process_group()


def test_rccl_comm_direct_capture():
    """dp.RcclComm without a process group (a one-rank communicator through the C-ABI's
    fen_rccl_*): an in-place SUM is the identity, it records into a hipGraph from a side
    thread (as autograd's hook thread issues it) and replays; the library it resolved is
    torch's own RCCL instance (one RCCL per process)."""
    import threading
    from src.training.dp import RcclComm
    assert not dist.is_initialized()
    comm = RcclComm(torch.device("cuda", torch.cuda.current_device()))
    assert comm.world == 1 and comm.rank == 0
    assert "torch/lib/librccl" in comm.library, comm.library    # torch imported first: its instance
    x = torch.randn(1 << 20, device=DEV)
    ref = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    comm.allreduce(x, s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    errs = []
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        x.mul_(2.0)
        base = torch.cuda.current_stream()

        def hook():
            try:
                side.wait_stream(base)
                comm.allreduce(x, side)
            except Exception as e:  # pragma: no cover - reported below
                errs.append(e)
        t = threading.Thread(target=hook)
        t.start()
        t.join()
        base.wait_stream(side)
        x.add_(1.0)
    assert not errs, errs
    x.copy_(ref)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    exp = ref.clone()
    for _ in range(3):
        exp = exp * 2.0 + 1.0
    assert torch.allclose(x, exp, rtol=0, atol=0)
    comm.check()
    RcclComm.destroy_all()
