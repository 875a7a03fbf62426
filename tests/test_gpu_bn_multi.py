"""Grouped BatchNorm launches (fen_bn_stats_n / fen_bn_apply_n / fen_bn_bwd_n, disc.hip) against
ng separate one-group calls: the D step's real and fake batches (reference trainer.py:433-434,
discriminator.py:47-55 -- train-mode BatchNorm2d + LeakyReLU(0.2)) run in the launches of one
batch, each with its own statistics, the running statistics moved group by group, dgamma / dbeta
summed in group order.  Bit-identical, for the per-channel-group kernels (C = 64, 512) and the
fallback's launch per group (bf16 C = 24)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _p(t):
    return t.data_ptr()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("C,npx,ng", [(64, 4096, 2), (512, 256, 2), (24, 1000, 3)])
def test_bn_grouped_equals_per_group(dt, C, npx, ng):
    from src.hip import lib as L
    lib = L.load()
    code = L.dtype_code(dt)
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(C + npx)
    y = (torch.randn(ng * npx, C, generator=g) * 1.7 + 0.3).to(DEV, dt)
    da = torch.randn(ng * npx, C, generator=g).to(DEV, dt)
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    rm0, rv0 = (0.05 * torch.randn(C, generator=g)).to(DEV), (1 + 0.1 * torch.rand(C, generator=g)).to(DEV)
    wf = lib.fen_bn_work_floats(C)
    esz = y.element_size()

    # one launch set for all groups
    stat_n = torch.zeros(ng, 2 * C, device=DEV)
    rm_n, rv_n = rm0.clone(), rv0.clone()
    work_n = torch.zeros(ng * wf, device=DEV)
    out_n = torch.empty_like(y)
    dy_n = torch.empty_like(y)
    dgam_n, dbet_n = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    L.check(lib.fen_bn_stats_n(code, ng, npx, C, _p(y), 1e-5, 0.1, _p(stat_n), _p(rm_n), _p(rv_n), _p(work_n), s))
    L.check(lib.fen_bn_apply_n(code, ng, npx, C, _p(y), _p(stat_n), _p(stat_n[0, C:]), 2 * C, _p(gamma), _p(beta),
                               0.2, _p(out_n), s))
    L.check(lib.fen_bn_bwd_n(code, ng, npx, C, _p(da), _p(y), _p(stat_n), _p(gamma), _p(beta), 0.2, _p(dy_n),
                             _p(dgam_n), _p(dbet_n), 0, _p(work_n), s))

    # ng one-group calls (the per-batch form)
    stat_1 = torch.zeros(ng, 2 * C, device=DEV)
    rm_1, rv_1 = rm0.clone(), rv0.clone()
    work_1 = torch.zeros(wf, device=DEV)
    out_1 = torch.empty_like(y)
    dy_1 = torch.empty_like(y)
    dgam_1, dbet_1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    for gi in range(ng):
        o = gi * npx * C * esz
        L.check(lib.fen_bn_stats(code, npx, C, _p(y) + o, 1e-5, 0.1, _p(stat_1[gi]), _p(rm_1), _p(rv_1), _p(work_1), s))
        L.check(lib.fen_bn_apply(code, npx, C, _p(y) + o, _p(stat_1[gi]), _p(stat_1[gi, C:]), _p(gamma), _p(beta), 0.2,
                                 _p(out_1) + o, s))
    for gi in range(ng):
        o = gi * npx * C * esz
        L.check(lib.fen_bn_bwd(code, npx, C, _p(da) + o, _p(y) + o, _p(stat_1[gi]), _p(gamma), _p(beta), 0.2,
                               _p(dy_1) + o, _p(dgam_1), _p(dbet_1), int(gi > 0), _p(work_1), s))
    torch.cuda.synchronize()

    assert torch.equal(stat_n, stat_1)
    assert torch.equal(rm_n, rm_1) and torch.equal(rv_n, rv_1)
    assert torch.equal(out_n, out_1)
    assert torch.equal(dy_n, dy_1)
    assert torch.equal(dgam_n, dgam_1) and torch.equal(dbet_n, dbet_1)
    # and the statistics are the batches' own (torch, fp32 over the stored values)
    yf = y.float().view(ng, npx, C)
    assert torch.allclose(stat_n[:, :C], yf.mean(1), rtol=1e-5, atol=1e-5)
    assert torch.allclose(stat_n[:, C:], (yf.var(1, unbiased=False) + 1e-5).rsqrt(), rtol=1e-4, atol=1e-5)
