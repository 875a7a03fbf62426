"""SSIM on the HIP path (csrc/ssim.hip via src/losses/ssim.py) against the reference's own
values (tests/golden/g7_ssim.npz, made by importing src/losses/ssim_loss.py) and the CPU
oracle's restatement; the engine's stage-2 step (L1 + w (1 - SSIM)) against autograd."""
import numpy as np
import pytest
import torch

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_ssim_matches_reference_golden(golden):
    from src.losses import SSIMLoss, ssim
    g = golden("g7_ssim.npz")
    p, t = torch.from_numpy(g["pred"]).to(DEV), torch.from_numpy(g["target"]).to(DEV)
    assert abs(float(ssim(p, t)) - float(g["ssim_mean"])) <= 2e-6
    assert np.allclose(ssim(p, t, size_average=False).cpu().numpy(), g["ssim_per_img"], atol=2e-6)
    assert abs(float(ssim(p, p)) - 1.0) <= 1e-6
    pr = p.clone().requires_grad_(True)
    loss = SSIMLoss()(pr, t)
    loss.backward()
    assert abs(float(loss) - float(g["loss"])) <= 2e-6
    ref = g["dpred"]
    assert np.abs(pr.grad.cpu().numpy() - ref).max() <= 1e-4 * np.abs(ref).max()


@pytest.mark.parametrize("B,C,H,W", [(2, 3, 100, 70), (1, 1, 31, 33), (3, 3, 64, 64), (1, 3, 8, 5)])
@pytest.mark.parametrize("size_average", [True, False])
def test_ssim_loss_vs_oracle(B, C, H, W, size_average):
    """Ragged tiles (100 x 70), images smaller than the window (8 x 5), one channel."""
    from src.losses import SSIMLoss
    torch.manual_seed(B * 1000 + H)
    p = torch.rand(B, C, H, W)
    t = (0.6 * p + 0.4 * torch.rand(B, C, H, W)).clamp(0, 1)
    pr = p.clone().requires_grad_(True)
    ref = 1 - O.ssim(pr, t, size_average=size_average)
    ref.sum().backward()
    pd = p.clone().to(DEV).requires_grad_(True)
    out = SSIMLoss(size_average=size_average)(pd, t.to(DEV))
    out.sum().backward()
    assert torch.allclose(out.detach().cpu(), ref.detach(), atol=2e-6)
    e = (pd.grad.cpu() - pr.grad).abs().max() / pr.grad.abs().max()
    assert e <= 1e-4, float(e)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ssim_grad_accumulates_into_nhwc16(dtype):
    """grad_mode 2: grad_scale * d(sum S)/dpred ADDED to channel c of an NHWC [B,H,W,16]
    buffer (the generator's dL/dsr), padding channels untouched."""
    from src.hip import lib as L
    from src.hip.program import ptr
    from src.losses.ssim import _window1d
    torch.manual_seed(4)
    B, C, H, W = 2, 3, 40, 36
    p = torch.rand(B, C, H, W)
    t = torch.rand(B, C, H, W)
    pr = p.clone().requires_grad_(True)
    O.ssim(pr, t).backward()                      # d(mean S)/dp
    scale = -0.3 / (B * C * H * W)
    expect = -0.3 * pr.grad                       # scale * d(sum S)/dp
    lib = L.load()
    base = 2e-4          # the order of the L1 gradient the buffer holds in the engine (w / N)
    buf = torch.full((B, H, W, 16), base, device=DEV, dtype=dtype)
    rows = lib.fen_ssim_parts(B, C, H, W)
    part = torch.empty(rows * B, device=DEV)
    win = _window1d(11, 1.5).to(DEV)
    pd, td = p.to(DEV), t.to(DEV)
    L.check(lib.fen_ssim(L.dtype_code(dtype), B, C, H, W, ptr(pd), ptr(td), ptr(win), 11, 1e-4, 9e-4, ptr(part),
                         ptr(buf), scale, 2, torch.cuda.current_stream().cuda_stream), "ssim")
    torch.cuda.synchronize()
    base_q = torch.tensor(base, dtype=dtype).float()
    got = buf[..., :C].float().cpu().permute(0, 3, 1, 2) - base_q
    tol = 1e-4 if dtype == torch.float32 else 1e-2      # relative to max |expect| (bf16 storage)
    assert (got - expect).abs().max() <= tol * (expect.abs().max() + base)
    assert bool((buf[..., C:].float().cpu() == base_q).all())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,H,W", [(2, 3, 40, 36), (3, 3, 256, 256), (1, 1, 64, 96)])
def test_ssim_two_launch_matches_fused(dtype, B, C, H, W):
    """fen_ssim_ex with a workspace (grad_mode 2: the map + a / b / c maps, then their filtering
    into the gradient) against the one-launch fen_ssim on the same buffers: the fp32 gradient
    bit-identical (fp32 maps, same per-pixel operation order).  The bf16 one (fp16 maps: each of
    G*a, 2p G*b, t G*c off by ~2^-11 of ITSELF, and they cancel where the gradient is small) per
    element within one bf16 ulp of the fused result plus 2e-3 of the tensor's largest magnitude
    (below the 2^-9 relative rounding that bf16 storage already puts on the largest elements),
    checked on a zeroed buffer (the raw gradient) and on one holding 3e-4 (the accumulation);
    the tile sums to fp32 summation order."""
    from src.hip import lib as L
    from src.hip.program import ptr
    from src.losses.ssim import _window1d
    torch.manual_seed(9)
    p = torch.rand(B, C, H, W, device=DEV)
    t = (p + 0.1 * torch.randn(B, C, H, W, device=DEV)).clamp(0, 1)
    lib = L.load()
    rows = lib.fen_ssim_parts(B, C, H, W)
    win = _window1d(11, 1.5).to(DEV)
    s = torch.cuda.current_stream().cuda_stream
    out = []
    for two, base in ((False, 3e-4), (True, 3e-4), (False, 0.0), (True, 0.0)):
        buf = torch.full((B, H, W, 16), base, device=DEV, dtype=dtype)
        part = torch.empty(rows * B, device=DEV)
        work = torch.empty(lib.fen_ssim_work_floats(B, C, H, W), device=DEV) if two else None
        L.check(lib.fen_ssim_ex(L.dtype_code(dtype), B, C, H, W, ptr(p), ptr(t), ptr(win), 11, 1e-4, 9e-4,
                                ptr(part), ptr(buf), -0.2 / (B * C * H * W), 2, ptr(work) if two else None, s),
                "ssim_ex")
        torch.cuda.synchronize()
        out.append((buf.clone(), part.clone()))
    for i in (0, 2):
        ref, got = out[i][0].float(), out[i + 1][0].float()
        d = (ref - got).abs()
        if dtype == torch.float32:
            allowed = torch.zeros_like(d)
        else:   # one bf16 ulp of the larger magnitude: 2^(floor(log2 |x|) - 7)
            mag = torch.maximum(ref.abs(), got.abs()).clamp_min(1e-30)
            allowed = torch.exp2(torch.floor(torch.log2(mag)) - 7) + 2e-3 * float(ref.abs().max())
        bad = (d > allowed).nonzero()
        print(f"{dtype} base {i // 2}: max |diff| {d.max().item():.3e}, max |grad| {ref.abs().max().item():.3e}")
        assert bad.numel() == 0, (f"{bad.shape[0]} gradient elements differ, max {d.max().item():.3e}; "
                                  f"first (b, y, x, ch): {bad[:8].tolist()}")
        assert torch.allclose(out[i][1], out[i + 1][1], rtol=1e-5, atol=1e-3)


def test_engine_step_with_ssim_fp32(golden):
    """FENEngine(ssim_weight=0.2) fp32: generator grads of L1 + 0.2 (1 - SSIM) vs oracle autograd."""
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    g1 = golden("g1_config1.npz")
    sd = {k[2:]: torch.from_numpy(v) for k, v in g1.items() if k.startswith("p/")}
    m = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                       res_scale=0.2, precision="fp32")
    m.load_state_dict(sd)
    hr = torch.from_numpy(g1["hr"])
    eng = FENEngine(m, batch=2, lr_hw=(32, 32), dtype=torch.float32, train=True, ssim_weight=0.2)
    eng.hr.copy_(hr.to(DEV))
    eng.ctx.run()
    torch.cuda.synchronize()
    shape = O.NetShape(64, 1, 2, 4, 4, 0.2)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
    out = O.forward(leaves, O.lr_from_hr(hr), shape, training=True)
    loss = (out - hr).abs().mean() + 0.2 * (1 - O.ssim(out, hr))
    loss.backward()
    assert abs(float(eng.total_loss()) - float(loss.detach())) <= 1e-5 * float(loss.detach())
    bad = {}
    for k, gg in eng.grads.items():
        ref = leaves[k].grad.double()
        e = float((gg.cpu().double() - ref).norm() / max(ref.norm(), 1e-30))
        if not e <= 1e-4:
            bad[k] = e
    assert not bad, bad


def test_ssim_two_launch_small_constants_bf16():
    """fen_ssim_ex's fp16 a / b / c maps overflow for small C1 / C2 (|c| <= 2 / C2,
    |a| up to ~8 / C2 + 1 / sqrt(C1)); below the bound in fen.h the bf16 gradient takes fp32
    maps.  At C1 = 1e-8, C2 = 1e-6 (8 / C2 = 8e6) the two-launch bf16 gradient is finite and
    within one bf16 ulp of the one-launch fen_ssim's."""
    from src.hip import lib as L
    from src.hip.program import ptr
    from src.losses.ssim import _window1d
    B, C, H, W = 2, 3, 64, 64
    torch.manual_seed(3)
    p = torch.rand(B, C, H, W, device=DEV)
    t = (p + 0.05 * torch.randn(B, C, H, W, device=DEV)).clamp(0, 1)
    p[:, :, :8, :8] = 0.25                       # flat patches: variances ~0, the coefficients ~1/C2
    t[:, :, :8, :8] = 0.25
    lib = L.load()
    rows = lib.fen_ssim_parts(B, C, H, W)
    win = _window1d(11, 1.5).to(DEV)
    s = torch.cuda.current_stream().cuda_stream
    out = []
    for two in (False, True):
        buf = torch.zeros((B, H, W, 16), device=DEV, dtype=torch.bfloat16)
        part = torch.empty(rows * B, device=DEV)
        work = torch.empty(lib.fen_ssim_work_floats(B, C, H, W), device=DEV)
        L.check(lib.fen_ssim_ex(L.dtype_code(torch.bfloat16), B, C, H, W, ptr(p), ptr(t), ptr(win), 11, 1e-8, 1e-6,
                                ptr(part), ptr(buf), 1.0 / (B * C * H * W), 2, ptr(work) if two else None, s),
                "ssim_ex")
        torch.cuda.synchronize()
        out.append(buf.float())
    ref, got = out
    assert bool(torch.isfinite(got).all())
    mag = torch.maximum(ref.abs(), got.abs()).clamp_min(1e-30)
    allowed = torch.exp2(torch.floor(torch.log2(mag)) - 7)
    assert bool(((ref - got).abs() <= allowed).all()), float((ref - got).abs().max())
