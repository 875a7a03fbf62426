"""The drop-in module API (src.models) on the GPU: reference-format weights in, reference
outputs/gradients/optimizer step out; full-size networks via seeded init (pinned by the
reference's init statistics) against the reference's own outputs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fen_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _sd(g, prefix="p/"):
    return {k[len(prefix):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(prefix)}


def _config1(precision="fp32"):
    from src.models import FaceEnhanceNet
    return FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2, reduction_ratio=4, scale_factor=4,
                          res_scale=0.2, precision=precision)


@pytest.fixture(scope="module")
def g1(golden):
    return golden("g1_config1.npz")


def test_module_forward_and_attention(g1):
    m = _config1()
    m.load_state_dict(_sd(g1))
    m = m.to(DEV)
    lr = torch.from_numpy(g1["lr"]).to(DEV)
    m.train()
    with torch.no_grad():
        out_t = m(lr).cpu().numpy()
    m.eval()
    with torch.no_grad():
        out_e = m(lr).cpu().numpy()
    assert np.abs(out_t - g1["out_train"]).max() <= 1e-3
    assert np.abs(out_e - g1["out_eval"]).max() <= 1e-3
    maps = m.get_attention_maps(lr)
    assert sorted(maps) == sorted(k[5:] for k in g1 if k.startswith("attn/"))
    for k, v in maps.items():
        assert np.abs(v.cpu().numpy() - g1["attn/" + k]).max() <= 1e-4


def test_module_autograd_and_reference_trainer_step(g1):
    """loss.backward() fills every .grad like the reference; one reference-style step
    (clip_grad_norm_ 0.5 + AdamW lr 1e-4, trainer.py:490-503) lands on the reference's params."""
    m = _config1()
    m.load_state_dict(_sd(g1))
    m = m.to(DEV).train()
    hr = torch.from_numpy(g1["hr"]).to(DEV)
    lr = torch.from_numpy(g1["lr"]).to(DEV)
    fwd_hooks, bwd_hooks = [], []
    m.residual_groups[0].register_forward_hook(lambda mod, i, o: fwd_hooks.append(o.shape))
    m.residual_groups[0].register_full_backward_hook(lambda mod, gi, go: bwd_hooks.append(go[0].shape))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.0)
    opt.zero_grad()
    loss = F.l1_loss(m(lr), hr)
    loss.backward()
    assert fwd_hooks and bwd_hooks
    assert abs(float(loss) - float(g1["l1_loss"])) < 1e-6
    for k, p in m.named_parameters():
        ref = torch.from_numpy(g1["g/" + k])
        rel = float((p.grad.cpu().double() - ref.double()).norm() / max(ref.double().norm(), 1e-30))
        assert rel <= 1e-4, (k, rel)
    torch.nn.utils.clip_grad_norm_(m.parameters(), 0.5)
    opt.step()
    for k, v in m.state_dict().items():
        d = np.abs(v.cpu().numpy() - g1["s/" + k]).max()
        assert d <= 2e-5, (k, d)  # |update| is ~lr=1e-4 per element


def _seeded(ctor, golden_npz):
    torch.manual_seed(0)
    m = ctor()
    sd = m.state_dict()
    names = list(golden_npz["stat_names"])
    for n, s1, s2 in zip(names, golden_npz["stat_sum"], golden_npz["stat_sumsq"]):
        t = sd[n].double()
        assert abs(float(t.sum()) - s1) <= 1e-9 * max(1, abs(s1)) and abs(float((t * t).sum()) - s2) <= 1e-9 * max(1, s2), n
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=g) * 1e-3)
    return m


@pytest.mark.parametrize("name,ctor", [
    ("g4_full.npz", lambda p: __import__("src.models", fromlist=["x"]).FaceEnhanceNet(
        num_channels=64, num_groups=6, blocks_per_group=10, reduction_ratio=4, scale_factor=4, precision=p)),
    ("g5_c128.npz", lambda p: __import__("src.models", fromlist=["x"]).FaceEnhanceNet(
        num_channels=128, num_groups=10, blocks_per_group=20, reduction_ratio=4, scale_factor=8, precision=p)),
    ("g6_lite.npz", lambda p: __import__("src.models", fromlist=["x"]).FaceEnhanceNetLite(precision=p)),
])
@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
def test_full_networks_vs_reference(golden, name, ctor, precision):
    g = golden(name)
    m = _seeded(lambda: ctor(precision), g).to(DEV)
    x = torch.from_numpy(g["x"]).to(DEV)
    with torch.no_grad():
        m.eval()
        out_e = m(x).cpu()
        m.train()
        out_t = m(x).cpu()
    ref_e, ref_t = torch.from_numpy(g["out_eval"]), torch.from_numpy(g["out_train"])
    if precision == "fp32":
        # |d| <= 1e-3 per pixel against the reference, unless the reference's own fp32
        # rounding (vs the reference in float64) already exceeds that -- then be at least
        # as close to the float64 reference as 2x the reference's fp32 error.
        f64 = torch.from_numpy(g["out_eval_f64"])
        ref_err = float((ref_e.double() - f64).abs().max())
        if ref_err < 5e-4:
            assert (out_e - ref_e).abs().max() <= 1e-3
            assert (out_t - ref_t).abs().max() <= 1e-3
        else:
            assert float((out_e.double() - f64).abs().max()) <= 2 * ref_err, ref_err
    else:
        # PSNR parity against a fixed target (the bicubic upsample of the input, in fp64; these
        # goldens have noise inputs and no HR -- g9, tests/test_gpu_northstar.py, is the HR case)
        tgt = O.bicubic(x.cpu().double(), m.scale_factor).clamp(0, 1)
        # 0.01 dB (north_star) for the 64-channel nets in both 16-bit formats (measured: bf16
        # 0.0084, fp16 0.0014 dB on g4), plus a per-pixel bound, 6e-3 on [0,1] outputs.  The
        # 128-channel x8 net (config 5, which the reference runs in fp16) carries body
        # activations of O(1e3): fp16 0.0051 dB (gate 0.01), bf16 0.0105 dB (gate 0.02, bf16's
        # weight rounding alone: test_oracle.py::test_bf16_weight_rounding_alone_exceeds_001db).
        tol = 0.01
        if name == "g5_c128.npz" and precision == "bf16":
            tol = 0.02
        d = abs(O.psnr(out_e, tgt) - O.psnr(ref_e, tgt))
        print(f"{name} {precision}: dPSNR {d:.5f} dB, max|d| {float((out_e - ref_e).abs().max()):.2e}")
        assert d <= tol, d
        if name != "g5_c128.npz":
            assert float((out_e - ref_e).abs().max()) <= 6e-3


def test_engine_matches_module(golden):
    """The static-buffer engine (graph-captured) == the module path, bf16, batch 4."""
    from src.hip.engine import FENEngine
    from src.models import FaceEnhanceNet
    g = golden("g4_full.npz")
    torch.manual_seed(0)
    m = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, precision="bf16")
    gen = torch.Generator().manual_seed(1)
    with torch.no_grad():
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=gen) * 1e-3)
    x = torch.rand(4, 3, 32, 32, generator=torch.Generator().manual_seed(9)).to(DEV)
    m = m.to(DEV).eval()
    with torch.no_grad():
        ref = m(x).clone()
    eng = FENEngine(m, batch=4, lr_hw=(32, 32), dtype=torch.bfloat16, train=False)
    eng.x.copy_(x)
    eng.capture()
    eng.replay()
    torch.cuda.synchronize()
    assert torch.equal(eng.out, ref)


def test_engine_train_step_matches_reference(g1):
    """One fused HIP train step (LR synthesis, fwd, L1, bwd, clip 0.5, AdamW) in fp32 ==
    the reference Trainer._train_epoch step on the same batch."""
    from src.hip.engine import FENEngine
    m = _config1()
    m.load_state_dict(_sd(g1))
    eng = FENEngine(m, batch=2, lr_hw=(32, 32), dtype=torch.float32, train=True, clip=0.5, lr=1e-4)
    loss = eng.step(torch.from_numpy(g1["hr"]).to(DEV))
    torch.cuda.synchronize()
    assert abs(float(loss) - float(g1["step_loss"])) < 1e-6
    for k, v in m.state_dict().items():
        d = np.abs(v.cpu().numpy() - g1["s/" + k]).max()
        assert d <= 2e-5, (k, d)


@pytest.mark.parametrize("order", ["junk_first", "hr_first"])
def test_trainer_accumulation_matches_reference(g1, tmp_path, order):
    """accumulation_steps = 2 on the fused engine, as the reference's loop runs it
    (trainer.py:457-503): batch 1 runs forward + backward and no update, batch 2 back-propagates
    loss / 2 and steps on that gradient alone (the reference zeroes the gradients every batch).
    AdamW's first step is invariant to the 1/2 (m/sqrt(v)), so with G1's batch last the
    parameters land on the reference's single-step parameters (g1 s/); with it first they do
    not.  The gradient the update consumed is half the G1 gradient (power-of-two scale)."""
    import torch.nn as nn
    from src.training import Trainer, TrainerConfig
    m = _config1()
    m.load_state_dict(_sd(g1))
    hr = torch.from_numpy(g1["hr"])
    junk = torch.rand(hr.shape, generator=torch.Generator().manual_seed(99))
    batches = [junk, hr] if order == "junk_first" else [hr, junk]
    cfg = TrainerConfig(learning_rate=1e-4, weight_decay=0.0, gradient_clip=0.5, accumulation_steps=2,
                        use_wandb=False, scheduler_type="none", checkpoint_dir=str(tmp_path))
    tr = Trainer(m, [{"hr": b} for b in batches], None, loss_fn=nn.L1Loss(), config=cfg)
    seen = []
    eng = tr.engine(2, 128, 128)
    run = eng.upd.run

    def upd_run(*a):
        seen.append(eng.flat_g.detach().clone())
        return run(*a)
    eng.upd.run = upd_run
    tr._train_epoch()
    torch.cuda.synchronize()
    assert tr.global_step == 1 and len(seen) == 1
    worst = max(float(np.abs(v.cpu().numpy() - g1["s/" + k]).max()) for k, v in m.state_dict().items())
    if order == "junk_first":
        assert worst <= 2e-5, worst
        off = 0
        for k, p in m.named_parameters():
            g = seen[0][off:off + p.numel()].view_as(p).cpu().double()
            ref = torch.from_numpy(g1["g/" + k]).double() / 2
            off += p.numel()
            assert float((g - ref).norm() / max(ref.norm(), 1e-30)) <= 1e-4, k
    else:
        assert worst >= 1e-4, worst
