"""Golden-vector generator (test infrastructure; runs ONLY in the survey container).

Imports the reference implementation from /root/reference (read-only, no bytecode
written) and records numeric input/output fixtures for the FaceEnhanceNet hot path
into tests/golden/*.npz.  Nothing from the reference travels except these numbers.

Fixtures:
  g1_config1.npz  config 1 (C=64, 1 group x 2 RCAB, x4), B=2, HR 128x128 -> LR 32x32:
                  seed-0 reference init (+ conv_last ~ N(0,1e-3) so the body is exercised),
                  train/eval forward, attention maps, L1 grads of every parameter,
                  parameters after one Trainer._train_epoch step (AdamW, clip 0.5).
  g2_rcab.npz     one RCAB (C=64) B=2 16x16 with random weights; out and all grads
                  of sum(out*R).
  g3_kat.npz      bicubic x2/x4/x8 up, bicubic x0.25 down, PixelShuffle(2) KATs.
  g4_full.npz     full 6x10 network, B=1, 32x32 input: init statistics + outputs
                  (fp32, and the eval output of the reference run in float64).
  g5_c128.npz     128-ch 10x20 x8 variant, B=1, 16x16 input: init statistics + output.
  g6_lite.npz     FaceEnhanceNetLite (C=32, r=2), B=1, 16x16 input: output.
  g9_full64.npz   full 6x10 network at the north-star shape: B=2, smooth uint8 HR 256x256
                  (tests/golden/smooth.py, seed 11) -> LR 64x64 by the reference's own
                  bicubic /4; init statistics, eval/train outputs, the eval output of the
                  reference run in float64, and its PSNR vs HR (trainer.py:621-628).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [g1 g2 ... g9]
"""
import copy
import os
import sys
import tempfile

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.dont_write_bytecode = True
REF = os.environ.get("FEN_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from src.models.custom import FaceEnhanceNet, FaceEnhanceNetLite  # noqa: E402  (reference)
from src.models.blocks import RCAB  # noqa: E402  (reference)

OUT = os.path.dirname(os.path.abspath(__file__))
torch.set_num_threads(8)


def sd_np(model, prefix="p/"):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def init_stats(model):
    names, s1, s2 = [], [], []
    for k, v in model.state_dict().items():
        v64 = v.detach().double()
        names.append(k)
        s1.append(float(v64.sum()))
        s2.append(float((v64 * v64).sum()))
    return {"stat_names": np.array(names), "stat_sum": np.array(s1), "stat_sumsq": np.array(s2)}


def perturb_conv_last(model, seed=1):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        model.conv_last.weight.copy_(torch.randn(model.conv_last.weight.shape, generator=g) * 1e-3)


class _L1(nn.Module):
    """Loss module with the (loss, components) contract Trainer expects (trainer.py:465)."""

    def forward(self, sr, hr):
        loss = F.l1_loss(sr, hr)
        return loss, {"l1": loss.detach()}


def g1():
    torch.manual_seed(0)
    model = FaceEnhanceNet(num_channels=64, num_groups=1, blocks_per_group=2,
                           reduction_ratio=4, scale_factor=4, res_scale=0.2)
    d = {}
    d.update(init_stats(model))
    perturb_conv_last(model, 1)
    d.update(sd_np(model, "p/"))
    hr = torch.rand(2, 3, 128, 128, generator=torch.Generator().manual_seed(2))
    lr = F.interpolate(hr, scale_factor=0.25, mode="bicubic", align_corners=False)
    d["hr"] = hr.numpy()
    d["lr"] = lr.numpy()
    model.train()
    with torch.no_grad():
        d["out_train"] = model(lr).numpy()
    model.eval()
    with torch.no_grad():
        d["out_eval"] = model(lr).numpy()
    attn = model.get_attention_maps(lr)
    for k, v in attn.items():
        d["attn/" + k] = v.numpy()
    # L1 gradients of every parameter (train mode, reference autograd)
    model.train()
    model.zero_grad()
    out = model(lr)
    loss = F.l1_loss(out, hr)
    loss.backward()
    d["l1_loss"] = np.array(float(loss))
    for k, p in model.named_parameters():
        d["g/" + k] = p.grad.detach().numpy().copy()
    # one step of the reference Trainer (trainer.py:390-550): AdamW + clip 0.5, fp32
    model.zero_grad()
    import src.training.trainer as T  # reference
    with tempfile.TemporaryDirectory() as tmp:
        cfg = T.TrainerConfig(learning_rate=1e-4, weight_decay=0.0, gradient_clip=0.5,
                              use_amp=False, use_wandb=False, device="cpu",
                              checkpoint_dir=tmp)
        tr = T.Trainer(model, [{"hr": hr}], [{"hr": hr}], _L1(), cfg)
        m = tr._train_epoch()
    d["step_loss"] = np.array(float(m["loss"]))
    for k, v in model.state_dict().items():
        d["s/" + k] = v.detach().numpy().copy()
    np.savez_compressed(os.path.join(OUT, "g1_config1.npz"), **d)


def g2():
    torch.manual_seed(3)
    rcab = RCAB(64, 3, 4, True, 0.2)
    with torch.no_grad():
        rcab.prelu.weight.copy_(0.25 + 0.2 * torch.randn(64))
        rcab.conv1.bias.copy_(0.05 * torch.randn(64))
        rcab.conv2.bias.copy_(0.05 * torch.randn(64))
    x = torch.randn(2, 64, 16, 16, requires_grad=True)
    r = torch.randn(2, 64, 16, 16)
    out = rcab(x)
    (out * r).sum().backward()
    d = {"x": x.detach().numpy(), "r": r.numpy(), "out": out.detach().numpy(), "dx": x.grad.numpy()}
    for k, v in rcab.state_dict().items():
        d["p/" + k] = v.numpy().copy()
    for k, p in rcab.named_parameters():
        d["g/" + k] = p.grad.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "g2_rcab.npz"), **d)


def g3():
    g = torch.Generator().manual_seed(5)
    d = {}
    x = torch.rand(2, 3, 8, 8, generator=g)
    d["up_in"] = x.numpy()
    for s in (2, 4, 8):
        d[f"up_x{s}"] = F.interpolate(x, scale_factor=s, mode="bicubic", align_corners=False).numpy()
    hr = torch.rand(2, 3, 32, 32, generator=g)
    d["down_in"] = hr.numpy()
    d["down_x4"] = F.interpolate(hr, scale_factor=0.25, mode="bicubic", align_corners=False).numpy()
    ps = torch.arange(2 * 8 * 3 * 5, dtype=torch.float32).reshape(2, 8, 3, 5)
    d["ps_in"] = ps.numpy()
    d["ps_out"] = nn.PixelShuffle(2)(ps).numpy()
    np.savez_compressed(os.path.join(OUT, "g3_kat.npz"), **d)


def g_net(fname, ctor, x_shape, seed_x):
    torch.manual_seed(0)
    model = ctor()
    d = init_stats(model)
    perturb_conv_last(model, 1)
    x = torch.rand(*x_shape, generator=torch.Generator().manual_seed(seed_x))
    d["x"] = x.numpy()
    with torch.no_grad():
        model.eval()
        d["out_eval"] = model(x).numpy()
        model.train()
        d["out_train"] = model(x).numpy()
        # the reference evaluated in float64: the accuracy yardstick for deep variants whose
        # fp32 rounding alone exceeds 1e-3 (e.g. 128 ch x 200 RCAB)
        model.double().eval()
        d["out_eval_f64"] = model(x.double()).numpy()
    np.savez_compressed(os.path.join(OUT, fname), **d)


def g9():
    sys.path.insert(0, OUT)
    from smooth import smooth_images_u8
    torch.manual_seed(0)
    model = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, reduction_ratio=4, scale_factor=4)
    d = init_stats(model)
    perturb_conv_last(model, 1)
    hr_u8 = smooth_images_u8(2, 256, 256, 11)
    hr = torch.from_numpy(hr_u8.astype(np.float32) / np.float32(255.0))
    lr = F.interpolate(hr, scale_factor=0.25, mode="bicubic", align_corners=False)   # trainer.py:416-421
    d["hr_u8"], d["lr"] = hr_u8, lr.numpy()
    with torch.no_grad():
        model.eval()
        d["out_eval"] = model(lr).numpy()
        model.train()
        d["out_train"] = model(lr).numpy()
        model.double().eval()
        f64 = model(lr.double())
        d["out_eval_f64"] = f64.float().numpy()
        mse = torch.mean((f64 - hr.double()) ** 2)
        d["psnr_eval_f64"] = np.array(float(10.0 * torch.log10(1.0 / mse)))
    np.savez_compressed(os.path.join(OUT, "g9_full64.npz"), **d)


# g10: tensors kept whole (the rest of the 5.1 M parameters are pinned by projections): the
# first and last RCAB, every group conv, the upsampler, conv_first, conv_last, conv_after_body
G10_FULL = ("conv_first.", "residual_groups.0.blocks.0.", "residual_groups.5.blocks.9.",
            "conv_after_body.", "upsample.", "conv_last.") + tuple(f"residual_groups.{g}.conv." for g in range(6))
G10_NPROJ = 4


def g10_full(name):
    return name.startswith(G10_FULL)


def g10_proj(index, arr):
    """G10_NPROJ seeded Gaussian projections of a tensor (float64) -- regenerated identically by
    the GPU test from (index, numel)."""
    r = np.random.default_rng(1000 + index).standard_normal((G10_NPROJ, arr.size))
    return r @ arr.astype(np.float64).ravel()


def g10():
    """Training at the north-star shape: g9's network, batch and HR (6x10, 64x64 -> 256x256,
    B=2).  The L1 gradient of every parameter in train mode (reference autograd, fp32, and the
    same in float64 as the accuracy yardstick), and the parameters after one reference
    Trainer._train_epoch step (trainer.py:458-503: AdamW lr 1e-4, clip 0.5).  Whole tensors
    for G10_FULL, seeded projections + norms for every tensor."""
    sys.path.insert(0, OUT)
    from smooth import smooth_images_u8
    torch.manual_seed(0)
    model = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, reduction_ratio=4, scale_factor=4)
    d = init_stats(model)
    perturb_conv_last(model, 1)
    hr_u8 = smooth_images_u8(2, 256, 256, 11)
    hr = torch.from_numpy(hr_u8.astype(np.float32) / np.float32(255.0))
    lr = F.interpolate(hr, scale_factor=0.25, mode="bicubic", align_corners=False)
    d["hr_u8"] = hr_u8
    names = [k for k, _ in model.named_parameters()]
    d["names"] = np.array(names)
    pre = {k: p.detach().clone() for k, p in model.named_parameters()}

    def grads(m, x, y):
        m.train()
        m.zero_grad()
        loss = F.l1_loss(m(x), y)
        loss.backward()
        return float(loss), {k: p.grad.detach().clone() for k, p in m.named_parameters()}

    loss32, g32 = grads(model, lr, hr)
    m64 = copy.deepcopy(model).double()
    loss64, g64 = grads(m64, lr.double(), hr.double())
    d["l1_loss"], d["l1_loss_f64"] = np.array(loss32), np.array(loss64)
    for i, k in enumerate(names):
        a32, a64 = g32[k].numpy(), g64[k].numpy()
        d["gproj/" + k] = g10_proj(i, a32)
        d["gproj64/" + k] = g10_proj(i, a64)
        d["gnorm/" + k] = np.array(np.linalg.norm(a32.astype(np.float64)))
        d["gerr64/" + k] = np.array(np.linalg.norm(a32.astype(np.float64) - a64))   # the reference's own fp32 error
        if g10_full(k):
            d["g/" + k] = a32
    model.zero_grad()
    import src.training.trainer as T  # reference
    with tempfile.TemporaryDirectory() as tmp:
        cfg = T.TrainerConfig(learning_rate=1e-4, weight_decay=0.0, gradient_clip=0.5,
                              use_amp=False, use_wandb=False, device="cpu", checkpoint_dir=tmp)
        tr = T.Trainer(model, [{"hr": hr}], [{"hr": hr}], _L1(), cfg)
        m = tr._train_epoch()
    d["step_loss"] = np.array(float(m["loss"]))
    for i, (k, p) in enumerate(model.named_parameters()):
        delta = (p.detach() - pre[k]).numpy()
        d["sproj/" + k] = g10_proj(i, delta)
        d["snorm/" + k] = np.array(np.linalg.norm(delta.astype(np.float64)))
        if g10_full(k):
            d["s/" + k] = p.detach().numpy().copy()
    np.savez_compressed(os.path.join(OUT, "g10_train64.npz"), **d)


ALL = {
    "g1": g1, "g2": g2, "g3": g3, "g10": g10,
    "g4": lambda: g_net("g4_full.npz", lambda: FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10,
                                                              reduction_ratio=4, scale_factor=4), (1, 3, 32, 32), 4),
    "g5": lambda: g_net("g5_c128.npz", lambda: FaceEnhanceNet(num_channels=128, num_groups=10, blocks_per_group=20,
                                                              reduction_ratio=4, scale_factor=8), (1, 3, 16, 16), 6),
    "g6": lambda: g_net("g6_lite.npz", lambda: FaceEnhanceNetLite(), (1, 3, 16, 16), 7),
    "g9": g9,
}

if __name__ == "__main__":
    for name in (sys.argv[1:] or list(ALL)):
        ALL[name]()
    print("golden fixtures written to", OUT)
