"""Which bf16 rounding costs the PSNR parity?  CPU emulation of the HIP bf16 forward (oracle
ops with bf16 rounding inserted where the kernels store bf16: activations AND weights), trunk in
bf16 vs in fp32.  (The weights-only effect -- activations fp32 -- is the CPU test
tests/test_oracle.py::test_bf16_weight_rounding_alone_exceeds_001db: -0.0187 dB bf16 vs
-0.0009 dB fp16 on g9.)

  python tools/numerics_bf16.py            # g4 (32x32 noise, bicubic target) + smooth 64x64 (HR target)
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import fen_oracle as O  # noqa: E402

torch.set_num_threads(8)


def r(x):
    return x.to(torch.bfloat16).to(torch.float32)


def conv(x, w, b):
    return F.conv2d(r(x), r(w), b, padding=1)


def fwd(p, x, trunk_fp32, t_round=True):
    bic = O.bicubic(x, 4)
    feat = r(F.conv2d(x, p["conv_first.weight"], p["conv_first.bias"], padding=1))
    res = feat
    tr = (lambda v: v) if trunk_fp32 else r
    for g in range(6):
        pre = f"residual_groups.{g}."
        h = feat
        for b in range(10):
            q = f"{pre}blocks.{b}."
            z = conv(h, p[q + "conv1.weight"], p[q + "conv1.bias"])
            a = r(O.prelu(z, p[q + "prelu.weight"]))
            t = conv(a, p[q + "conv2.weight"], p[q + "conv2.bias"])
            s = O.channel_attention(t, p, q + "channel_attention.")
            tt = r(t) if t_round else t
            h = tr(tt * s[:, :, None, None] * 0.2 + h)
        feat = tr(conv(h, p[pre + "conv.weight"], p[pre + "conv.bias"]) + feat)
    feat = r(conv(feat, p["conv_after_body.weight"], p["conv_after_body.bias"]) + res)
    for st in range(2):
        pre = f"upsample.stages.{st}."
        feat = r(O.prelu(O.pixel_shuffle(conv(feat, p[pre + "conv.weight"], p[pre + "conv.bias"]), 2),
                         p[pre + "prelu.weight"]))
    out = conv(feat, p["conv_last.weight"], p["conv_last.bias"]) + bic
    return out.clamp(0, 1)


def seeded_params():
    from src.models import FaceEnhanceNet
    torch.manual_seed(0)
    m = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, reduction_ratio=4, scale_factor=4,
                       precision="fp32")
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=g) * 1e-3)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def smooth_hr(B, H, W, seed):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from smooth import smooth_images
    return smooth_images(B, H, W, seed)


def main():
    p = seeded_params()
    shape = O.NetShape(64, 6, 10, 4, 4, 0.2)
    cases = []
    g4 = np.load(os.path.join(ROOT, "tests/golden/g4_full.npz"))
    x4 = torch.from_numpy(g4["x"])
    cases.append(("g4 32x32 noise, target bicubic(x)", x4, O.bicubic(x4.double(), 4).clamp(0, 1)))
    hr = smooth_hr(2, 256, 256, 11)
    cases.append(("smooth 64x64 B=2, target HR", O.lr_from_hr(hr), hr))
    for name, x, tgt in cases:
        with torch.no_grad():
            ref = O.forward(p, x, shape, training=False)
            base = O.psnr(ref, tgt)
            print(f"{name}: ref psnr {base:.4f} dB")
            for label, kw in (("bf16 trunk", dict(trunk_fp32=False)), ("fp32 trunk", dict(trunk_fp32=True)),
                              ("fp32 trunk, t unrounded", dict(trunk_fp32=True, t_round=False))):
                out = fwd(p, x, **kw)
                print(f"   {label:24s} dPSNR {O.psnr(out, tgt) - base:+.5f} dB  max|d| {float((out - ref).abs().max()):.2e}")


if __name__ == "__main__":
    main()
