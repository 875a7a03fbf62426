"""PSNR parity spread of the bf16 full network (g4 golden) for the fused / per-op RCAB paths."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import numpy as np, torch
from oracle import fen_oracle as O
from src.hip import net
from src.models import FaceEnhanceNet
g = dict(np.load(os.path.join(ROOT, "tests/golden/g4_full.npz")))
x = torch.from_numpy(g["x"]).cuda()
ref_e = torch.from_numpy(g["out_eval"])


def seeded():
    torch.manual_seed(0)
    m = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, reduction_ratio=4, scale_factor=4,
                       precision="bf16")
    gg = torch.Generator().manual_seed(1)
    with torch.no_grad():
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=gg) * 1e-3)
    return m


for fused in (True, False):
    net.FUSED_RCAB = fused
    m = seeded().cuda().eval()
    with torch.no_grad():
        out = m(x).cpu()
    tgt = O.bicubic(x.cpu().double(), m.scale_factor).clamp(0, 1)
    print("fused" if fused else "perop", "psnr", O.psnr(out, tgt), "ref", O.psnr(ref_e, tgt),
          "d", abs(O.psnr(out, tgt) - O.psnr(ref_e, tgt)), "maxabs", float((out - ref_e).abs().max()))
