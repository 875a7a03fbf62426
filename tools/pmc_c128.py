"""One 128-channel ResidualGroup on fen_rcab_c128 (BASELINE configs[4] shape: B=4, 128x128x128,
fp16; NB=2 RCABs + the group conv = 5 launches) run eagerly REPS times, random weights, for
rocprofv3 --pmc passes on k_rcab128 (modes 1 with the deferred gate, 2, 3).
Usage: rocprofv3 --pmc SQ_... -d DIR -o run --output-format csv -- python tools/pmc_c128.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402

from src.hip.net import Forward, NetSpec, Weights  # noqa: E402
from src.hip.program import Ctx  # noqa: E402

REPS = int(os.environ.get("REPS", "10"))
B, H, W, C, CR, NB = 4, 128, 128, 128, 32, 2
g = torch.Generator().manual_seed(0)
q = {}
for j in range(NB):
    b = f"rg.blocks.{j}."
    q[b + "conv1.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.04
    q[b + "conv1.bias"] = torch.randn(C, generator=g) * 0.1
    q[b + "prelu.weight"] = torch.full((C,), 0.25)
    q[b + "conv2.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.04
    q[b + "conv2.bias"] = torch.randn(C, generator=g) * 0.1
    q[b + "channel_attention.fc.0.weight"] = torch.randn(CR, C, generator=g) * 0.2
    q[b + "channel_attention.fc.2.weight"] = torch.randn(C, CR, generator=g) * 0.3
q["rg.conv.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.035
q["rg.conv.bias"] = torch.randn(C, generator=g) * 0.1
pd = {k: v.cuda() for k, v in q.items()}
ctx = Ctx(torch.float16, "cuda", record=True)
Wt = Weights(pd, torch.float16, "cuda")
x = torch.randn(B, H, W, C, generator=g).to("cuda", torch.float16)
fw = Forward(NetSpec(C=C, G=1, NB=NB, Cr=CR), ctx, Wt, save=False)
assert fw._c128_ok(x)
y, _ = fw.group(x, 0, pre="rg.")
for _ in range(REPS):
    ctx.run()
torch.cuda.synchronize()
print("ops", [o[0] for o in ctx.ops])
