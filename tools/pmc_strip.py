"""Launch the bench's dominant kernel REPS times, plainly (no graph), for rocprofv3 passes:
one ResidualGroup on fen_group_strip (10 RCABs + group conv, inference, B=32, 64x64x64, fp16;
PREC=bf16 for bf16), or with CHAIN=6 the body's 6 groups on fen_group_strip_chain, random weights.  Prints the algorithmic bytes per launch: the group input
read once, the group output written once, 21 packed 64->64 filters, the SE weights and biases.
Usage: rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python tools/pmc_strip.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
import torch  # noqa: E402

from src.hip.net import Forward, NetSpec, Weights  # noqa: E402
from src.hip.program import Ctx  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
CHAIN = int(os.environ.get("CHAIN", "0"))      # >0: the body's CHAIN groups as one fen_group_strip_chain launch
dt = torch.bfloat16 if os.environ.get("PREC", "fp16") == "bf16" else torch.float16
B, H, W, C, CR, NB = 32, 64, 64, 64, 16, 10
g = torch.Generator().manual_seed(0)
q = {}
NG = max(CHAIN, 1)
for gi, j in [(gi, j) for gi in range(NG) for j in range(NB)]:
    b = (f"residual_groups.{gi}." if CHAIN else "rg.") + f"blocks.{j}."
    q[b + "conv1.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
    q[b + "conv1.bias"] = torch.randn(C, generator=g) * 0.1
    q[b + "prelu.weight"] = torch.full((C,), 0.25)
    q[b + "conv2.weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.06
    q[b + "conv2.bias"] = torch.randn(C, generator=g) * 0.1
    q[b + "channel_attention.fc.0.weight"] = torch.randn(CR, C, generator=g) * 0.3
    q[b + "channel_attention.fc.2.weight"] = torch.randn(C, CR, generator=g) * 0.3
for pre in ([f"residual_groups.{gi}.conv." for gi in range(NG)] + ["conv_after_body."] if CHAIN else ["rg.conv."]):
    q[pre + "weight"] = torch.randn(C, C, 3, 3, generator=g) * 0.05
    q[pre + "bias"] = torch.randn(C, generator=g) * 0.1
pd = {k: v.cuda() for k, v in q.items()}
ctx = Ctx(dt, "cuda", record=True)
Wt = Weights(pd, dt, "cuda")
x = torch.randn(B, H, W, C, generator=g).to("cuda", dt)
fw = Forward(NetSpec(C=C, G=NG, NB=NB, Cr=CR), ctx, Wt, save=False)
if CHAIN:
    assert fw._chain_ok(x)
    outs = [torch.empty_like(x), torch.empty_like(x)]
    fb = torch.empty_like(x)                  # conv_after_body as the chain's last step
    y, _ = fw.body(x, [outs[gi & 1] for gi in range(NG)], fb=fb)
    assert [op[0] for op in ctx.ops] == ["group_strip_chain"] and fw.fb_done
else:
    assert fw._strip_ok(x)
    y, _ = fw.group(x, 0, pre="rg.")
for _ in range(REPS):
    ctx.run()
torch.cuda.synchronize()
# the input read and the (last) output written once, every group's filters, SE weights and biases
alg = 2 * x.numel() * 2 + NG * ((2 * NB + 1) * 9 * C * C * 2 + NB * 2 * CR * C * 4 + (3 * NB + 1) * C * 4)
if CHAIN:   # + conv_after_body: its filter and bias, its output written (the body output is then internal)
    alg += 9 * C * C * 2 + C * 4
print("algorithmic_bytes_per_launch", alg)
