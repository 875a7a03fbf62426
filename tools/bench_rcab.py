"""Fused RCAB (fen_rcab_fused) vs the per-op launches, B=32 64x64x64 bf16, graph-replayed.
Prints one JSON line: us per RCAB block and TFLOP/s on the algorithmic 19.33 GFLOP."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch
from src.hip import net
from src.hip.net import Forward, NetSpec, Weights
from src.hip.program import Ctx

B = int(os.environ.get("B", "32"))
torch.manual_seed(0)
p = {"conv1.weight": torch.randn(64, 64, 3, 3) * 0.06, "conv1.bias": torch.zeros(64), "prelu.weight": torch.full((64,), .25),
     "conv2.weight": torch.randn(64, 64, 3, 3) * 0.06, "conv2.bias": torch.zeros(64),
     "channel_attention.fc.0.weight": torch.randn(16, 64) * .3, "channel_attention.fc.2.weight": torch.randn(64, 16) * .3}
pd = {k: v.cuda() for k, v in p.items()}
x = torch.randn(B, 64, 64, 64, device='cuda', dtype=torch.bfloat16)
res = {"B": B}
for fused in (True, False):
    for train in (False, True):
        net.FUSED_RCAB = fused
        ctx = Ctx(torch.bfloat16, 'cuda', record=True)
        Wt = Weights(pd, torch.bfloat16, 'cuda')
        fw = Forward(NetSpec(C=64, G=1, NB=1, Cr=16), ctx, Wt, save=train)
        h = x
        for i in range(10):
            h, _ = fw.rcab(h, "", out=ctx.scratch(f"pp{i & 1}", x.shape))
        for _ in range(2): ctx.run()
        torch.cuda.synchronize()
        print("eager ok", fused, train, flush=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ctx.run()
        g.replay(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5): g.replay()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        key = ("fused" if fused else "perop") + ("_train" if train else "")
        print(key, round(us, 2), flush=True)
        res[key + "_us"] = round(us, 2)
        res[key + "_tflops"] = round(19.327e9 * B / 32 / us / 1e6, 1)
print(json.dumps(res))
