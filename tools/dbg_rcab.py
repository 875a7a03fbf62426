import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import numpy as np, torch
from src.hip.net import Backward, Forward, NetSpec, Weights
from src.hip.program import Ctx
from oracle import fen_oracle as O
g = dict(np.load('tests/golden/g2_rcab.npz'))
P = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith('p/')}
def rel(a, b): return float((a.double()-b.double()).norm()/b.double().norm())
for dtype in (torch.float32, torch.bfloat16):
    p = {k: v.cuda() for k, v in P.items()}
    spec = NetSpec(C=64, G=1, NB=1, Cr=16)
    ctx = Ctx(dtype, 'cuda'); Wt = Weights(p, dtype, 'cuda')
    x = torch.from_numpy(g['x']).permute(0,2,3,1).contiguous().cuda().to(dtype)
    y, sv = Forward(spec, ctx, Wt, save=True).rcab(x, '')
    r = torch.from_numpy(g['r']).permute(0,2,3,1).contiguous().cuda().to(dtype)
    G = {k: torch.zeros_like(v) for k, v in p.items()}
    dx = Backward(spec, ctx, Wt, G).rcab(sv, r, '')
    torch.cuda.synchronize()
    # oracle run on the *rounded* inputs for bf16 to separate input rounding from kernel error
    xr = x.float().cpu().permute(0,3,1,2); rr = r.float().cpu().permute(0,3,1,2)
    out_o, dx_o, g_o = O.rcab_with_grads(P, xr, rr)
    print(dtype, 'out', rel(y.float().cpu().permute(0,3,1,2), torch.from_numpy(g['out'])), 'vs rounded-input oracle', rel(y.float().cpu().permute(0,3,1,2), out_o))
    print('  dx', rel(dx.float().cpu().permute(0,3,1,2), torch.from_numpy(g['dx'])), rel(dx.float().cpu().permute(0,3,1,2), dx_o))
    for k in G: print('  ', k, rel(G[k].cpu(), torch.from_numpy(g['g/'+k])), rel(G[k].cpu(), g_o[k]))
