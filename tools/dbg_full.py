import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch, numpy as np
from src.models import FaceEnhanceNet
from src.hip.net import Forward, NetSpec, Weights
from src.hip.program import Ctx
from oracle import fen_oracle as O
torch.manual_seed(0)
m = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10)
gen = torch.Generator().manual_seed(1)
with torch.no_grad(): m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=gen)*1e-3)
sd = {k: v.detach().clone() for k,v in m.state_dict().items()}
x = torch.rand(1,3,32,32, generator=torch.Generator().manual_seed(4))
pd = {k: v.cuda() for k,v in sd.items()}
spec = NetSpec(C=64, G=6, NB=10, Cr=16)
for save in (False, True):
    ctx = Ctx(torch.float32, 'cuda'); Wt = Weights(pd, torch.float32, 'cuda')
    fw = Forward(spec, ctx, Wt, save=save)
    xd = x.cuda()
    f0 = fw.head(xd)
    ref0 = torch.nn.functional.conv2d(x, sd['conv_first.weight'], sd['conv_first.bias'], padding=1)
    nh = lambda t: t.float().cpu().permute(0,3,1,2)
    print('save', save, 'head', float((nh(f0)-ref0).abs().max()))
    h, hr = f0, ref0
    for g in range(6):
        # block-by-block within group
        pre = f'residual_groups.{g}.'
        hb, hbr = h, hr
        for b in range(10):
            hb, _ = fw.rcab(hb, f'{pre}blocks.{b}.')
            hbr = O.rcab(hbr, sd, f'{pre}blocks.{b}.', 0.2)
            e = float((nh(hb)-hbr).abs().max())
            if e > 1e-4: print('  g',g,'b',b,'err',e, 'mag', float(hbr.abs().max()))
        h, _ = fw.group(h, g)
        hr = O.residual_group(hr, sd, pre, 10, 0.2)
        print(' group', g, float((nh(h)-hr).abs().max()), float(hr.abs().max()))
    torch.cuda.synchronize()
