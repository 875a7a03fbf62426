import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch, torch.nn.functional as F
from src.hip import lib as L, net
from src.hip.program import Ctx, ptr
torch.manual_seed(0)
B,H,W,C = 2,16,16,64
def rel(a,b): return float((a.double()-b.double()).norm()/b.double().norm())
for dtype in (torch.float32, torch.bfloat16):
    dt = torch.randn(B,C,H,W).to(dtype).double()
    w = (torch.randn(C,C,3,3)*0.05).to(dtype).double()
    z = torch.randn(B,C,H,W).to(dtype).double()
    a = torch.rand(C).double()*0.5
    da = F.conv_transpose2d(dt, w, padding=1)
    dz = torch.where(z>0, da, da*a.view(1,-1,1,1))
    ctx = Ctx(dtype, 'cuda')
    n = ctx.lib.fen_packed_elems(2, C, C); wp = torch.empty(n, dtype=dtype, device='cuda'); wd = w.float().cuda()
    ctx.emit('p', ctx.lib.fen_pack_conv_w, ctx.code, 2, C, C, ptr(wd), ptr(wp))
    nh = lambda t: t.permute(0,2,3,1).contiguous().cuda().to(dtype)
    y = ctx.alloc((B,H,W,C)); part = ctx.alloc((B*net.tiles(H,W), C), torch.float32)
    net.conv(ctx, nh(dt), wp, B,H,W,C,C, epi=L.EPI_PRELU_BWD, alpha=a.float().cuda(), pre_in=nh(z), y=y, part=part)
    y2 = ctx.alloc((B,H,W,C))
    net.conv(ctx, nh(dt), wp, B,H,W,C,C, y=y2)
    torch.cuda.synchronize()
    yc = y.double().cpu().permute(0,3,1,2); y2c = y2.double().cpu().permute(0,3,1,2)
    print(dtype, 'dgrad plain rel', rel(y2c, da), 'prelu_bwd rel', rel(yc, dz), 'maxabs', float((yc-dz).abs().max()), float(dz.abs().max()))
    # also the forward plain conv with same rounding
    y3 = ctx.alloc((B,H,W,C)); n0 = ctx.lib.fen_packed_elems(0, C, C); wp0 = torch.empty(n0, dtype=dtype, device='cuda')
    ctx.emit('p', ctx.lib.fen_pack_conv_w, ctx.code, 0, C, C, ptr(wd), ptr(wp0))
    net.conv(ctx, nh(dt), wp0, B,H,W,C,C, y=y3); torch.cuda.synchronize()
    print('   fwd plain rel', rel(y3.double().cpu().permute(0,3,1,2), F.conv2d(dt, w, padding=1)))
