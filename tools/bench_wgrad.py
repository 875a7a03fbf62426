"""Microbenchmark of the batched weight gradient (fen_wgrad3x3_multi: k_wgrad_p<64> + k_wgrad_fin)
at the strip backward's shape: NJOBS (default 21) 64->64 convs, bf16, B=32, 64x64.  Load a
variant library with FEN_HIP_LIB.  Prints one JSON line (us per multi launch, GFLOP/s)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import torch  # noqa: E402
from src.hip import lib as L  # noqa: E402

n = int(os.environ.get("NJOBS", "21"))
B, H, W, C = 32, 64, 64, 64
g = torch.Generator(device="cuda").manual_seed(0)
xs = [torch.randn(B, H, W, C, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(n)]
dys = [torch.randn(B, H, W, C, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(n)]
dws = [torch.empty(C, C, 3, 3, device="cuda") for _ in range(n)]
dbs = [torch.empty(C, device="cuda") for _ in range(n)]
arr = (L.WgradDesc * n)()
for i in range(n):
    d = arr[i]
    d.dtype, d.B, d.H, d.W, d.Cin, d.Cout, d.cout_valid = L.dtype_code(torch.bfloat16), B, H, W, C, C, C
    d.x, d.dy, d.dw, d.db, d.accumulate = xs[i].data_ptr(), dys[i].data_ptr(), dws[i].data_ptr(), dbs[i].data_ptr(), 0
lib = L.load()
nwork = lib.fen_wgrad_multi_work_floats(n, ctypes.cast(arr, ctypes.c_void_p))
work = torch.empty(nwork, device="cuda")
arr[0].work = work.data_ptr()


def launch():
    s = torch.cuda.current_stream().cuda_stream
    L.check(lib.fen_wgrad3x3_multi(n, ctypes.cast(arr, ctypes.c_void_p), ctypes.c_void_p(s)), "wgrad_multi")


for _ in range(2):
    launch()
torch.cuda.synchronize()
# check job 0 against torch (fp32 conv weight gradient of the same bf16 operands)
x0 = xs[0].float().permute(0, 3, 1, 2)
dy0 = dys[0].float().permute(0, 3, 1, 2)
ref = torch.nn.grad.conv2d_weight(x0, (C, C, 3, 3), dy0, padding=1)
rel = float((dws[0] - ref).abs().max() / ref.abs().max())
reps = 10
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(reps):
        launch()
gr.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e30
for _ in range(5):
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
flop = 2.0 * B * H * W * C * C * 9 * n
print(json.dumps({"lib": os.path.basename(L.LIB_PATH), "jobs": n, "us": round(best, 2),
                  "tflops": round(flop / best / 1e6, 1), "rel_err_job0": rel}))
