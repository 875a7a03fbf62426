"""Device data path throughput: 256x256x3 uint8 images, B=32, P=256 (the FFHQ-256 training
shape): img/s of the whole pipeline (host gather into pinned staging + async H2D + augment
kernel) and of the augment kernel alone (GB/s vs the 8 TB/s HBM roofline)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'face-super-resolution_amd'))
import numpy as np
import torch
from src.data.device_loader import DeviceHRLoader
from src.hip import lib as L
from src.hip.program import ptr
B, P = 32, 256
rng = np.random.default_rng(0)
imgs = [rng.integers(0, 256, (P, P, 3), dtype=np.uint8) for _ in range(8 * B)]
ld = DeviceHRLoader(imgs, B, P, color_jitter_prob=0.3, saturation=0.0, seed=1)
out = torch.empty(B, 3, P, P, device="cuda")
for _ in ld.batches(out=out):
    pass
torch.cuda.synchronize()
t0 = time.perf_counter()
n = 0
for _ in range(3):
    for _ in ld.batches(out=out):
        n += B
torch.cuda.synchronize()
el = time.perf_counter() - t0
lib = L.load()
s = torch.cuda.current_stream().cuda_stream
f = lambda: L.check(lib.fen_augment_u8(B, P, ptr(ld.dev[0]), ptr(ld.dparams[0]), ptr(ld.sums), ptr(out), s), "aug")
for _ in range(5): f()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): f()
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 50
nbytes = 2 * B * P * P * 3 + B * 3 * P * P * 4          # uint8 read twice (sum + transform), fp32 write
print(json.dumps({"pipeline_img_s": round(n / el, 1), "kernel_us": round(us, 2),
                  "kernel_GBs": round(nbytes / us / 1e3, 1), "batch": B, "patch": P}))
