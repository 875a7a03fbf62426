"""Probe: can the stage-3 GAN iteration (Trainer._gan_step, module autograd path, B=16) be
captured into one hipGraph?  Two trainers from the same seeds: A runs N eager steps; B runs 2
eager warm-ups, captures one step and replays it N-2 times.  Prints the per-iteration times
and the largest parameter differences between A and B (generator flat arena, discriminator)."""
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from src.losses import create_loss_function  # noqa: E402
from src.models import GANLoss, VGGStyleDiscriminator  # noqa: E402
from src.training import Trainer, TrainerConfig  # noqa: E402

N = int(os.environ.get("N", "8"))
B = 16


def trainer():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        loss_fn = create_loss_function(l1_weight=0.01, perceptual_weight=1.0, ssim_weight=0.0,
                                       perceptual_layers=["conv3_4"])
    torch.manual_seed(7)
    D = VGGStyleDiscriminator(input_size=256, precision="bf16")
    cfg = TrainerConfig(learning_rate=1e-4, weight_decay=0.0, gradient_clip=0.5, gan_weight=0.005,
                        d_learning_rate=1e-4, use_wandb=False, scheduler_type="none",
                        checkpoint_dir="/tmp/fen_probe_ckpt")
    tr = Trainer(bench.build_model("bf16"), [], None, loss_fn=loss_fn, config=cfg, discriminator=D,
                 gan_loss=GANLoss("vanilla"))
    for g in tr.optimizer_d.param_groups:
        g["capturable"] = True
    return tr


def diffs(X, Y):
    dg = float((X.model._fen_flat - Y.model._fen_flat).abs().max())
    dd = max(float((p.detach() - q.detach()).abs().max())
             for p, q in zip(X.discriminator.parameters(), Y.discriminator.parameters()))
    db = max(float((p - q).abs().max()) for p, q in zip(X.discriminator.buffers(), Y.discriminator.buffers())
             if p.is_floating_point())
    return dg, dd, db


hr = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(99)).cuda()
# determinism of the eager path: two trainers, the same 3 steps; then C with every weight
# re-packed on use (as inside a capture) against A
import src.hip.autograd as _ag  # noqa: E402
import src.models.discriminator as _dm  # noqa: E402
A, C = trainer(), trainer()
for _ in range(3):
    A._gan_step(hr)
    C._gan_step(hr)
torch.cuda.synchronize()
print("eager vs eager after 3 steps (max |dG|, |dD|, |dD buffers|):", diffs(A, C), flush=True)
C2 = trainer()
_ag._FORCE_REPACK = _dm._FORCE_REPACK = True
for _ in range(3):
    C2._gan_step(hr)
_ag._FORCE_REPACK = _dm._FORCE_REPACK = False
torch.cuda.synchronize()
print("eager vs eager-repacking after 3 steps (0 = the version-keyed caches are fresh):", diffs(A, C2), flush=True)
# captured: B warms up 2 eager steps (as A's first 2), captures one step, replays it once -> A's step 3
Bt = trainer()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        Bt._gan_step(hr)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    lb = Bt._gan_step(hr)
g.replay()
torch.cuda.synchronize()
print("replay-1 vs eager step 3:", diffs(A, Bt), flush=True)
for _ in range(N):
    A._gan_step(hr)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    la = A._gan_step(hr)
torch.cuda.synchronize()
print("eager ms/iter", round(1000 * (time.perf_counter() - t0) / N, 3), flush=True)
t0 = time.perf_counter()
for _ in range(N):
    g.replay()
torch.cuda.synchronize()
print("replay ms/iter", round(1000 * (time.perf_counter() - t0) / N, 3), "loss", float(lb), flush=True)
