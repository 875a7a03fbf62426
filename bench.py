#!/usr/bin/env python
"""FaceEnhanceNet 64->256 (x4) super-resolution throughput on MI355X.

Metric (BASELINE.json): images/sec at batch 32 per GPU on 1/2/4/8 GPUs; PSNR vs ref.  The
workload of `value` is BASELINE configs[1]: the full network (6 groups x 10 RCAB, 64 ch),
inference, batch 32 per GPU, synthetic 64x64x3 inputs resident in HBM (the bicubic /4 of
smooth synthetic 256x256 HR images, tests/golden/smooth.py), random-init weights of the
reference architecture (seeded reference init + conv_last ~ N(0,1e-3)).  One "step" = one
forward of one 32-image batch, replayed from a hipGraph.  With N>1 each rank runs its own
replica on its own shard (inference has no exchange step: weak scaling).

16-bit format: `value` runs in fp16 (--precision), the reference's own mixed-precision
dtype, at the same MFMA peak as bf16; the metric's "PSNR vs ref" clause (within 0.01 dB,
north_star) holds in fp16 (measured ~0.002 dB) but not in bf16 (~0.012 dB: bf16's 8-bit
mantissa on the weights alone moves this net's PSNR by that much).
The bf16 run of the same workload is reported beside it ("bf16"), with its own parity.
psnr_parity: PSNR of the GPU output and of the CPU oracle's fp32 output (the cpu_baseline
leg's B=32 pass over the same batch) against the HR images, trainer.py:621-628.

Also reported (field "train"): the stage-1 generator training step (bicubic /4 LR
synthesis, forward, L1, backward, RCCL gradient all-reduce over xGMI for N>1, clip,
AdamW) at batch 32 per GPU -- the DP path of the north star.

roofline: the dominant kernel is k_group_strip (group_strip.hip) in its chained form
  (fen_group_strip_chain): the body's 6 ResidualGroups -- each 10 fused RCABs (conv1 -> PReLU ->
  conv2 -> SE gate -> scaled residual) + the group conv + skip, 64 ch, 64x64, B=32 -- as one
  persistent launch, conv_after_body its last step; algorithmic FLOPs per launch = (6 x 21 + 1)
  convs x 2 * 32*64*64 px * 64 co * 576 (= 9 taps * 64 ci) = 1227.3 GFLOP (9.66 per conv),
  timed live here with HIP events on the launch stream; peak = 2500 TFLOP/s fp16 / bf16 dense.
pcie_inclusive: the same forward with the batch handed over as NCHW fp32 pinned host buffers
(H2D of the LR batch, graph replay, D2H of the SR batch, serial on one stream), and
("pipelined") with consecutive batches' copies on a copy stream under the replays -- reported
beside `value`, never as it.
cpu_baseline: the CPU oracle (oracle/fen_oracle.py, fp32 PyTorch-CPU restatement of the
reference forward) on this node's host cores, rank 0, N=1 only: eval at B=2 and B=32 and one
L1 train step (fwd + bwd + clip + AdamW) at B=2, each the min of 3 after 1 warm-up.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "face-super-resolution_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 / fp16 MFMA (MI355X_MICROARCH.md chip table)
PEAK_HBM_GBS = 8000.0
RCAB_CONV_FLOP = 2.0 * 32 * 64 * 64 * 64 * 576


def build_model(precision):
    from src.models import FaceEnhanceNet
    torch.manual_seed(42)  # stage1_psnr_config.yaml project.seed
    m = FaceEnhanceNet(num_channels=64, num_groups=6, blocks_per_group=10, reduction_ratio=4, scale_factor=4,
                       precision=precision)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        m.conv_last.weight.copy_(torch.randn(m.conv_last.weight.shape, generator=g) * 1e-3)
    return m


DTYPES = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}


def bench_batch(B, rank):
    """The bench's synthetic batch: smooth 256x256 HR images (uint8 levels, seeded per rank)
    and their bicubic /4 (trainer.py:416-421) computed on the GPU by the framework's own
    k_bicubic_down4."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from smooth import smooth_images
    from src.hip import lib as L
    hr = smooth_images(B, 256, 256, 1234 + rank).cuda()
    lr = torch.empty(B, 3, 64, 64, device="cuda")
    L.check(L.load().fen_bicubic_down4(B, 3, 256, 256, hr.data_ptr(), lr.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream), "bicubic_down4")
    return hr, lr


def log(msg):
    """progress on stderr (the JSON line on stdout stays the only stdout output)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def psnr(pred, target):
    """trainer.py:621-628 (batch-mean MSE), in fp64."""
    mse = torch.mean((pred.double().cpu() - target.double().cpu()) ** 2)
    return float(10.0 * torch.log10(1.0 / mse))


def timed(fn, steps, warmup, world):
    for _ in range(warmup):
        fn()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], device="cuda", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt)


def dominant_op(engine):
    """The launch the roofline is quoted on: the body's G ResidualGroups (fen_group_strip_chain,
    one persistent launch; algorithmic FLOPs = G (2 NB + 1) 64->64 convs), else a whole
    ResidualGroup (fen_group_strip: NB fused RCABs -- conv1 + PReLU + conv2 + SE gate + scaled
    residual each -- and the group conv; (2 NB + 1) convs), else an RCAB of the per-RCAB chain
    (fen_rcab_deferred), else the RCAB conv1 (64->64, 64x64, B=32) of the per-op path."""
    for op in engine.ctx.ops:
        if op[0] == "group_strip_chain":
            ds, ng, tail = op[2]
            d = ds[0]
            conv = 2.0 * d.B * d.H * d.W * 64 * 576
            return op, "k_group_strip chain (the body: %d ResidualGroups in one launch, each %d x [conv1+PReLU+conv2+" \
                       "SE gate+residual] + group conv + skip%s, 64ch %dx%d, B=%d)" % (
                           ng, d.nb, "; + conv_after_body" if tail is not None else "", d.H, d.W, d.B), \
                (ng * (2 * d.nb + 1) + (1 if tail is not None else 0)) * conv
    for op in engine.ctx.ops:
        if op[0] == "group_strip":
            d = op[2][0]._obj
            conv = 2.0 * d.B * d.H * d.W * 64 * 576
            return op, "k_group_strip (a ResidualGroup in one launch: %d x [conv1+PReLU+conv2+SE gate+residual] + " \
                       "group conv + skip, 64ch %dx%d, B=%d)" % (d.nb, d.H, d.W, d.B), (2 * d.nb + 1) * conv
    for op in engine.ctx.ops:
        if op[0] == "rcab_deferred":
            d = op[2][0]._obj
            if d.tp:
                return op, "k_rcab_d (RCAB: prev. SE gate + residual applied to the input halo, conv1+PReLU+conv2+" \
                           "tile sums, 64ch 64x64, B=%d)" % d.B, 2 * 2.0 * d.B * d.H * d.W * 64 * 576
    for op in engine.ctx.ops:
        if op[0] == "conv3x3" and op[1] is not None:
            d = op[2][0]._obj
            if d.Cin == 64 and d.Cout == 64 and d.H == 64 and d.W == 64:
                return op, "k_conv3x3 (RCAB conv1 64->64 + bias + PReLU, 64x64, B=%d)" % d.B, \
                    2.0 * d.B * d.H * d.W * 64 * 576
    raise RuntimeError("no RCAB launch in the program")


def time_dominant_kernel(engine, reps=50):
    """Average duration of the dominant launch, timed with HIP events on the stream it runs on
    (torch's current stream), replayed back to back."""
    from src.hip.program import current_stream_handle
    (name, fn, args), label, flop = dominant_op(engine)
    s = current_stream_handle()
    for _ in range(5):
        fn(*args, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(*args, s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, label, flop  # ms


def captured_or_eager(eng, world):
    """A training engine's step replayed from its captured hipGraph -- at N > 1 with the bucket
    all-reduces recorded in it (stream-ordered RCCL exchange) -- or, should the capture fail at
    N > 1, the same step run eagerly (the line says which)."""
    try:
        eng.capture()
        return eng.replay, "hipGraph replay" + (" (RCCL all-reduces captured)" if world > 1 else "")
    except Exception as e:   # noqa: BLE001 -- reported, and the eager step is timed instead
        if world == 1:
            raise
        torch.cuda.synchronize()
        return eng.step, f"eager (capture failed: {type(e).__name__}: {str(e)[:120]})"


def time_pcie_inclusive(eng, x, steps, warmup, world):
    """images/s when the boundary hands over host buffers: NCHW fp32 LR batch in pinned host
    memory -> H2D into the engine's input, the captured forward, SR batch D2H into pinned
    host memory; serial on torch's current stream (no overlap of copies with compute)."""
    hx = x.cpu().pin_memory()
    hout = torch.empty(eng.out.shape, dtype=eng.out.dtype).pin_memory()

    def step():
        eng.x.copy_(hx, non_blocking=True)
        eng.replay()
        hout.copy_(eng.out, non_blocking=True)
    t = timed(step, steps, warmup, world)
    B = x.shape[0]
    return {"value": round(B * world * steps / t, 2), "unit": "images/sec", "ms_per_step": round(1000.0 * t / steps, 4),
            "bytes_h2d": hx.numel() * 4, "bytes_d2h": hout.numel() * 4,
            "note": "NCHW fp32 pinned host in/out, copies serial with the graph replay"}


def time_pcie_pipelined(eng, x, steps, warmup, world):
    """images/s when the boundary hands over host buffers and consecutive batches are pipelined:
    the H2D of batch i+1 and the D2H of batch i-1 run on a copy stream while batch i's graph
    replays (pinned host buffers and device staging buffers, two of each; the staging copies into
    / out of the engine's own buffers are D2D on the compute stream)."""
    main = torch.cuda.current_stream()
    cs = torch.cuda.Stream()
    hx = [x.cpu().pin_memory() for _ in range(2)]
    hout = [torch.empty(eng.out.shape, dtype=eng.out.dtype).pin_memory() for _ in range(2)]
    din = [torch.empty_like(eng.x) for _ in range(2)]
    dout = [torch.empty_like(eng.out) for _ in range(2)]
    ev = {k: [torch.cuda.Event() for _ in range(2)] for k in ("in", "used", "out", "d2h")}

    def run(n):
        with torch.cuda.stream(cs):
            din[0].copy_(hx[0], non_blocking=True)
            ev["in"][0].record(cs)
        for i in range(n):
            b = i & 1
            with torch.cuda.stream(cs):                   # the next batch's H2D, its staging buffer free
                cs.wait_event(ev["used"][1 - b])
                din[1 - b].copy_(hx[1 - b], non_blocking=True)
                ev["in"][1 - b].record(cs)
            main.wait_event(ev["in"][b])
            eng.x.copy_(din[b])
            ev["used"][b].record(main)
            main.wait_event(ev["d2h"][b])                 # this staging output free (batch i-2's D2H done)
            eng.replay()
            dout[b].copy_(eng.out)
            ev["out"][b].record(main)
            with torch.cuda.stream(cs):                   # this batch's D2H under the next replay
                cs.wait_event(ev["out"][b])
                hout[b].copy_(dout[b], non_blocking=True)
                ev["d2h"][b].record(cs)
        cs.synchronize()

    run(warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt)
    B = x.shape[0]
    return {"value": round(B * world * steps / dt, 2), "unit": "images/sec", "ms_per_step": round(1000.0 * dt / steps, 4),
            "note": "NCHW fp32 pinned host in/out; H2D of batch i+1 and D2H of batch i-1 on a copy stream under "
                    "batch i's replay"}


def conv_flop(cin, cout, h, w, k=3):
    return 2.0 * cin * cout * k * k * h * w


# ---- algorithmic FLOPs of the training legs (every 3x3 conv counted as
# 2 Cin Cout 9 Hout Wout; a data or weight gradient costs what its forward costs; SE, PReLU, BN,
# pools, bicubic and the elementwise work are excluded) ----
def gen_fwd_flop(hw=64, C=64, G=6, R=10, scale=4):
    """One image through FaceEnhanceNet (custom.py:147-190): conv_first, G x (2R + 1) body
    convs, conv_after_body, log2(scale) conv + PixelShuffle stages, conv_last."""
    f = conv_flop(3, C, hw, hw) + (G * (2 * R + 1) + 1) * conv_flop(C, C, hw, hw)
    s = hw
    while s < hw * scale:
        f += conv_flop(C, 4 * C, s, s)
        s *= 2
    return f + conv_flop(C, 3, s, s)


def gen_train_flop(hw=64):
    """forward + data gradients + weight gradients, less conv_first's data gradient (no gradient
    flows to the LR input): 133.9 GFLOP per image at the bench shape."""
    return 3.0 * gen_fwd_flop(hw) - conv_flop(3, 64, hw, hw)


def vgg_flops(hr_hw=256, last="conv3_4"):
    """VGG19 up to the feature layer (perceptual.py:13-169): (forward FLOPs per image, data-
    gradient FLOPs per image of the pred half, conv1_1's included -- the gradient reaches sr)."""
    from src.hip.vgg import LAYER_MAP, vgg19_convs
    fwd = bwd = 0.0
    s = hr_hw
    for c in vgg19_convs():
        if c["idx"] > LAYER_MAP[last]:
            break
        fwd += conv_flop(c["cin"], c["cout"], s, s)
        bwd += conv_flop(c["cin"], c["cout"], s, s)
        if c["pool_after"]:
            s //= 2
    return fwd, bwd


def disc_flops(hw=256, bc=64):
    """VGGStyleDiscriminator (discriminator.py:58-90) per image: (forward FLOPs, the first conv's
    forward FLOPs); the stride-2 convs at their output resolution; the classifier's two GEMMs."""
    cfg = [(3, bc, 1), (bc, bc, 2), (bc, 2 * bc, 1), (2 * bc, 2 * bc, 2), (2 * bc, 4 * bc, 1), (4 * bc, 4 * bc, 2),
           (4 * bc, 8 * bc, 1), (8 * bc, 8 * bc, 2), (8 * bc, 8 * bc, 1), (8 * bc, 8 * bc, 2)]
    f, s, first = 0.0, hw, None
    for cin, cout, st in cfg:
        s //= st
        f += conv_flop(cin, cout, s, s)
        first = first if first is not None else conv_flop(cin, cout, s, s)
    f += 2.0 * 8 * bc * s * s * 1024 + 2.0 * 1024
    return f, first


def gan_iteration_flop(B=16, hw=64, freeze_d=True, reuse_g=True):
    """One Trainer._gan_step (trainer.py:424-485, d_updates_per_g = 1): D step = G forward (no
    grad) + D forward on real and fake + D backward of both (weight gradients, data gradients
    but the first conv's); G step = G training pass + VGG19 conv3_4 perceptual (forward on
    [sr; hr], backward on sr) + D forward on sr + D's data gradients down to sr (the first
    conv's included).  D's weight gradients in the G step are counted only with
    freeze_d_in_g_step=False (the reference computes them and never uses them:
    TrainerConfig.freeze_d_in_g_step skips them by default), the D step's own generator forward
    only with reuse_g_forward=False (the reference recomputes the G step's forward there: same
    input, same weights)."""
    g_fwd = gen_fwd_flop(hw)
    d_fwd, d_first = disc_flops(4 * hw)
    v_fwd, v_bwd = vgg_flops(4 * hw)
    d_step = (0 if reuse_g else g_fwd) + 2 * d_fwd + 2 * (2 * d_fwd - d_first)
    g_step = gen_train_flop(hw) + 2 * v_fwd + v_bwd + d_fwd + (d_fwd if freeze_d else 2 * d_fwd)
    return B * (d_step + g_step)


def step_roofline(flop, ms, note):
    """roofline object of a whole training step: algorithmic FLOPs / the step's wall time."""
    tf = flop / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / PEAK_BF16_TFLOPS, 4), "flop_per_step": flop, "traffic": None,
            "basis": "whole step wall time (graph replay), " + note}


def time_stress(steps=3, warmup=1, B=4, hw=128, precision="fp16"):
    """BASELINE configs[4]: the 128-ch / 10x20 RCAB x8 stress variant, inference, 128x128 ->
    1024x1024 (x8 from a 128 input), in its stated fp16; the body,
    conv_after_body and the upsampler on fen_rcab_c128 (rcab128.hip).  Algorithmic FLOPs: every 3x3 conv
    (head, 400 RCAB convs, 10 group convs, conv_after_body, 3 upsampler stages, conv_last)."""
    from src.models import FaceEnhanceNet
    from src.hip.engine import FENEngine
    C, G, R, S = 128, 10, 20, 8
    torch.manual_seed(42)
    m = FaceEnhanceNet(num_channels=C, num_groups=G, blocks_per_group=R, reduction_ratio=4, scale_factor=S,
                       precision=precision)
    eng = FENEngine(m, batch=B, lr_hw=(hw, hw), dtype=DTYPES[precision], train=False, device="cuda")
    eng.x.copy_(torch.rand(B, 3, hw, hw, generator=torch.Generator().manual_seed(7)).cuda())
    eng.capture()
    t = timed(eng.replay, steps, warmup, 1)
    flop = conv_flop(3, C, hw, hw) + (2 * G * R + G + 1) * conv_flop(C, C, hw, hw)
    flop += sum(conv_flop(C, 4 * C, hw << i, hw << i) for i in range(3)) + conv_flop(C, 3, hw * S, hw * S)
    flop *= B
    ms = 1000.0 * t / steps
    out = {"metric": "images/sec (128ch 10x20 RCAB x8 stress, 128->1024)", "value": round(B * steps / t, 3),
           "unit": "images/sec", "batch": B, "ms_per_step": round(ms, 3), "dtype": precision,
           "gflop_per_step": round(flop / 1e9, 1), "achieved_TFLOPs": round(flop / (t / steps) / 1e12, 1),
           "frac_peak": round(flop / (t / steps) / 1e12 / PEAK_BF16_TFLOPS, 4)}
    del eng, m
    torch.cuda.empty_cache()
    return out


def _cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    # a shared GPU box exposes the whole machine's CPUs but allots this job a share, which it
    # states in OMP_NUM_THREADS (16 on the MI355X pool): use that many, not more
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    return model, usable


def cpu_baseline(model, lr32, hr32):
    """The CPU oracle (fp32 PyTorch-CPU restatement of the reference path) on this host:
    eval forward at B=2 and at B=32 (the bench's own batch) and one L1 train step at B=2
    (forward, backward, clip 0.5, AdamW), each the min of 3 timed passes after 1 warm-up, on
    every core this process may run on (os.sched_getaffinity: on a shared GPU box
    os.cpu_count() reports the whole machine).  The B=32 pass's output is the fp32 reference
    for psnr_parity."""
    from oracle import fen_oracle as O
    cpu_model, usable = _cpu_info()
    torch.set_num_threads(usable)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    shape = O.NetShape(64, 6, 10, 4, 4, 0.2)
    lr32 = lr32.float().cpu()

    def best(fn):
        fn()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t0)
        return min(ts), r

    with torch.no_grad():
        t2, _ = best(lambda: O.forward(sd, lr32[:2], shape, training=False))
        t32, ref = best(lambda: O.forward(sd, lr32, shape, training=False))
    ttr, _ = best(lambda: O.train_step(sd, hr32[:2].float().cpu(), shape, lr=1e-4, clip=0.5))
    legs = {"eval_b2": {"images_per_sec": round(2 / t2, 3), "ms": round(1e3 * t2, 2)},
            "eval_b32": {"images_per_sec": round(32 / t32, 3), "ms": round(1e3 * t32, 2)},
            "train_b2": {"images_per_sec": round(2 / ttr, 3), "ms": round(1e3 * ttr, 2)}}
    out = {"value": legs["eval_b32"]["images_per_sec"], "unit": "images/sec", "cores": usable, "kind": "port",
           "cpu_model": cpu_model, "os_cpu_count": os.cpu_count(), "torch_threads": torch.get_num_threads(),
           "sample": "oracle fp32 eval forward of the bench's own B=32 batch (full 6x10 net, 64x64 -> 256x256); "
                     "min of 3 after 1 warm-up",
           "legs": legs}
    return out, ref


def time_gan_step(steps, B=16):
    """Stage 3 (stage3_gan_config.yaml:40-60, BASELINE C4, B=16/GPU): one Trainer iteration =
    discriminator update (G forward, D on real + fake, D backward, AdamW) + generator update
    (G forward, content L1 x 0.01 + perceptual x 1 + adversarial x 0.005 through D, backward,
    clip, AdamW) on the module autograd path; timed as the Trainer runs it (replayed from a
    captured hipGraph) and eagerly ("eager")."""
    import warnings
    from src.losses import create_loss_function
    from src.models import GANLoss, VGGStyleDiscriminator
    from src.training import Trainer, TrainerConfig
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        loss_fn = create_loss_function(l1_weight=0.01, perceptual_weight=1.0, ssim_weight=0.0,
                                       perceptual_layers=["conv3_4"])
    torch.manual_seed(7)
    D = VGGStyleDiscriminator(input_size=256, precision="bf16")
    cfg = TrainerConfig(learning_rate=1e-4, weight_decay=0.0, gradient_clip=0.5, gan_weight=0.005,
                        d_learning_rate=1e-4, use_wandb=False, scheduler_type="none",
                        checkpoint_dir="/tmp/fen_bench_ckpt",
                        freeze_d_in_g_step=os.environ.get("FEN_GAN_FREEZE_D", "1") == "1",   # (A/B switches)
                        reuse_g_forward=os.environ.get("FEN_GAN_REUSE_G", "1") == "1")
    tr = Trainer(build_model("bf16"), [], None, loss_fn=loss_fn, config=cfg, discriminator=D,
                 gan_loss=GANLoss("vanilla"))
    hr = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(99)).cuda()

    def run(fn):
        for _ in range(3):               # the captured path: 2 eager warm-ups + the capture
            fn(hr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = fn(hr)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, float(loss)

    el_e, _ = run(tr._gan_step)
    el, loss = run(tr._gan_iteration)
    frz = bool(getattr(tr.config, "freeze_d_in_g_step", True))
    reu = bool(getattr(tr.config, "reuse_g_forward", True))
    flop = gan_iteration_flop(B, freeze_d=frz, reuse_g=reu)
    return {"roofline": step_roofline(flop, 1000.0 * el / steps,
                                      "algorithmic FLOPs of one iteration (bench.gan_iteration_flop: "
                                      + ("" if reu else "G fwd + ") + "D fwd x2 + "
                                      "D bwd x2; G train + VGG19 conv3_4 fwd x2 + dgrad + D fwd + D "
                                      + ("data gradients (freeze_d_in_g_step: D's unused weight gradients not computed)"
                                         if frz else "bwd") + ") at B=16"),
            "metric": "training images/sec (stage-3 GAN iteration: D update + G update, L1 0.01 + perceptual 1 + "
                      "adversarial 0.005) at batch 16/GPU", "value": round(B * steps / el, 2),
            "ms_per_step": round(1000.0 * el / steps, 3), "steps": steps, "loss": loss,
            "path": ("Trainer iteration replayed from a captured hipGraph (capture_gan_step; module autograd "
                     "over the HIP kernels), VGG19 and D random-init" if tr._capture_gan() else
                     "Trainer iteration, eager (N > 1: the module path's hook-issued RCCL all-reduces are not "
                     "captured unless FEN_GAN_CAPTURE_DP=1), VGG19 and D random-init"),
            "eager": {"value": round(B * steps / el_e, 2), "ms_per_step": round(1000.0 * el_e / steps, 3)}}


def time_ssim(eng, reps=50):
    """The stage-2 SSIM op of a training engine (fwd map + tile sums + gradient added to dL/dsr;
    fen_ssim_ex's two launches), timed with HIP events on the current stream, against the HBM
    roofline: algorithmic bytes = pred + target (fp32 NCHW) read + dL/dsr (NHWC16 bf16) read +
    write (the a / b / c workspace is the implementation's, not counted)."""
    name, fn, fargs = next(op for op in eng.ctx.ops if op[0] == "ssim")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        fn(*fargs, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(*fargs, s)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    B, C, H, W = eng.B, 3, eng.H, eng.W
    nbytes = 2 * B * C * H * W * 4 + 2 * B * H * W * 16 * 2
    return {"kernel": "k_ssim + k_ssim_g2 (csrc/ssim.hip, fen_ssim_ex: map + a/b/c, then the gradient)",
            "us": round(us, 2), "bytes": nbytes,
            "achieved_GBs": round(nbytes / us / 1e3, 1), "peak_GBs": 8000.0,
            "frac": round(nbytes / us / 1e3 / 8000.0, 4), "bound": "hbm"}


def exchange_label(backend, world):
    """what carries a training leg's gradient all-reduce (src/training/dp.py)"""
    if world <= 1:
        return "none"
    from src.training.dp import use_direct_rccl
    if backend != "nccl":
        return f"torch.distributed {backend}, per-group buckets, overlapped with backward"
    path = ("RCCL called directly (fen_rccl_allreduce_bucket, include/fen.h)" if use_direct_rccl()
            else "RCCL through torch.distributed (ProcessGroupNCCL)")
    return path + ", per-group buckets on a side stream, overlapped with backward"


def load_traffic(label):
    """HBM bytes per launch of the dominant kernel from its committed PMC summary
    (profiles/rNN_pmc_*.json, tools/prof_summary.py pmc; the latest round's first), or None
    when none matches it."""
    import glob
    best = None                                   # the longest matching key; latest round first
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_*.json")), reverse=True):
        with open(p) as f:
            js = json.load(f)
        key = js.get("kernel_key")
        if key and label.startswith(key) and (best is None or len(key) > len(best[0])):
            best = (key, js.get("hbm_bytes_per_launch"))
    return best[1] if best else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--no-perceptual", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stress", action="store_true")
    ap.add_argument("--precision", choices=["fp16", "bf16"], default="fp16",
                    help="16-bit format of the headline inference run (the other one is reported beside it)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FEN_BENCH_BACKEND=gloo + ranks sharing one device: a rehearsal of the N>1 path on a
    # one-GPU box (the driver's multi-GPU runs use the default, RCCL, one GPU per rank)
    backend = os.environ.get("FEN_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            from src.training.dp import init_rccl
            init_rccl(torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from src.hip.engine import FENEngine

    B = args.batch
    prec = args.precision
    other = "bf16" if prec == "fp16" else "fp16"
    hr, x = bench_batch(B, rank)

    def run_inference(p):
        m = build_model(p)
        e = FENEngine(m, batch=B, lr_hw=(64, 64), dtype=DTYPES[p], train=False, device="cuda")
        e.x.copy_(x)
        e.capture()
        tt = timed(e.replay, args.steps, args.warmup, world)
        km, kl, kf = time_dominant_kernel(e)
        e.replay()
        torch.cuda.synchronize()
        return e, tt, km, kl, kf, e.out.detach().cpu().clone()

    cpu_model_sd = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_model_sd = build_model("fp32")
    log(f"inference {prec}")
    eng, t, kern_ms, kern_label, kern_flop, out_main = run_inference(prec)
    value = B * world * args.steps / t
    ms = 1000.0 * t / args.steps
    achieved = kern_flop / (kern_ms * 1e-3) / 1e12
    out = {
        "metric": "images/sec (64->256 4x SR) at batch 32/GPU",
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": prec,
        "data": "synthetic: bicubic /4 of smooth 256x256 uint8-level HR images (tests/golden/smooth.py, seeded per "
                "rank), resident in HBM; seeded random-init weights of the reference architecture",
        "config": {"workload": f"FaceEnhanceNet full (6x10 RCAB, 64ch) inference 64->256, {prec} "
                               "(BASELINE configs[1]; its bf16 run is the 'bf16' leg)",
                   "global_batch": B * world, "per_gpu_batch": B,
                   "parallelism": f"replicas x{world}" if world > 1 else "single"},
        "roofline": {"bound": "mfma", "kernel": kern_label,
                     "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "kernel_ms": round(kern_ms, 5),
                     "flop_per_launch": kern_flop, "traffic": load_traffic(kern_label),
                     "per_rcab_us_equiv": round(kern_ms * 1e3 * RCAB_CONV_FLOP * 2 / kern_flop, 3)},
    }
    out["pcie_inclusive"] = time_pcie_inclusive(eng, x, args.steps, args.warmup, world)
    out["pcie_inclusive"]["pipelined"] = time_pcie_pipelined(eng, x, args.steps, args.warmup, world)
    del eng
    torch.cuda.empty_cache()
    # the same workload in the other 16-bit format (BASELINE configs[1] names bf16)
    log(f"inference {other}")
    eng2, t2, k2_ms, _, k2_flop, out_other = run_inference(other)
    out[other] = {"value": round(B * world * args.steps / t2, 2), "unit": "images/sec",
                  "ms_per_step": round(1000.0 * t2 / args.steps, 4),
                  "roofline_frac": round(k2_flop / (k2_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                  "kernel_ms": round(k2_ms, 5)}
    del eng2
    torch.cuda.empty_cache()
    if not args.no_train:
        tm = build_model("bf16")
        log("stage-1 L1 training")
        teng = FENEngine(tm, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda")
        hr_t = hr   # the smooth synthetic HR batch (LR synthesis runs inside the step)
        teng.hr.copy_(hr_t)
        fn, tpath = captured_or_eager(teng, world)
        tt = timed(fn, args.train_steps, 3, world)
        out["train"] = {"metric": "training images/sec (stage-1 L1 generator step) at batch 32/GPU",
                        "value": round(B * world * args.train_steps / tt, 2),
                        "ms_per_step": round(1000.0 * tt / args.train_steps, 3), "steps": args.train_steps,
                        "loss": float(teng.loss), "path": tpath, "allreduce": exchange_label(backend, world),
                        "roofline": step_roofline(B * gen_train_flop(), 1000.0 * tt / args.train_steps,
                                                  "generator fwd + dgrad + wgrad (133.9 GFLOP/img) x B")}
        del teng
        torch.cuda.empty_cache()
        if not args.no_perceptual:
            # the stage-1 recipe proper (stage1_psnr_config.yaml:40-50): L1 x 1 + VGG19 conv3_4
            # perceptual x 1; VGG19 randomly initialised (no ImageNet weights offline)
            import warnings
            from src.losses import PerceptualLoss
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                spec = PerceptualLoss(layers=["conv3_4"]).to("cuda").fused_spec(1.0)
            pm = build_model("bf16")
            log("stage-1 training with the perceptual term")
            peng = FENEngine(pm, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda",
                             perceptual=spec)
            peng.hr.copy_(hr_t)
            fn, ppath = captured_or_eager(peng, world)
            vf, vb = vgg_flops()
            tp = timed(fn, args.train_steps, 3, world)
            out["train_perceptual"] = {
                "metric": "training images/sec (stage-1 step: L1 + VGG19 conv3_4 perceptual) at batch 32/GPU",
                "value": round(B * world * args.train_steps / tp, 2),
                "ms_per_step": round(1000.0 * tp / args.train_steps, 3), "steps": args.train_steps,
                "loss": float(peng.total_loss()), "vgg": "random-init VGG19 (no ImageNet weights offline)",
                "path": ppath, "allreduce": exchange_label(backend, world),
                "roofline": step_roofline(B * (gen_train_flop() + 2 * vf + vb), 1000.0 * tp / args.train_steps,
                                          "generator train (133.9 GFLOP/img) + VGG19 conv3_4 fwd on [sr; hr] + dgrad "
                                          "on sr (%.1f GFLOP/img) x B" % ((2 * vf + vb) / 1e9))}
            del peng
            torch.cuda.empty_cache()
            # stage 2 (stage2_ssim_config.yaml:40-50): L1 x 1 + perceptual x 0.5 + (1 - SSIM) x 0.2
            spec2 = dict(spec, weight=0.5)
            sm = build_model("bf16")
            log("stage-2 training")
            seng = FENEngine(sm, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda",
                             perceptual=spec2, ssim_weight=0.2)
            seng.hr.copy_(hr_t)
            fn, spath = captured_or_eager(seng, world)
            ts = timed(fn, args.train_steps, 3, world)
            out["train_stage2"] = {
                "metric": "training images/sec (stage-2 step: L1 + 0.5 perceptual + 0.2 (1 - SSIM)) at batch 32/GPU",
                "value": round(B * world * args.train_steps / ts, 2),
                "ms_per_step": round(1000.0 * ts / args.train_steps, 3), "steps": args.train_steps,
                "loss": float(seng.total_loss()), "path": spath, "allreduce": exchange_label(backend, world),
                "roofline": step_roofline(B * (gen_train_flop() + 2 * vf + vb), 1000.0 * ts / args.train_steps,
                                          "as train_perceptual (SSIM is HBM-bound: aux.ssim_loss_grad)")}
            if world == 1:
                out["aux"] = {"ssim_loss_grad": time_ssim(seng)}
            del seng
            torch.cuda.empty_cache()
            if world == 1:
                log("stage-3 GAN iteration")
                out["train_gan"] = time_gan_step(args.train_steps)
    if world == 1 and not args.no_stress:
        log("stress config (128 ch, x8)")
        out["stress_c128_x8"] = time_stress()
    if cpu_model_sd is not None:
        log("CPU baseline + PSNR parity")
        out["cpu_baseline"], ref = cpu_baseline(cpu_model_sd, x, hr)
        p_ref = psnr(ref, hr)
        pp = {}
        for name, o in ((prec, out_main), (other, out_other)):
            pg = psnr(o, hr)
            pp[name] = {"psnr_gpu": round(pg, 5), "psnr_ref": round(p_ref, 5), "delta_db": round(pg - p_ref, 5),
                        "max_abs_diff": float((o - ref).abs().max())}
        out["psnr_parity"] = dict(pp[prec], images=B, target="HR (smooth synthetic, uint8 levels)",
                                  ref="CPU oracle fp32 (pinned to the reference, tests/test_oracle.py)",
                                  tolerance_db=0.01, **{other: pp[other]})
    # every strip launch of the timed regions reported through the status word: a timed-out
    # hand-off wait (invalid outputs) fails the run here instead of passing as a number
    from src.hip import lib as L
    torch.cuda.synchronize()
    L.check_strip_status()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        from src.training.dp import RcclComm
        RcclComm.destroy_all()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
