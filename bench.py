#!/usr/bin/env python
"""FaceEnhanceNet 64->256 (x4) super-resolution throughput on MI355X.

Metric (BASELINE.json): images/sec at batch 32 per GPU on 1/2/4/8 GPUs.  The workload of
`value` is BASELINE configs[1]: the full network (6 groups x 10 RCAB, 64 ch) in bf16,
inference, batch 32 per GPU, synthetic 64x64x3 inputs resident in HBM, random-init
weights of the reference architecture (seeded reference init + conv_last ~ N(0,1e-3)).
One "step" = one forward of one 32-image batch, replayed from a hipGraph.  With N>1 each
rank runs its own replica on its own shard (inference has no exchange step: weak scaling).

Also reported (field "train"): the stage-1 generator training step (bicubic /4 LR
synthesis, forward, L1, backward, RCCL gradient all-reduce over xGMI for N>1, clip,
AdamW) at batch 32 per GPU -- the DP path of the north star.

roofline: the dominant kernel is the fused RCAB k_rcab (conv1 -> PReLU -> conv2 -> SE gate ->
  residual, 64 ch, 64x64, B=32): algorithmic FLOPs per launch = 2 convs x 2 * 32*64*64 px * 64 co
  * 576 (= 9 taps * 64 ci) = 19.33 GFLOP, timed live here with HIP events on the launch stream;
  peak = 2500 TFLOP/s bf16 dense.
pcie_inclusive: the same forward with the batch handed over as NCHW fp32 pinned host buffers
(H2D of the LR batch, graph replay, D2H of the SR batch, serial on one stream) -- reported
beside `value`, never as it.
cpu_baseline: the CPU oracle (oracle/fen_oracle.py, fp32 PyTorch-CPU restatement of the
reference forward) on this node's host cores, rank 0, N=1 only, bounded sample.
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

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
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
    """The launch the roofline is quoted on: the fused RCAB block (fen_rcab_fused) when the
    engine uses it, else the RCAB conv1 (64->64, 64x64, B=32) of the per-op path."""
    for op in engine.ctx.ops:
        if op[0] == "rcab_fused":
            d = op[2][0]._obj
            return op, "k_rcab (fused RCAB: conv1+PReLU+conv2+SE gate+residual, 64ch 64x64, B=%d)" % d.B, \
                2 * 2.0 * d.B * d.H * d.W * 64 * 576
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


def conv_flop(cin, cout, h, w, k=3):
    return 2.0 * cin * cout * k * k * h * w


def time_stress(steps=3, warmup=1, B=4, hw=128):
    """BASELINE configs[4]: the 128-ch / 10x20 RCAB x8 stress variant, inference, 128x128 ->
    1024x1024 (x8 from a 128 input), bf16 on the per-op kernels
    (the fused RCAB covers 64 ch only); the reference runs it in fp16, which this build does
    not implement.  Algorithmic FLOPs: every 3x3 conv (head, 400 RCAB convs, 10 group convs,
    conv_after_body, 3 upsampler stages, conv_last)."""
    from src.models import FaceEnhanceNet
    from src.hip.engine import FENEngine
    C, G, R, S = 128, 10, 20, 8
    torch.manual_seed(42)
    m = FaceEnhanceNet(num_channels=C, num_groups=G, blocks_per_group=R, reduction_ratio=4, scale_factor=S,
                       precision="bf16")
    eng = FENEngine(m, batch=B, lr_hw=(hw, hw), dtype=torch.bfloat16, train=False, device="cuda")
    eng.x.copy_(torch.rand(B, 3, hw, hw, generator=torch.Generator().manual_seed(7)).cuda())
    eng.capture()
    t = timed(eng.replay, steps, warmup, 1)
    flop = conv_flop(3, C, hw, hw) + (2 * G * R + G + 1) * conv_flop(C, C, hw, hw)
    flop += sum(conv_flop(C, 4 * C, hw << i, hw << i) for i in range(3)) + conv_flop(C, 3, hw * S, hw * S)
    flop *= B
    ms = 1000.0 * t / steps
    out = {"metric": "images/sec (128ch 10x20 RCAB x8 stress, 128->1024)", "value": round(B * steps / t, 3),
           "unit": "images/sec", "batch": B, "ms_per_step": round(ms, 3), "dtype": "bf16 (reference: fp16)",
           "gflop_per_step": round(flop / 1e9, 1), "achieved_TFLOPs": round(flop / (t / steps) / 1e12, 1),
           "frac_bf16_peak": round(flop / (t / steps) / 1e12 / PEAK_BF16_TFLOPS, 4)}
    del eng, m
    torch.cuda.empty_cache()
    return out


def cpu_baseline(model, seconds=10.0):
    from oracle import fen_oracle as O
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    shape = O.NetShape(64, 6, 10, 4, 4, 0.2)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1234))
    threads = torch.get_num_threads()
    with torch.no_grad():
        O.forward(sd, x, shape, training=False)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            O.forward(sd, x, shape, training=False)
            n += 1
            el = time.perf_counter() - t0
            if (el >= seconds and n >= 3) or n >= 200:
                break
    return {"value": round(2 * n / el, 3), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"oracle fp32 eval forward, full 6x10 net, batch 2 of 64x64, {n} passes in {el:.1f}s"}


def time_gan_step(steps, B=16):
    """Stage 3 (stage3_gan_config.yaml:40-60, BASELINE C4, B=16/GPU): one Trainer iteration =
    discriminator update (G forward, D on real + fake, D backward, AdamW) + generator update
    (G forward, content L1 x 0.01 + perceptual x 1 + adversarial x 0.005 through D, backward,
    clip, AdamW) on the module autograd path (not graph-captured)."""
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
                        checkpoint_dir="/tmp/fen_bench_ckpt")
    tr = Trainer(build_model("bf16"), [], None, loss_fn=loss_fn, config=cfg, discriminator=D,
                 gan_loss=GANLoss("vanilla"))
    hr = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(99)).cuda()
    for _ in range(2):
        tr._gan_step(hr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = tr._gan_step(hr)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"metric": "training images/sec (stage-3 GAN iteration: D update + G update, L1 0.01 + perceptual 1 + "
                      "adversarial 0.005) at batch 16/GPU", "value": round(B * steps / el, 2),
            "ms_per_step": round(1000.0 * el / steps, 3), "steps": steps, "loss": float(loss),
            "path": "module autograd (eager launches), VGG19 and D random-init"}


def time_ssim(eng, reps=50):
    """The stage-2 SSIM launch of a training engine (fwd map + tile sums + gradient added to
    dL/dsr), timed with HIP events on the current stream, against the HBM roofline:
    algorithmic bytes = pred + target (fp32 NCHW) read + dL/dsr (NHWC16 bf16) read + write."""
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
    return {"kernel": "k_ssim<GRAD> (csrc/ssim.hip)", "us": round(us, 2), "bytes": nbytes,
            "achieved_GBs": round(nbytes / us / 1e3, 1), "peak_GBs": 8000.0,
            "frac": round(nbytes / us / 1e3 / 8000.0, 4), "bound": "hbm"}


def load_traffic(label):
    """HBM bytes per launch of the dominant kernel from its committed PMC summary
    (profiles/pmc_*.json, tools/prof_summary.py pmc), or None when none matches it."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        with open(p) as f:
            js = json.load(f)
        key = js.get("kernel_key")
        if key and label.startswith(key):
            return js.get("hbm_bytes_per_launch")
    return None


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
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
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
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from src.hip.engine import FENEngine

    B = args.batch
    model = build_model("bf16")
    cpu_model_sd = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_model_sd = build_model("fp32")
    eng = FENEngine(model, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=False, device="cuda")
    x = torch.rand(B, 3, 64, 64, generator=torch.Generator().manual_seed(1234 + rank)).cuda()
    eng.x.copy_(x)
    eng.capture()
    t = timed(eng.replay, args.steps, args.warmup, world)
    value = B * world * args.steps / t
    ms = 1000.0 * t / args.steps
    kern_ms, kern_label, kern_flop = time_dominant_kernel(eng)
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
        "dtype": "bf16",
        "data": "synthetic U[0,1) 64x64x3 batches resident in HBM; seeded random-init weights of the reference "
                "architecture",
        "config": {"workload": "FaceEnhanceNet full (6x10 RCAB, 64ch) inference 64->256, bf16", "global_batch": B * world,
                   "per_gpu_batch": B, "parallelism": f"replicas x{world}" if world > 1 else "single"},
        "roofline": {"bound": "mfma", "kernel": kern_label,
                     "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "kernel_ms": round(kern_ms, 5),
                     "flop_per_launch": kern_flop, "traffic": load_traffic(kern_label)},
    }
    out["pcie_inclusive"] = time_pcie_inclusive(eng, x, args.steps, args.warmup, world)
    del eng
    torch.cuda.empty_cache()
    if not args.no_train:
        tm = build_model("bf16")
        teng = FENEngine(tm, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda")
        hr = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(4321 + rank)).cuda()
        teng.hr.copy_(hr)
        if world == 1:
            teng.capture()
            fn = teng.replay
        else:
            fn = teng.step
        tt = timed(fn, args.train_steps, 3, world)
        out["train"] = {"metric": "training images/sec (stage-1 L1 generator step) at batch 32/GPU",
                        "value": round(B * world * args.train_steps / tt, 2),
                        "ms_per_step": round(1000.0 * tt / args.train_steps, 3), "steps": args.train_steps,
                        "loss": float(teng.loss), "allreduce": (("RCCL (torch.distributed nccl backend)" if backend == "nccl" else backend)
                                      + ", 8 buckets, overlapped with backward") if world > 1 else "none"}
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
            peng = FENEngine(pm, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda",
                             perceptual=spec)
            peng.hr.copy_(hr)
            if world == 1:
                peng.capture()
                fn = peng.replay
            else:
                fn = peng.step
            tp = timed(fn, args.train_steps, 3, world)
            out["train_perceptual"] = {
                "metric": "training images/sec (stage-1 step: L1 + VGG19 conv3_4 perceptual) at batch 32/GPU",
                "value": round(B * world * args.train_steps / tp, 2),
                "ms_per_step": round(1000.0 * tp / args.train_steps, 3), "steps": args.train_steps,
                "loss": float(peng.total_loss()), "vgg": "random-init VGG19 (no ImageNet weights offline)"}
            del peng
            torch.cuda.empty_cache()
            # stage 2 (stage2_ssim_config.yaml:40-50): L1 x 1 + perceptual x 0.5 + (1 - SSIM) x 0.2
            spec2 = dict(spec, weight=0.5)
            sm = build_model("bf16")
            seng = FENEngine(sm, batch=B, lr_hw=(64, 64), dtype=torch.bfloat16, train=True, device="cuda",
                             perceptual=spec2, ssim_weight=0.2)
            seng.hr.copy_(hr)
            if world == 1:
                seng.capture()
                fn = seng.replay
            else:
                fn = seng.step
            ts = timed(fn, args.train_steps, 3, world)
            out["train_stage2"] = {
                "metric": "training images/sec (stage-2 step: L1 + 0.5 perceptual + 0.2 (1 - SSIM)) at batch 32/GPU",
                "value": round(B * world * args.train_steps / ts, 2),
                "ms_per_step": round(1000.0 * ts / args.train_steps, 3), "steps": args.train_steps,
                "loss": float(seng.total_loss())}
            if world == 1:
                out["aux"] = {"ssim_loss_grad": time_ssim(seng)}
            del seng
            torch.cuda.empty_cache()
            if world == 1:
                out["train_gan"] = time_gan_step(args.train_steps)
    if world == 1 and not args.no_stress:
        out["stress_c128_x8"] = time_stress()
    if cpu_model_sd is not None:
        out["cpu_baseline"] = cpu_baseline(cpu_model_sd, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
