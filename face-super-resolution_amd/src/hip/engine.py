"""Static-buffer execution engine for FaceEnhanceNet on one MI355X.

The engine records the whole forward (and, for training, the backward, the gradient
all-reduce hooks and the clip+AdamW update) once into C-ABI programs over persistent
buffers, so one call = one replay of ~400-1100 launches with no allocation -- and the
replay is capturable into a single hipGraph (`capture()`).

Data parallelism: one process per GPU; the loss gradient is pre-scaled by
1/world so a SUM all-reduce yields the global-batch mean.  Gradients live in one flat fp32
arena laid out in parameter order, so each ResidualGroup's gradients are one contiguous
bucket; the backward program issues `dist.all_reduce(bucket, async_op=True)` as soon as a
bucket's last weight-gradient kernel is enqueued -- RCCL then runs on its own HIP stream
beside the remaining backward kernels -- and the update waits for all buckets.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import lib as L
from .net import Backward, Forward, NetSpec, Weights, colsum, tiles
from .program import Ctx, ptr


def flatten_params(model: torch.nn.Module, device) -> Dict[str, torch.Tensor]:
    """Re-home every parameter of `model` into one flat fp32 arena (module order) and
    return {name: view}.  Parameters keep their identity (state_dict / hooks unaffected)."""
    named = list(model.named_parameters())
    total = sum(p.numel() for _, p in named)
    flat = torch.empty(total, dtype=torch.float32, device=device)
    views, off = {}, 0
    for name, p in named:
        n = p.numel()
        v = flat[off:off + n].view_as(p)
        v.copy_(p.data.to(device=device, dtype=torch.float32))
        p.data = v
        views[name] = v
        off += n
    model._fen_flat = flat
    return views


class FENEngine:
    def __init__(self, model, batch: int, lr_hw, dtype: torch.dtype = torch.bfloat16, train: bool = False,
                 device="cuda", loss_weight: float = 1.0, clip: float = 0.5, lr: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, process_group=None,
                 perceptual: Optional[dict] = None, ssim_weight: float = 0.0, exchange=None,
                 adam_state=None, accumulation_steps: int = 1):
        """perceptual (training only): the stage configs' VGG19 term (perceptual.py:144-169) as
        dict(weight=, layers=, criterion=, normalize=, params={'features.i.weight': ...},
        layer_weights=None); its gradient joins the fused L1 gradient in dL/dsr.  ssim_weight
        (training only): the stage-2 term weight * (1 - SSIM) (ssim_loss.py:174-226), likewise.
        exchange (training only): a factory `(flat_grads, bucket_plan) -> obj` with `world`,
        `launch(tag)` and `wait()` replacing the RCCL BucketExchange (the tests' stand-in rank
        pair); the loss gradients are pre-scaled by its `world`.  adam_state (training only): an
        (exp_avg, exp_avg_sq, scal) triple over the parameter arena to update (the Trainer's one
        generator optimizer state, shared by every engine and its module-path optimizer), else
        a fresh one.  accumulation_steps (training only): the loss gradients are divided by it
        (reference trainer.py:477); `step(update=False)` then runs forward + backward without
        the update, as the reference's non-stepping batches do."""
        if train and dtype == torch.float16:
            raise NotImplementedError("fp16 is an inference precision on the HIP backend (train in bf16 or fp32)")
        self.spec = NetSpec.from_config(model.config)
        self.dtype, self.device, self.train = dtype, torch.device(device), train
        self.B, (self.h, self.w) = batch, lr_hw
        s = self.spec
        self.H, self.W = self.h * s.scale, self.w * s.scale
        self.clip, self.betas, self.eps, self.wd = clip, betas, eps, weight_decay
        self.pg = process_group
        self.world = 1
        if process_group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(process_group)
        if train and exchange is not None:
            from ..training.dp import model_bucket_plan
            self._exchange_factory = lambda flat: exchange(flat, model_bucket_plan(model))
        else:
            from ..training.dp import BucketExchange, model_bucket_plan
            self._exchange_factory = lambda flat: BucketExchange(flat, model_bucket_plan(model), process_group)

        model.to(self.device)
        if getattr(model, "_fen_flat", None) is None:
            self.params = flatten_params(model, self.device)
        else:
            self.params = {n: p.data for n, p in model.named_parameters()}
        self.flat_p = model._fen_flat
        self.Wt = Weights(self.params, dtype, self.device)

        B, h, w = batch, self.h, self.w
        self.x = torch.zeros(B, s.in_ch, h, w, device=self.device)
        self.out = torch.zeros(B, s.out_ch, self.H, self.W, device=self.device)
        self.ctx = Ctx(dtype, self.device, record=True)
        ctx = self.ctx
        if not train:
            self._build_forward(training=False)
        else:
            self.l1_weight = loss_weight
            self.ssim_weight = float(ssim_weight)
            self.ssim_val = torch.zeros(1, device=self.device)
            self.vgg = None
            self.loss_perc = torch.zeros(1, device=self.device)
            if perceptual:
                # pred and target share one [2B,3,H,W] buffer: the frozen VGG runs once over both
                self.x2 = torch.zeros(2 * B, s.out_ch, self.H, self.W, device=self.device)
                self.out, self.hr = self.x2[:B], self.x2[B:]
                from .vgg import VGGPerceptual
                pw = float(perceptual.get("weight", 1.0))
                layers = list(perceptual.get("layers", ["conv3_4"]))
                lw = perceptual.get("layer_weights") or {}
                self.vgg = VGGPerceptual(ctx, perceptual["params"], layers=layers,
                                         weights={n: pw * float(lw.get(n, 1.0)) for n in layers},
                                         criterion=perceptual.get("criterion", "l1"),
                                         normalize=perceptual.get("normalize", True))
            else:
                self.hr = torch.zeros(B, s.out_ch, self.H, self.W, device=self.device)
            n = self.flat_p.numel()
            self.flat_g = torch.zeros(n, device=self.device)
            if adam_state is None:
                from ..training.optim import adamw_state
                adam_state = adamw_state(self.flat_p)
            self.flat_m, self.flat_v, self.scal = adam_state
            self._model_params = [p for _, p in model.named_parameters()]
            self.grads, off = {}, 0
            for name, p in model.named_parameters():
                self.grads[name] = self.flat_g[off:off + p.numel()].view_as(p)
                p.grad = self.grads[name]
                off += p.numel()
            self.exchange = self._exchange_factory(self.flat_g)
            self.world = self.exchange.world
            self.accum = max(1, int(accumulation_steps))
            gdiv = self.world * self.accum        # the loss gradients' pre-scale (DP mean, accumulation)
            self.scal[3] = lr
            self.loss = torch.zeros(1, device=self.device)
            ctx.emit("bicubic_down4", ctx.lib.fen_bicubic_down4, B, s.out_ch, self.H, self.W, ptr(self.hr),
                     ptr(self.x))
            self.l1_scale = loss_weight / (B * s.out_ch * self.H * self.W * gdiv)
            self._build_forward(training=True)
            self._build_backward()
            self._build_update()

    # ------------------------------------------------------------------ build
    def _build_forward(self, training: bool):
        s, ctx = self.spec, self.ctx
        fw = Forward(s, ctx, self.Wt, save=self.train)
        feat0 = fw.head(self.x)
        fb = fw.fb_for_chain(feat0)      # conv_after_body's output, if the chained launch computes it
        if self.train:   # every group output kept: the next group's saved input
            h, self.saved = fw.body(feat0, [ctx.alloc(feat0.shape) for _ in range(s.G)], fb=fb)
        else:
            h, self.saved = fw.body(feat0, [ctx.scratch(f"grp_pp{g & 1}", feat0.shape) for g in range(s.G)], fb=fb)
        hr = self.hr if self.train else None
        _, self.saved_tail = fw.tail(h, feat0, self.x, training, out=self.out, hr=hr,
                                     l1_scale=self.l1_scale if self.train else 0.0, fb=fb if fw.fb_done else None)
        if self.train:
            lp = self.saved_tail["loss_part"]
            colsum(ctx, lp, lp.shape[0], 1, self.loss, scale=1.0 / (self.B * s.out_ch * self.H * self.W))
            if self.vgg is not None:
                self.vgg.build(self.x2, self.loss_perc, self.saved_tail["dout"], grad_scale=1.0 / (self.world * self.accum))
            if self.ssim_weight:
                self._build_ssim()

    def _build_ssim(self):
        """weight * (1 - mean SSIM(sr, hr)): the SSIM map's tile sums and its gradient, added
        to dL/dsr (NHWC16) in the same launch; then per-image and batch means."""
        ctx, s = self.ctx, self.spec
        B, C, H, W = self.B, s.out_ch, self.H, self.W
        from ..losses.ssim import _window1d
        self.ssim_win = _window1d(11, 1.5).to(self.device)
        rows = ctx.lib.fen_ssim_parts(B, C, H, W)
        part = ctx.scratch("ssim_part", (rows * B,), torch.float32)
        per = ctx.scratch("ssim_img", (B,), torch.float32)
        n = B * C * H * W
        # two launches (the map + its gradient coefficients a, b, c to a workspace, then their
        # filtering into dL/dsr): fen_ssim_ex, equal results to the one-launch fen_ssim
        work = ctx.scratch("ssim_work", (int(ctx.lib.fen_ssim_work_floats(B, C, H, W)),), torch.float32)
        ctx.emit("ssim", ctx.lib.fen_ssim_ex, ctx.code, B, C, H, W, ptr(self.out), ptr(self.hr), ptr(self.ssim_win), 11,
                 0.01 ** 2, 0.03 ** 2, ptr(part), ptr(self.saved_tail["dout"]), -self.ssim_weight / (n * self.world * self.accum), 2,
                 ptr(work))
        ctx.emit("ssim_img", ctx.lib.fen_colsum, rows, B, ptr(part), 1.0 / (C * H * W), ptr(per), 0)
        ctx.emit("ssim_mean", ctx.lib.fen_colsum, B, 1, ptr(per), 1.0 / B, ptr(self.ssim_val), 0)

    def _build_backward(self):
        s, ctx = self.spec, self.ctx
        bw = Backward(s, ctx, self.Wt, self.grads)
        ex = self.exchange
        d = bw.tail(self.saved_tail)
        ctx.mark("allreduce_tail", lambda: ex.launch("tail"))
        for g in reversed(range(s.G)):
            extra = (self.saved_tail["d_fb"],) if g == 0 else ()
            d = bw.group(self.saved[g], d, g, extra_res=extra, dx_out=ctx.scratch(f"bw_grp{g & 1}", d.shape))
            ctx.mark(f"allreduce_rg{g}", lambda t=f"rg{g}": ex.launch(t))
        bw.head(self.x, d)
        ctx.mark("allreduce_head", lambda: ex.launch("head"))

    def _build_update(self):
        self.upd = Ctx(self.dtype, self.device, record=True)
        u, lib = self.upd, self.upd.lib
        n = self.flat_g.numel()
        nparts = lib.fen_sumsq_parts(n)
        self.sq_part = torch.zeros(nparts, device=self.device)
        b1, b2 = self.betas
        u.emit("sumsq", lib.fen_sumsq, n, ptr(self.flat_g), ptr(self.sq_part))
        u.emit("optim_prepare", lib.fen_optim_prepare, nparts, ptr(self.sq_part), float(self.clip), b1, b2,
               float(self.wd), ptr(self.scal))
        u.emit("adamw", lib.fen_adamw, n, ptr(self.flat_p), ptr(self.flat_g), ptr(self.flat_m), ptr(self.flat_v),
               ptr(self.scal), b1, b2, float(self.eps))

    # ------------------------------------------------------------------ run
    def pack(self):
        self.Wt.pack()

    def forward(self, x: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Inference: x NCHW fp32 [B,3,h,w] -> out NCHW fp32 [B,3,H,W] (eval: clamped)."""
        L.check_strip_status()
        if x is not None:
            self.x.copy_(x)
        self.ctx.run()
        return self.out

    def step(self, hr: Optional[torch.Tensor] = None, update: bool = True) -> torch.Tensor:
        """One training step on HR [B,3,H,W]: LR synthesis, fwd, L1 (+ perceptual), bwd,
        all-reduce, clip, AdamW (the last three skipped without `update`: a non-stepping batch
        under accumulation).  Returns the (device) total loss of this rank's shard."""
        L.check_strip_status()
        if hr is not None:
            self.hr.copy_(hr)
        self.ctx.run()
        self.exchange.wait()
        if not update:
            return self.total_loss()
        self.upd.run()
        self.Wt.pack()
        from ..training.optim import bump_versions
        bump_versions(self._model_params)   # the module path re-packs the updated weights
        return self.total_loss()

    def total_loss(self) -> torch.Tensor:
        """weight * L1 (+ the weighted perceptual term), on the device."""
        if self.vgg is None and not self.ssim_weight:
            return self.loss if self.l1_weight == 1.0 else self.loss * self.l1_weight
        t = self.loss * self.l1_weight
        if self.vgg is not None:
            t = t + self.loss_perc
        if self.ssim_weight:
            t = t + self.ssim_weight * (1 - self.ssim_val)
        return t

    def set_lr(self, lr: float):
        self.scal[3] = lr

    @property
    def grad_norm(self) -> torch.Tensor:
        return self.scal[0]

    def capture(self):
        """Capture one forward (inference) or one full training step in a hipGraph.  At N > 1
        the step's bucket all-reduces are recorded too: the exchange is stream-ordered (RCCL on
        a side stream forked from the capture stream at each bucket's mark, joined before the
        update), so a replay is the whole DP step with no host round trip."""
        if self.train and self.world > 1 and not getattr(self.exchange, "capturable", False):
            raise RuntimeError("graph capture of the DP step needs a stream-ordered exchange")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm-up on the side stream (allocator + lazy init)
            self._replay_body()
        torch.cuda.current_stream().wait_stream(s)
        if self.train:              # the warm-up was a training step
            from ..training.optim import bump_versions
            bump_versions(self._model_params)
        g = torch.cuda.CUDAGraph()
        # thread-local capture: ProcessGroupNCCL's watchdog thread polls the warm-up step's
        # collectives with hipEventQuery, which a global-mode capture forbids process-wide
        torch.cuda.synchronize()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._replay_body()
        self.graph = g
        return g

    def _replay_body(self):
        self.ctx.run()
        if self.train:
            self.exchange.wait()
            self.upd.run()
            self.Wt.pack()

    def check_status(self) -> None:
        """Raise FenError if a strip launch of an earlier step reported a timed-out hand-off wait
        (forward / step / replay check before they enqueue; call this after the last step, once
        the stream has drained, to cover it too)."""
        L.check_strip_status()

    def replay(self):
        L.check_strip_status()
        self.graph.replay()
        if self.train:
            from ..training.optim import bump_versions
            bump_versions(self._model_params)
