"""Training loop with the reference's API (src/training/trainer.py), data-parallel on MI355X.

Same TrainerConfig fields/defaults, EarlyStopping, Trainer(model, train_loader, val_loader,
loss_fn, config) with train / _train_epoch / _validate_epoch / _save_checkpoint /
load_checkpoint, and overfit_test.  What changes (trainer row):
  * the G step: with an L1 content loss the whole step -- on-device LR synthesis
    (trainer.py:416-421), forward, L1, backward, clip_grad_norm_, AdamW (458-503) -- is the
    fused HIP program of src.hip.engine.FENEngine (one hipGraph-able replay);
  * data parallel: one process per GPU (torchrun), each rank steps on its shard of the
    batch stream (src.data.rank_shard: equal-count shards per rank), gradients are summed by RCCL
    all-reduce buckets issued from inside the backward and overlapped with it; clip and
    AdamW run after the reduce so every rank stays identical; rank 0 logs/checkpoints;
  * one generator AdamW state (exp_avg / exp_avg_sq / step over the flat parameter arena)
    shared by every fused engine and the module-path optimizer of the GAN / generic steps,
    as the reference keeps one torch AdamW across all of them (trainer.py:217-221);
  * checkpoints keep the reference's dict layout (model/optimizer/scheduler state dicts,
    torch.optim.AdamW-format optimizer state, the discriminator and its optimizer for
    stage 3, trainer.py:701-760).
Out of scope here: W&B logging and sample-image grids.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..hip.engine import FENEngine, flatten_params
from ..hip.lib import check_strip_status
from ..hip.program import Ctx, ptr
from .dp import broadcast_arena
from .optim import FusedAdamW, HipAdamW, adamw_state, bump_versions, state_view


@dataclass
class TrainerConfig:
    """Configuration for trainer (reference trainer.py:85-131)."""
    epochs: int = 50
    learning_rate: float = 1e-4
    weight_decay: float = 1e-4
    gradient_clip: float = 1.0
    accumulation_steps: int = 1
    use_amp: bool = True
    scheduler_type: str = "cosine"
    scheduler_T_max: int = 50
    scheduler_eta_min: float = 1e-7
    scheduler_step_size: int = 10
    scheduler_gamma: float = 0.5
    early_stopping_patience: int = 10
    early_stopping_metric: str = "val_psnr"
    early_stopping_mode: str = "max"
    checkpoint_dir: str = "checkpoints"
    save_every: int = 10
    save_best: bool = True
    log_every: int = 100
    log_images_every: int = 5
    use_wandb: bool = True
    wandb_project: str = "face-super-resolution"
    device: str = "cuda"
    gan_weight: float = 0.0
    gan_type: str = "vanilla"
    d_learning_rate: float = 1e-4
    d_weight_decay: float = 0.0
    d_updates_per_g: int = 1
    gan_start_epoch: int = 0
    # (HIP extension) stage-3 iterations replay from one captured hipGraph after two eager
    # warm-up iterations -- world size 1; re-captured when the batch shape or a learning rate
    # changes; results identical to the eager iteration (tests/test_gpu_gan_capture.py)
    capture_gan_step: bool = True
    # (HIP extension) the generator step's pass through D takes no gradient for D's parameters:
    # the reference computes them (trainer.py:458-475) and never uses them -- optimizer_d has
    # already stepped, and its next zero_grad() drops them before the next D update -- so every
    # weight update is identical (tests/test_gpu_gan_step.py); only D's .grad after an
    # iteration differs (the D step's gradients alone).  False: the reference's dead work too.
    freeze_d_in_g_step: bool = True
    # (HIP extension) the iteration's generator forward runs once: the reference runs it twice
    # on the same LR batch with the same weights -- under no_grad for the D step(s), again with
    # grad for the G step (trainer.py:430-431, 461) -- so the D step takes the G step's output,
    # detached (the same values; the G weights do not move in between).  False: both passes.
    reuse_g_forward: bool = True


class EarlyStopping:
    """Patience-based early stopping (reference trainer.py:134-164)."""

    def __init__(self, patience: int = 10, mode: str = "max", min_delta: float = 0.0):
        self.patience, self.mode, self.min_delta = patience, mode, min_delta
        self.counter = 0
        self.best_score = None
        self.should_stop = False

    def __call__(self, score: float) -> bool:
        if self.best_score is None:
            self.best_score = score
            return False
        better = score > self.best_score + self.min_delta if self.mode == "max" else \
            score < self.best_score - self.min_delta
        if better:
            self.best_score, self.counter = score, 0
        else:
            self.counter += 1
            if self.counter >= self.patience:
                self.should_stop = True
        return self.should_stop


def dist_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def reduce_val_metrics(tl: float, tp: float, ts: float, n: int, world: int, device=None):
    """Per-rank validation sums -> the global batch means (trainer.py:552-619 computes the mean
    over all validation batches).  Under DP every rank validates its own shard, so the sums and
    batch counts are all-reduced first: every rank then sees the same metrics, so plateau
    scheduling, best-model selection and early stopping decide identically on every rank (a
    rank-local decision would let one rank leave train() while the others block in the next
    all-reduce)."""
    if world > 1:
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([tl, tp, ts, float(n)], dtype=torch.float64, device=device)
        dist.all_reduce(t)
        tl, tp, ts, n = t.tolist()
    n = max(n, 1)
    return {"loss": tl / n, "psnr": tp / n, "ssim": ts / n}


def bicubic_down4(hr: torch.Tensor) -> torch.Tensor:
    """trainer.py:416-421 LR synthesis on the GPU (fen_bicubic_down4)."""
    B, C, H, W = hr.shape
    hr = hr.contiguous().float()
    lr = torch.empty(B, C, H // 4, W // 4, device=hr.device)
    c = Ctx(torch.float32, hr.device)
    c.emit("bicubic_down4", c.lib.fen_bicubic_down4, B, C, H, W, ptr(hr), ptr(lr))
    return lr


class Trainer:
    """Single-node, multi-GPU training manager for FaceEnhanceNet (reference trainer.py:167-760)."""

    def __init__(self, model: nn.Module, train_loader, val_loader, loss_fn: nn.Module,
                 config: Optional[TrainerConfig] = None, discriminator: Optional[nn.Module] = None,
                 gan_loss: Optional[nn.Module] = None):
        self.config = config or TrainerConfig()
        self.rank, self.world = dist_info()
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if not torch.cuda.is_available():
            raise RuntimeError("the MI355X trainer needs a ROCm GPU (there is no CPU path)")
        self.device = torch.device("cuda", local)
        torch.cuda.set_device(self.device)
        self.model = model.to(self.device)
        if self.world > 1:  # identical start on every rank (RCCL broadcast of the flat arena)
            flatten_params(self.model, self.device)
            broadcast_arena(self.model._fen_flat, src=0)
        elif getattr(self.model, "_fen_flat", None) is None:
            flatten_params(self.model, self.device)
        self.train_loader, self.val_loader = train_loader, val_loader
        self.loss_fn = loss_fn.to(self.device) if loss_fn is not None else None
        self.fused_l1 = getattr(loss_fn, "fused_l1_weight", None)
        self.fused_perceptual = getattr(loss_fn, "fused_perceptual", None)
        self.fused_ssim = getattr(loss_fn, "fused_ssim_weight", 0.0)
        if self.fused_l1 is None and isinstance(loss_fn, nn.L1Loss):
            self.fused_l1 = 1.0
        # torch AdamW object = param_groups/lr holder for the schedulers and the checkpoint
        # format; the update itself is the fused HIP kernel
        self.optimizer = torch.optim.AdamW(self.model.parameters(), lr=self.config.learning_rate,
                                           weight_decay=self.config.weight_decay)
        self.scheduler = self._create_scheduler()
        # the generator's one AdamW state: every engine's update program and the module-path
        # FusedAdamW step on these buffers, so switching paths keeps moments and step count
        self.adam_state = adamw_state(self.model._fen_flat)
        self.adam_state[2][3] = self.lr
        self._engines: Dict[tuple, FENEngine] = {}
        self._generic_opt: Optional[FusedAdamW] = None
        self._flat_g: Optional[torch.Tensor] = None
        # stage-3 GAN (trainer.py:230-250): the reference's discriminator optimizer object
        self.use_gan = self.config.gan_weight > 0 and discriminator is not None
        self.discriminator = self.optimizer_d = self.gan_loss = None
        if self.use_gan:
            from ..models.discriminator import GANLoss
            self.discriminator = discriminator.to(self.device)
            self.gan_loss = gan_loss.to(self.device) if gan_loss is not None else GANLoss(self.config.gan_type)
            # torch.optim.AdamW's state and format, its step on the HIP multi-tensor kernel
            self.optimizer_d = HipAdamW(self.discriminator.parameters(), lr=self.config.d_learning_rate,
                                        weight_decay=self.config.d_weight_decay)
            self._make_d_capturable()
        self._gan_graph: Optional[dict] = None
        self._gan_eager_left = 2
        # data-parallel gradient exchanges of the module-autograd path (generator, discriminator):
        # bucketed, launched from post-accumulate hooks as the backward completes each bucket,
        # stream-ordered (capturable); built on first use.  _dp_force: exchange at world size 1
        # too (the one-rank RCCL tests)
        self._g_ex = self._d_ex = None
        self._dp_force = False
        self.early_stopping = EarlyStopping(self.config.early_stopping_patience, self.config.early_stopping_mode)
        self.checkpoint_dir = Path(self.config.checkpoint_dir)
        if self.rank == 0:
            self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        self.best_metric = None
        self.current_epoch = 0
        self.global_step = 0
        self.training_history: Dict[str, List] = {"train_loss": [], "val_loss": [], "val_psnr": [], "val_ssim": [],
                                                  "learning_rate": []}
        self.use_wandb = False

    # ------------------------------------------------------------------ pieces
    def _create_scheduler(self):
        c = self.config
        if c.scheduler_type == "cosine":
            return torch.optim.lr_scheduler.CosineAnnealingLR(self.optimizer, T_max=c.scheduler_T_max,
                                                              eta_min=c.scheduler_eta_min)
        if c.scheduler_type == "step":
            return torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=c.scheduler_step_size,
                                                   gamma=c.scheduler_gamma)
        if c.scheduler_type == "plateau":
            return torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, mode="max", factor=0.5, patience=5)
        return None

    @property
    def lr(self) -> float:
        return self.optimizer.param_groups[0]["lr"]

    def engine(self, B: int, H: int, W: int) -> FENEngine:
        key = (B, H, W)
        if key not in self._engines:
            dtype = self.model.compute_dtype
            eng = FENEngine(self.model, batch=B, lr_hw=(H // self.model.scale_factor, W // self.model.scale_factor),
                            dtype=dtype, train=True, device=self.device, loss_weight=self.fused_l1,
                            clip=self.config.gradient_clip, lr=self.lr, weight_decay=self.config.weight_decay,
                            perceptual=self.fused_perceptual, ssim_weight=self.fused_ssim,
                            adam_state=self.adam_state, accumulation_steps=self._accum())
            self._engines[key] = eng
        return self._engines[key]

    def _shard(self, hr: torch.Tensor) -> torch.Tensor:
        """If the loader hands every rank the global batch, keep this rank's slice."""
        if self.world > 1 and getattr(self.train_loader, "_fen_global_batches", False):
            return hr.chunk(self.world)[self.rank]
        return hr

    def _dp_exchanges(self) -> None:
        """The generator's gradients land in `_flat_g` (the fused AdamW's arena) bucket by bucket
        -- tail, rg{G-1}..rg0, head: dp.bucket_plan's groups -- each all-reduced as soon as the
        backward completes it; the discriminator's in two buckets, copied back into `.grad` for
        optimizer_d.  Only when exchanging (world > 1, or forced)."""
        if self._flat_g is None:
            self._flat_g = torch.zeros_like(self.model._fen_flat)
        if not (self.world > 1 or self._dp_force) or self._g_ex is not None:
            return
        from .dp import ParamGradExchange, _group_of, even_buckets
        names = [n for n, _ in self.model.named_parameters()]
        runs, a = [], 0
        for i in range(1, len(names) + 1):
            if i == len(names) or _group_of(names[i]) != _group_of(names[a]):
                runs.append((a, i))
                a = i
        self._g_ex = ParamGradExchange(list(self.model.parameters()), self._flat_g, runs, force=self._dp_force)
        if self.use_gan:
            dps = list(self.discriminator.parameters())
            dflat = torch.zeros(sum(p.numel() for p in dps), device=self.device)
            self._d_ex = ParamGradExchange(dps, dflat, even_buckets(len(dps), 2), force=self._dp_force,
                                           copy_back=True)

    def _generic_step(self, hr: torch.Tensor, update: bool = True) -> torch.Tensor:
        """Any other content loss: module autograd path + RCCL grad all-reduce + fused AdamW
        (only on the accumulation step, `update`; the loss is divided by accumulation_steps as
        trainer.py:477 does)."""
        self._dp_exchanges()
        lr = bicubic_down4(hr)
        sr = self.model(lr)
        loss = self._content(sr, hr)
        for p in self.model.parameters():
            p.grad = None
        if update and self._g_ex is not None:
            self._g_ex.arm()
        (loss / (self.world * self._accum())).backward()
        if update:
            self._apply_generic_update()
        return loss.detach()

    def _content(self, sr: torch.Tensor, hr: torch.Tensor) -> torch.Tensor:
        """The content loss: CombinedLoss returns (loss, components) (combined.py:158-203), a
        plain criterion a tensor; L1 without a loss function."""
        if self.loss_fn is None:
            from ..losses import L1Loss
            return L1Loss()(sr, hr)
        out = self.loss_fn(sr, hr)
        return out[0] if isinstance(out, tuple) else out

    def _gan_step(self, hr: torch.Tensor, update: bool = True) -> torch.Tensor:
        """One stage-3 iteration (trainer.py:424-485): d_updates_per_g discriminator updates on
        real vs detached fake, then the generator on content + gan_weight x adversarial loss.
        Both networks run on the HIP path through their module autograd."""
        D, gl = self.discriminator, self.gan_loss
        self._dp_exchanges()
        lr = bicubic_down4(hr)
        D.train()
        reuse = getattr(self.config, "reuse_g_forward", True)
        sr = self.model(lr) if reuse else None
        for _ in range(self.config.d_updates_per_g):
            self.optimizer_d.zero_grad()
            if reuse:
                sr_d = sr.detach()
            else:
                with torch.no_grad():
                    sr_d = self.model(lr)
            # (the HIP discriminator takes both batches in one pass, per-batch BatchNorm statistics)
            d_real, d_fake = D.forward_pair(hr, sr_d.detach()) if hasattr(D, "forward_pair") else \
                (D(hr), D(sr_d.detach()))
            d_loss = (gl(d_real, True) + gl(d_fake, False)) / 2
            if self._d_ex is not None:
                self._d_ex.arm()
            (d_loss / self.world).backward()
            if self._d_ex is not None:
                self._d_ex.wait()        # D's two buckets, all-reduced as the backward completed them
            self.optimizer_d.step()
        if not reuse:
            sr = self.model(lr)
        content = self._content(sr, hr)
        frozen = []
        if getattr(self.config, "freeze_d_in_g_step", True):
            frozen = [p for p in D.parameters() if p.requires_grad]
            for p in frozen:
                p.requires_grad_(False)
        try:
            adv = gl(D(sr), True)
        finally:
            for p in frozen:
                p.requires_grad_(True)
        loss = content + self.config.gan_weight * adv
        for p in self.model.parameters():
            p.grad = None
        if update and self._g_ex is not None:
            self._g_ex.arm()
        (loss / (self.world * self._accum())).backward()
        if update:
            self._apply_generic_update()
        return loss.detach()

    def _capture_gan(self) -> bool:
        """Captured at world size 1, and with an exchange whose bucket all-reduces are direct
        RCCL calls (dp.RcclComm, the C-ABI's fen_rccl_allreduce_bucket: the tests' forced one-rank
        group, or N > 1 with FEN_DP_COMM=rccl) -- they record into the graph from autograd's hook
        thread like any kernel, no ProcessGroupNCCL work, event or watchdog involved (the round-4
        watchdog abort).  With torch's collectives (the default at N > 1 until the
        direct path has run on two or more GPUs, dp.use_direct_rccl) the iteration runs eagerly
        unless FEN_GAN_CAPTURE_DP=1; gloo never captures."""
        import os
        from .dp import _rccl_capture_ok, use_direct_rccl
        if not (bool(self.config.capture_gan_step) and torch.cuda.is_available() and self._accum() == 1):
            return False
        if self.world > 1 or getattr(self, "_dp_force", False):
            if use_direct_rccl():
                return True
            return (os.environ.get("FEN_GAN_CAPTURE_DP") == "1" and dist.is_available() and dist.is_initialized()
                    and _rccl_capture_ok())
        return True

    def _make_d_capturable(self) -> None:
        """The captured GAN iteration steps optimizer_d inside the graph: its param groups need
        `capturable` and its per-parameter step counts on the device as float32.  Also after
        load_state_dict, which restores the saved groups' flag (False in checkpoints of the
        reference trainer, of a DP run or of a run without capture) and CPU step counts."""
        if not self._capture_gan():
            return
        for g in self.optimizer_d.param_groups:
            g["capturable"] = True
        for st in self.optimizer_d.state.values():
            if "step" in st:
                v = st["step"]
                st["step"] = (v.to(self.device, torch.float32) if torch.is_tensor(v)
                              else torch.tensor(float(v), dtype=torch.float32, device=self.device))

    def _accum(self) -> int:
        return max(1, int(self.config.accumulation_steps))

    def _gan_iteration(self, hr: torch.Tensor, update: bool = True) -> torch.Tensor:
        """_gan_step, eagerly or (config.capture_gan_step) replayed from a hipGraph: the first
        two iterations run eagerly (lazy initialisation, allocator warm-up), the third is
        captured and every later one copies its batch into the captured input and replays.
        The update kernels write the parameters behind torch's version counters, so both
        networks' counters are bumped after a replay (the module path then re-packs)."""
        if not self._capture_gan():
            return self._gan_step(hr, update)
        key = (tuple(hr.shape), float(self.lr), tuple(float(g["lr"]) for g in self.optimizer_d.param_groups),
               self.config.d_updates_per_g)
        st = self._gan_graph
        if st is not None and st["key"] != key:
            self._gan_graph = st = None
        if st is None:
            if self._gan_eager_left > 0:
                self._gan_eager_left -= 1
                return self._gan_step(hr)
            static_hr = hr.detach().clone()
            graph = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            # thread-local: the RCCL watchdog thread's event polls stay legal (FENEngine.capture)
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                loss = self._gan_step(static_hr)
            st = self._gan_graph = {"graph": graph, "hr": static_hr, "loss": loss, "key": key}
        st["hr"].copy_(hr)
        if self._generic_opt is not None:
            self._generic_opt.set_lr(self.lr)
        st["graph"].replay()
        bump_versions(list(self.model.parameters()) + list(self.discriminator.parameters()))
        return st["loss"]

    def _apply_generic_update(self):
        if self._flat_g is None:
            self._flat_g = torch.zeros_like(self.model._fen_flat)
        if self._generic_opt is None:
            flat = self.model._fen_flat
            self._generic_opt = FusedAdamW(list(self.model.parameters()), flat, self._flat_g, lr=self.lr,
                                           weight_decay=self.config.weight_decay, max_norm=self.config.gradient_clip,
                                           state=self.adam_state)
        if getattr(self, "_flat_g_views", None) is None:
            self._flat_g_views, off = [], 0
            for p in self.model.parameters():
                self._flat_g_views.append(self._flat_g[off:off + p.numel()].view_as(p))
                off += p.numel()
        if self._g_ex is not None:
            self._g_ex.wait()            # the buckets, copied and all-reduced during the backward
        else:
            # one multi-tensor copy (a few launches) instead of one copy per parameter (444 here)
            torch._foreach_copy_(self._flat_g_views, [p.grad for p in self.model.parameters()])
            if self.world > 1:
                dist.all_reduce(self._flat_g)
        self._generic_opt.set_lr(self.lr)
        self._generic_opt.step()

    # ------------------------------------------------------------------ loops
    def _train_epoch(self) -> Dict[str, float]:
        """trainer.py:390-550.  accumulation_steps = k as the reference runs it: every batch
        zeroes the generator's gradients (trainer.py:457) and back-propagates loss / k
        (477-485); every k-th batch clips and steps (488-503) -- so the step sees the last
        batch's gradient / k -- and counts a global step; the tracked loss is the undivided
        one (508)."""
        self.model.train()
        total, n = 0.0, 0
        k = self._accum()
        ds = getattr(self.train_loader, "dataset", None)
        if hasattr(ds, "set_epoch"):
            ds.set_epoch(self.current_epoch)     # fresh per-sample augmentation draws each epoch
        for bi, batch in enumerate(self.train_loader):
            hr = self._shard(batch["hr"]).to(self.device, non_blocking=True)
            update = (bi + 1) % k == 0
            if self.use_gan and self.current_epoch >= self.config.gan_start_epoch:
                loss = self._gan_iteration(hr, update)
            elif self.fused_l1 is not None:
                B, _, H, W = hr.shape
                eng = self.engine(B, H, W)
                eng.set_lr(self.lr)
                loss = eng.step(hr, update=update)
            else:
                loss = self._generic_step(hr, update)
            if update:
                self.global_step += 1
            total += float(loss)  # per-step host sync, as trainer.py:508
            check_strip_status()  # ... so a strip launch's timed-out wait raises at its own step
            n += 1
        if self.world > 1:
            t = torch.tensor([total, n], device=self.device, dtype=torch.float64)
            dist.all_reduce(t)
            total, n = float(t[0]), int(t[1])
        return {"loss": total / max(n, 1), "l1": total / max(n, 1)}

    @torch.no_grad()
    def _validate_epoch(self) -> Dict[str, float]:
        """trainer.py:552-619 (sample grids / W&B images out of scope); DP: global means."""
        self.model.eval()
        tl, tp, ts, n = 0.0, 0.0, 0.0, 0
        for batch in self.val_loader:
            hr = batch["hr"].to(self.device)
            sr = self.model(bicubic_down4(hr))
            loss = self._content(sr, hr)
            tl += float(loss)
            tp += self._compute_psnr(sr, hr)
            ts += self._compute_ssim(sr, hr)
            n += 1
        return reduce_val_metrics(tl, tp, ts, n, self.world)

    def _compute_ssim(self, pred: torch.Tensor, target: torch.Tensor) -> float:
        """ssim(pred, target) with the reference defaults (trainer.py:630-634), on the HIP kernel."""
        from ..losses.ssim import ssim
        return float(ssim(pred, target))

    def _compute_psnr(self, pred: torch.Tensor, target: torch.Tensor) -> float:
        """10 log10(1/MSE) over the batch (trainer.py:621-628)."""
        mse = torch.mean((pred - target) ** 2)
        if mse == 0:
            return float("inf")
        return float(10 * torch.log10(1.0 / mse))

    def train(self) -> Dict[str, Any]:
        for epoch in range(self.current_epoch, self.config.epochs):
            self.current_epoch = epoch
            tm = self._train_epoch()
            vm = self._validate_epoch() if self.val_loader is not None else {"loss": tm["loss"], "psnr": 0.0,
                                                                             "ssim": float("nan")}
            if self.scheduler is not None:
                if self.config.scheduler_type == "plateau":
                    self.scheduler.step(vm["psnr"])
                else:
                    self.scheduler.step()
            self._log_epoch_metrics(epoch, tm, vm, self.lr)
            if (epoch + 1) % self.config.save_every == 0:
                self._save_checkpoint(f"epoch_{epoch + 1}.pth")
            metric = vm.get(self.config.early_stopping_metric.replace("val_", ""), vm.get("psnr", 0))
            if self.config.save_best and self._is_best(metric):
                self._save_checkpoint("best_model.pth", is_best=True)
            if self.early_stopping(metric):
                if self.rank == 0:
                    print(f"\nEarly stopping triggered at epoch {epoch + 1}")
                break
        self._save_checkpoint("final_model.pth")
        return self.training_history

    def _log_epoch_metrics(self, epoch, tm, vm, lr):
        h = self.training_history
        h["train_loss"].append(tm["loss"])
        h["val_loss"].append(vm["loss"])
        h["val_psnr"].append(vm["psnr"])
        h["val_ssim"].append(vm["ssim"])
        h["learning_rate"].append(lr)
        if self.rank == 0:
            print(f"\nEpoch {epoch + 1}/{self.config.epochs}\n  Train Loss: {tm['loss']:.4f}\n"
                  f"  Val Loss:   {vm['loss']:.4f}\n  Val PSNR:   {vm['psnr']:.2f} dB\n  LR:         {lr:.2e}")

    def _is_best(self, value: float) -> bool:
        if self.best_metric is None:
            self.best_metric = value
            return True
        better = value > self.best_metric if self.config.early_stopping_mode == "max" else value < self.best_metric
        if better:
            self.best_metric = value
        return better

    # ------------------------------------------------------------------ checkpoints
    def _adam_view(self) -> FusedAdamW:
        return state_view(self.model.parameters(), self.adam_state, lr=self.lr,
                          weight_decay=self.config.weight_decay)

    def _optimizer_state(self) -> Dict:
        """The generator's AdamW state in torch.optim.AdamW's format (empty before a step)."""
        view = self._adam_view()
        return view.state_dict() if view.steps > 0 else self.optimizer.state_dict()

    def _save_checkpoint(self, filename: str, is_best: bool = False) -> None:
        """Reference checkpoint layout (trainer.py:701-723); rank 0 only."""
        if self.rank != 0:
            return
        sd = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        ckpt = {
            "epoch": self.current_epoch,
            "global_step": self.global_step,
            "model_state_dict": sd,
            "optimizer_state_dict": self._optimizer_state(),
            "scheduler_state_dict": self.scheduler.state_dict() if self.scheduler else None,
            "best_metric": self.best_metric,
            "training_history": self.training_history,
            "config": dict(self.config.__dict__),
        }
        if self.use_gan:
            ckpt["discriminator_state_dict"] = {k: v.detach().cpu() for k, v in self.discriminator.state_dict().items()}
            ckpt["optimizer_d_state_dict"] = self.optimizer_d.state_dict()
        torch.save(ckpt, self.checkpoint_dir / filename)
        if is_best:
            print(f"  New best model saved: {self.best_metric:.4f}")

    def load_checkpoint(self, path: str, weights_only: bool = False) -> None:
        """Full resume or fine-tune (weights only) from a reference-format checkpoint
        (trainer.py:725-760).  Loaded with torch.load(weights_only=True)."""
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        self._gan_graph = None          # a captured iteration holds the pre-load state tensors
        self.model.load_state_dict(ckpt["model_state_dict"])
        if weights_only:
            return
        osd = ckpt.get("optimizer_state_dict")
        if osd:
            self.optimizer.load_state_dict(osd)
            self._adam_view().load_state_dict(osd)   # the one state both step paths use
        if self.scheduler and ckpt.get("scheduler_state_dict"):
            self.scheduler.load_state_dict(ckpt["scheduler_state_dict"])
        self.current_epoch = ckpt["epoch"] + 1
        self.global_step = ckpt["global_step"]
        self.best_metric = ckpt["best_metric"]
        self.training_history = ckpt["training_history"]
        if self.use_gan and "discriminator_state_dict" in ckpt:
            self.discriminator.load_state_dict(ckpt["discriminator_state_dict"])
            if ckpt.get("optimizer_d_state_dict"):
                self.optimizer_d.load_state_dict(ckpt["optimizer_d_state_dict"])
                self._make_d_capturable()


def overfit_test(model: nn.Module, dataloader, loss_fn: nn.Module, num_images: int = 10,
                 num_iterations: int = 1000, device: str = "cuda") -> Dict[str, Any]:
    """Overfit a few images with MSE on clamped output, Adam lr 2e-4 (reference trainer.py:763-848)."""
    dev = torch.device(device)
    model = model.to(dev).train()
    hr = next(iter(dataloader))["hr"][:num_images].to(dev)
    lr = bicubic_down4(hr)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4)
    losses, psnrs = [], []
    for _ in range(num_iterations):
        opt.zero_grad()
        sr = torch.clamp(model(lr), 0.0, 1.0)
        loss = F.mse_loss(sr, hr)
        loss.backward()
        opt.step()
        with torch.no_grad():
            psnrs.append(float(10 * torch.log10(1.0 / torch.mean((sr - hr) ** 2))))
        losses.append(float(loss))
    return {"final_loss": losses[-1], "final_psnr": psnrs[-1], "loss_history": losses, "psnr_history": psnrs,
            "converged": psnrs[-1] > 35}
