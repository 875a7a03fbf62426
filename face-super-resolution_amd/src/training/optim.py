"""clip_grad_norm_ + AdamW over one flat fp32 parameter/gradient arena, on the GPU
(reference trainer.py:217-221 optimizer, 490-503 clip + step).

Three launches per step (fen_sumsq -> fen_optim_prepare -> fen_adamw), no host sync: the
global grad norm, the clip coefficient and the bias corrections are computed on the
device.  `state_dict()` / `load_state_dict()` speak torch.optim.AdamW's format so
checkpoints interchange with the reference's Trainer (trainer.py:701-760).
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ..hip import lib as L
from ..hip.program import Ctx, ptr


def adamw_state(flat_p: torch.Tensor):
    """(exp_avg, exp_avg_sq, scal) for a flat arena; scal = [grad norm, clip coef, step, lr,
    bias corrections...] as fen_optim_prepare / fen_adamw read and write it."""
    return torch.zeros_like(flat_p), torch.zeros_like(flat_p), torch.zeros(8, device=flat_p.device)


def bump_versions(params) -> None:
    """The update kernels write the parameters through raw pointers, which torch's version
    counters do not see; bump them, so everything keyed on `p._version` (the module path's
    packed-weight caches: hip/autograd.py LiveWeights, the discriminator's packs) re-packs
    before the next forward instead of running on the pre-update weights."""
    for p in params:
        torch.autograd.graph.increment_version(p)


def state_view(params, state, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0) -> "FusedAdamW":
    """A FusedAdamW over an existing state triple without a step program: for state_dict()
    and load_state_dict() only."""
    opt = FusedAdamW.__new__(FusedAdamW)
    opt.params = list(params)
    opt.m, opt.v, opt.scal = state
    opt.lr, opt.betas, opt.eps, opt.wd = float(lr), betas, eps, weight_decay
    return opt


class FusedAdamW:
    def __init__(self, params: List[torch.nn.Parameter], flat_p: torch.Tensor, flat_g: torch.Tensor, lr=1e-4,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_norm=0.0, state=None):
        """state: an existing (m, v, scal) triple to step on (the Trainer's one generator
        state, shared with the fused engine's update program), else fresh zeros."""
        self.params = list(params)
        self.flat_p, self.flat_g = flat_p, flat_g
        dev = flat_p.device
        if state is None:
            state = adamw_state(flat_p)
        self.m, self.v, self.scal = state
        self.betas, self.eps, self.wd, self.max_norm = betas, eps, weight_decay, max_norm
        self.set_lr(lr)
        n = flat_p.numel()
        self.ctx = Ctx(torch.float32, dev, record=True)
        lib = self.ctx.lib
        nparts = lib.fen_sumsq_parts(n)
        self.part = torch.zeros(nparts, device=dev)
        b1, b2 = betas
        self.ctx.emit("sumsq", lib.fen_sumsq, n, ptr(flat_g), ptr(self.part))
        self.ctx.emit("optim_prepare", lib.fen_optim_prepare, nparts, ptr(self.part), float(max_norm), b1, b2,
                      float(weight_decay), ptr(self.scal))
        self.ctx.emit("adamw", lib.fen_adamw, n, ptr(flat_p), ptr(flat_g), ptr(self.m), ptr(self.v), ptr(self.scal),
                      b1, b2, float(eps))

    def set_lr(self, lr: float):
        # (inside a graph capture the device value is left as it is: a host write cannot be
        # captured, and the trainer sets the rate before each replay instead)
        self.lr = float(lr)
        if not torch.cuda.is_current_stream_capturing():
            self.scal[3] = self.lr

    def step(self):
        self.ctx.run()
        bump_versions(self.params)

    @property
    def grad_norm(self) -> torch.Tensor:
        return self.scal[0]

    @property
    def steps(self) -> int:
        return int(self.scal[2])

    # ---- torch.optim.AdamW-compatible state ----
    def _views(self, flat):
        out, off = [], 0
        for p in self.params:
            out.append(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out

    def state_dict(self) -> Dict:
        step = torch.tensor(float(self.scal[2]))
        ms, vs = self._views(self.m), self._views(self.v)
        state = {i: {"step": step.clone(), "exp_avg": ms[i].detach().cpu().clone(),
                     "exp_avg_sq": vs[i].detach().cpu().clone()} for i in range(len(self.params))}
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd, "amsgrad": False,
                 "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "params": list(range(len(self.params)))}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd: Dict) -> None:
        ms, vs = self._views(self.m), self._views(self.v)
        step = 0.0
        for i, st in sd.get("state", {}).items():
            i = int(i)
            ms[i].copy_(st["exp_avg"])
            vs[i].copy_(st["exp_avg_sq"])
            step = float(st["step"])
        self.scal[2] = step
        if sd.get("param_groups"):
            self.set_lr(sd["param_groups"][0]["lr"])


class HipAdamW(torch.optim.AdamW):
    """torch.optim.AdamW whose step runs as two HIP launches over every parameter tensor
    (fen_adamw_multi) instead of torch's multi-tensor passes: the discriminator's optimizer_d
    (reference trainer.py:230-250, 446-451).  Same constructor, param_groups, per-parameter state
    (exp_avg, exp_avg_sq, a float32 step tensor on the device: torch's capturable form) and
    state_dict, so schedulers, checkpoints and the captured GAN iteration see a torch AdamW.
    amsgrad / maximize / differentiable groups fall back to torch's own step."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, **kw):
        kw.setdefault("capturable", True)
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, **kw)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            if group.get("amsgrad") or group.get("maximize") or group.get("differentiable"):
                raise NotImplementedError("HipAdamW: amsgrad / maximize / differentiable groups")
            jobs = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32 or not p.is_cuda:
                    raise RuntimeError("HipAdamW: dense fp32 GPU parameters only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                elif not (torch.is_tensor(st["step"]) and st["step"].is_cuda):
                    st["step"] = torch.tensor(float(st["step"]), dtype=torch.float32, device=p.device)
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                for t in (p, st["exp_avg"], st["exp_avg_sq"]):
                    if not t.is_contiguous():
                        raise RuntimeError("HipAdamW: contiguous parameters and moments only")
                jobs.append(L.AdamwJob(ptr(p), ptr(g), ptr(st["exp_avg"]), ptr(st["exp_avg_sq"]), ptr(st["step"]),
                                       p.numel()))
            b1, b2 = group["betas"]
            lib = L.load()
            # the kernel writes the parameters behind torch's version counters: bump them, so
            # the packed-weight caches keyed on p._version (the discriminator's) re-pack
            bump_versions([p for p in group["params"] if p.grad is not None])
            for i in range(0, len(jobs), 48):
                chunk = jobs[i:i + 48]
                arr = (L.AdamwJob * len(chunk))(*chunk)
                L.check(lib.fen_adamw_multi(len(chunk), arr, float(group["lr"]), float(b1), float(b2), 1.0 - b1, 1.0 - b2,
                                            float(group["eps"]), float(group["weight_decay"]),
                                            torch.cuda.current_stream().cuda_stream), "adamw_multi")
        return loss
