"""Data-parallel gradient exchange for the flat fp32 gradient arena.

One process per GPU.  The reference wraps the generator in DDP (`trainer.py:126-134`,
`scripts/train.py:325-330`); here the gradients of every parameter live in one flat fp32
arena in `named_parameters()` order, so each backward-ordered slice of the network is one
contiguous bucket:

    tail   conv_after_body + upsample + conv_last   (its grads complete first in backward)
    rg{G-1} ... rg0                                  (one residual group each, ~0.75 MB)
    head   conv_first                                (last)

`bucket_plan` computes those slices from the parameter names alone; `BucketExchange`
launches one async SUM all-reduce per bucket as the backward program reaches it (RCCL on
its own stream over xGMI; gloo on CPU in the tests) and joins them before the update.
Callers pre-scale the loss gradient by 1/world, so SUM = the gradient of the global-batch
mean loss, exactly the DDP semantics; clip and AdamW run after the join on every rank on
identical data (`trainer.py:490-503` ordering).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import torch
import torch.distributed as dist

Bucket = Tuple[str, int, int]  # (tag, lo, hi) element offsets into the flat arena


def init_rccl(device: torch.device, **kw) -> None:
    """`init_process_group("nccl")` for a graph-captured DP step.  ProcessGroupNCCL's event
    cache hands a finished eager collective's HIP events to the next collective; when that one
    is issued inside a capture, the event is re-recorded on a capturing stream while the
    watchdog thread (or the flight recorder's stale entry) may still query it, and the query
    fails with hipErrorCapturedEvent -- which the watchdog turns into an abort (seen once in
    three runs of tests/test_gpu_rccl.py's captured GAN iteration).  Fresh events per
    collective cost microseconds, and only on eager steps: a replayed graph creates none."""
    import os
    v = os.environ.get(EVENT_CACHE_VAR)
    if v not in (None, "0"):
        raise RuntimeError(f"{EVENT_CACHE_VAR}={v!r} is inherited from the environment; a captured DP "
                           "step needs it off (ProcessGroupNCCL re-records cached events inside the "
                           "capture). Unset it or set it to 0.")
    os.environ[EVENT_CACHE_VAR] = "0"
    # the flight recorder keeps every collective's events for its dumps; nothing here reads
    # them, and an entry recorded inside a capture is one more event a host-side query can
    # trip on (a user's explicit setting is kept)
    os.environ.setdefault("TORCH_NCCL_TRACE_BUFFER_SIZE", "0")
    dist.init_process_group("nccl", device_id=device, **kw)


EVENT_CACHE_VAR = "TORCH_NCCL_CUDA_EVENT_CACHE"


def exchange_capturable(group=None) -> bool:
    """Whether a collective on `group` may be recorded into a hipGraph: world size 1 (nothing
    is exchanged), or RCCL with the event cache off (what `init_rccl` sets up).  gloo stages
    CUDA tensors through the host, and a user's own `init_process_group('nccl')` with the
    event cache on can abort the watchdog inside a capture (see `init_rccl`)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return True
    return _rccl_capture_ok(group)


def _rccl_capture_ok(group=None) -> bool:
    import os
    return dist.get_backend(group) == "nccl" and os.environ.get(EVENT_CACHE_VAR) == "0"


def _group_of(name: str) -> str:
    if name.startswith("conv_first."):
        return "head"
    if name.startswith("residual_groups."):
        return "rg" + name.split(".")[1]
    return "tail"


def bucket_plan(named_numels: Iterable[Tuple[str, int]], num_groups: int) -> List[Bucket]:
    """Buckets in the order the backward completes them: tail, rg{G-1}..rg0, head.

    Raises if a bucket is not one contiguous slice of the arena (a parameter order the
    engine's arena does not produce)."""
    spans, off = {}, 0
    for name, n in named_numels:
        tag = _group_of(name)
        lo, hi = spans.get(tag, (off, off))
        if tag in spans and hi != off:
            raise ValueError(f"bucket {tag} is not contiguous in the parameter order (at {name})")
        spans[tag] = (lo, off + n)
        off += n
    order = ["tail"] + [f"rg{g}" for g in reversed(range(num_groups))] + ["head"]
    if set(spans) != set(order):
        raise ValueError(f"unexpected parameter groups {sorted(spans)} for {num_groups} residual groups")
    plan = [(t, *spans[t]) for t in order]
    if sum(hi - lo for _, lo, hi in plan) != off:
        raise ValueError("buckets do not tile the arena")
    return plan


def model_bucket_plan(model: torch.nn.Module) -> List[Bucket]:
    return bucket_plan(((n, p.numel()) for n, p in model.named_parameters()), len(model.residual_groups))


class BucketExchange:
    """SUM all-reduce of arena slices, one per bucket as the backward reaches it, joined by
    `wait()`; a no-op at world size 1 (unless `force`: the tests' one-rank RCCL group).

    On the GPU the exchange is stream-ordered and graph-capturable: `launch` forks a side
    stream from the current one (event record / wait -- the bucket's gradients are enqueued
    before the fork), issues the collective there (RCCL runs behind it on its own stream), and
    `wait` joins the side stream back into the current one.  No host synchronisation anywhere,
    so a whole DP training step (forward, backward with the bucket all-reduces overlapped, the
    join, clip, AdamW) records into one hipGraph.  On CPU tensors (gloo, the CPU tests) the
    collectives are async work handles joined by the host."""

    def __init__(self, flat: torch.Tensor, plan: Sequence[Bucket], group=None, force: bool = False):
        self.flat, self.group = flat, group
        self.plan = list(plan)
        self.views = {tag: flat[lo:hi] for tag, lo, hi in plan}
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.active = self.world > 1 or force
        # gloo stages CUDA tensors through the host (not stream-ordered): only RCCL captures,
        # and only with ProcessGroupNCCL's event cache off (init_rccl)
        self.capturable = bool(flat.is_cuda) and (not self.active or _rccl_capture_ok(group))
        self.stream = torch.cuda.Stream(device=flat.device) if (self.active and flat.is_cuda) else None
        self.works: List = []
        self._forked = False

    def launch(self, tag: str) -> None:
        if not self.active:
            return
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(self.stream):
                dist.all_reduce(self.views[tag], group=self.group)
            self._forked = True
        else:
            self.works.append(dist.all_reduce(self.views[tag], group=self.group, async_op=True))

    def wait(self) -> None:
        if self._forked:
            torch.cuda.current_stream(self.flat.device).wait_stream(self.stream)
            self._forked = False
        for w in self.works:
            w.wait()
        self.works = []


class ParamGradExchange:
    """Bucketed, overlapped gradient all-reduce for module-autograd parameters (the generator
    on the module path, the discriminator): each bucket is a run of parameters in
    `named_parameters()` order; a post-accumulate-grad hook per parameter counts its bucket's
    arrivals, and the bucket's last one copies the bucket's `.grad`s into its slice of `flat`
    (one multi-tensor copy) and launches that slice's all-reduce (BucketExchange: stream-
    ordered, capturable).  `wait()` joins; `flat` then holds the global-batch gradients (the
    caller's loss is pre-scaled by 1/world).  `copy_back` also writes them into the `.grad`s
    (for optimisers that read `.grad`).  Hooks fire only while `armed` (an accumulation batch
    that does not step exchanges nothing)."""

    def __init__(self, params: Sequence[torch.Tensor], flat: torch.Tensor, buckets: Sequence[Tuple[int, int]],
                 group=None, force: bool = False, copy_back: bool = False):
        self.params = list(params)
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o += p.numel()
        if o != flat.numel():
            raise ValueError("flat buffer does not match the parameters")
        self.flat, self.copy_back = flat, copy_back
        self.fviews = [flat[a:a + p.numel()].view_as(p) for a, p in zip(offs, self.params)]
        plan = []
        for i, (a, b) in enumerate(buckets):
            lo = offs[a]
            hi = offs[b - 1] + self.params[b - 1].numel()
            plan.append((f"b{i}", lo, hi))
        self.ranges = [(a, b) for a, b in buckets]
        self.ex = BucketExchange(flat, plan, group, force)
        self.world, self.active = self.ex.world, self.ex.active
        self.armed = False
        self._left = [b - a for a, b in self.ranges]
        self._hooks = []
        if self.active:
            for bi, (a, b) in enumerate(self.ranges):
                for i in range(a, b):
                    self._hooks.append(self.params[i].register_post_accumulate_grad_hook(
                        lambda _p, bi=bi: self._arrived(bi)))

    def _arrived(self, bi: int) -> None:
        if not self.armed:
            return
        self._left[bi] -= 1
        if self._left[bi] == 0:
            a, b = self.ranges[bi]
            torch._foreach_copy_(self.fviews[a:b], [p.grad for p in self.params[a:b]])
            self.ex.launch(f"b{bi}")

    def arm(self) -> None:
        self.armed = True
        self._left = [b - a for a, b in self.ranges]

    def wait(self) -> None:
        """Join; every bucket must have been launched by this backward."""
        if not self.armed:
            return
        if any(self._left):
            raise RuntimeError(f"gradient buckets not complete after backward: {self._left}")
        self.ex.wait()
        if self.copy_back:
            torch._foreach_copy_([p.grad for p in self.params], self.fviews)
        self.armed = False

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


def even_buckets(n: int, k: int) -> List[Tuple[int, int]]:
    """k contiguous runs of n parameters, the last run first in backward order."""
    k = max(1, min(k, n))
    cuts = [round(i * n / k) for i in range(k + 1)]
    return [(cuts[i], cuts[i + 1]) for i in range(k)]


def broadcast_arena(flat: torch.Tensor, src: int = 0, group=None) -> None:
    """Identical start on every rank: rank `src`'s parameters overwrite the others."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)
