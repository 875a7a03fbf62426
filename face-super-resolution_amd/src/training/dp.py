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
    """Async SUM all-reduce of arena slices, joined by `wait()`; a no-op at world size 1."""

    def __init__(self, flat: torch.Tensor, plan: Sequence[Bucket], group=None):
        self.flat, self.group = flat, group
        self.views = {tag: flat[lo:hi] for tag, lo, hi in plan}
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.works: List = []

    def launch(self, tag: str) -> None:
        if self.world > 1:
            self.works.append(dist.all_reduce(self.views[tag], group=self.group, async_op=True))

    def wait(self) -> None:
        for w in self.works:
            w.wait()
        self.works = []


def broadcast_arena(flat: torch.Tensor, src: int = 0, group=None) -> None:
    """Identical start on every rank: rank `src`'s parameters overwrite the others."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)
