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

Two collective paths on the GPU, chosen by `FEN_DP_COMM`:
- `rccl`: RCCL called directly through the C-ABI (`RcclComm`: `fen_rccl_allreduce_bucket`,
  include/fen.h): one ncclAllReduce per bucket on a side stream, no c10d Work object, no HIP
  events, no watchdog -- torch.distributed only carries the communicator's unique id.  That is
  what makes a capture of collectives issued from autograd's device thread (the module path's
  post-accumulate hooks) safe: ProcessGroupNCCL hands a work issued outside the capturing
  thread's view to its watchdog, whose event queries then fail with hipErrorCapturedEvent and
  abort the process (round 4).
- `torch`: torch.distributed's collectives (ProcessGroupNCCL = RCCL; gloo always uses them).
The default (`auto`) is the direct path on a one-rank communicator (what the one-GPU tests
exercise) and torch's collectives at world size > 1: the direct path has not yet run with
two or more GPUs, so a multi-GPU job takes the collective path torch itself validates until
it has (`FEN_DP_COMM=rccl` opts in).
"""
from __future__ import annotations

import collections
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
    if use_direct_rccl(group):
        return True
    return dist.get_backend(group) == "nccl" and os.environ.get(EVENT_CACHE_VAR) == "0"


def use_direct_rccl(group=None) -> bool:
    """Whether the exchange's collectives go through `RcclComm` (the C-ABI): FEN_DP_COMM=rccl
    on a process group whose backend is nccl (RCCL); FEN_DP_COMM=torch never; the default
    (auto) only on a one-rank group or without one (see the module docstring)."""
    import os
    mode = os.environ.get("FEN_DP_COMM", "auto")
    if mode not in ("auto", "rccl", "torch"):
        raise ValueError(f"FEN_DP_COMM={mode!r}: expected auto, rccl or torch")
    if mode == "torch":
        return False
    if not (dist.is_available() and dist.is_initialized()):
        return True
    if dist.get_backend(group) != "nccl":
        return False
    return mode == "rccl" or dist.get_world_size(group) == 1


class RcclComm:
    """One RCCL communicator over `group`'s ranks (one process per GPU), created through the
    C-ABI (`fen_rccl_init`): rank 0 makes the unique id, torch.distributed broadcasts it
    (the rendezvous is the only thing torch.distributed does here).  `allreduce(t, stream)`
    enqueues an in-place fp32 SUM of `t` on `stream` -- graph-capturable from any thread.
    Without an initialised process group it is a one-rank communicator (the tests)."""

    _cache = {}

    def __init__(self, device: torch.device, group=None):
        import ctypes
        from ..hip.lib import check, load
        lib = load()
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if dist_on else 0
        self.device = torch.device(device)
        uid = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            check(lib.fen_rccl_unique_id(uid.data_ptr()), "fen_rccl_unique_id")
        if self.world > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            t = uid.to(self.device)
            dist.broadcast(t, src=src, group=group)
            uid = t.cpu()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.fen_rccl_init(ctypes.byref(h), uid.data_ptr(), self.world, self.rank, self.device.index),
                  "fen_rccl_init")
        self.handle = h.value
        self.library = lib.fen_rccl_library().decode()

    @staticmethod
    def _key(device: torch.device, group=None):
        """(device, group, world, rank, backend): a communicator made before
        init_process_group (one rank) or under a destroyed and re-created default group is
        never handed to an exchange over a different set of ranks."""
        dist_on = dist.is_available() and dist.is_initialized()
        return (str(torch.device(device)), id(group),
                dist.get_world_size(group) if dist_on else 1, dist.get_rank(group) if dist_on else 0,
                str(dist.get_backend(group)) if dist_on else None)

    @classmethod
    def get(cls, device: torch.device, group=None) -> "RcclComm":
        """One communicator per (device, group, world, rank, backend) for the process (the
        engines, the module-path exchanges and the trainer share it)."""
        key = cls._key(device, group)
        c = cls._cache.get(key)
        if c is None:
            c = cls._cache[key] = cls(device, group)
        if c.world != key[2] or c.rank != key[3]:
            raise RuntimeError(f"RcclComm cache: communicator of world {c.world} rank {c.rank} under key {key}")
        return c

    def allreduce(self, t: torch.Tensor, stream: torch.cuda.Stream) -> None:
        from ..hip.lib import check, load
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
            raise ValueError("RcclComm.allreduce: a contiguous fp32 tensor on the communicator's device")
        check(load().fen_rccl_allreduce_bucket(self.handle, t.data_ptr(), t.numel(), stream.cuda_stream),
              "fen_rccl_allreduce_bucket")

    def check(self) -> None:
        from ..hip.lib import check, load
        check(load().fen_rccl_check(self.handle), "rccl")

    @classmethod
    def destroy_all(cls) -> None:
        from ..hip.lib import load
        for c in cls._cache.values():
            load().fen_rccl_destroy(c.handle)
        cls._cache = {}


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
        # direct RCCL (RcclComm) on the GPU; gloo stages CUDA tensors through the host (not
        # stream-ordered) and is never captured; torch's RCCL only with the event cache off
        self.comm = (RcclComm.get(flat.device, group) if (self.active and flat.is_cuda and use_direct_rccl(group))
                     else None)
        self.capturable = bool(flat.is_cuda) and (not self.active or _rccl_capture_ok(group))
        self.stream = torch.cuda.Stream(device=flat.device) if (self.active and flat.is_cuda) else None
        self.works: List = []
        self._forked = False
        self.base = None              # the stream launches fork from (default: the current one)
        # per launch: was the fork inside a capture (the last 256 launches; replays add none)
        self.captured_launches = collections.deque(maxlen=256)

    def launch(self, tag: str) -> None:
        if not self.active:
            return
        if self.stream is not None:
            base = self.base if self.base is not None else torch.cuda.current_stream(self.flat.device)
            self.stream.wait_stream(base)
            with torch.cuda.stream(self.stream):
                self.captured_launches.append(torch.cuda.is_current_stream_capturing())
                if self.comm is not None:
                    self.comm.allreduce(self.views[tag], self.stream)
                else:
                    dist.all_reduce(self.views[tag], group=self.group)
            self._forked = True
        else:
            self.works.append(dist.all_reduce(self.views[tag], group=self.group, async_op=True))

    def wait(self) -> None:
        if self._forked:
            base = self.base if self.base is not None else torch.cuda.current_stream(self.flat.device)
            base.wait_stream(self.stream)
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
        """Runs on autograd's device thread.  The copy and the fork are pinned to the stream
        that was current on the thread that armed the exchange (the backward's forward stream:
        under a capture, the capturing stream), not to whatever the hook thread has current."""
        if not self.armed:
            return
        self._left[bi] -= 1
        if self._left[bi] == 0:
            a, b = self.ranges[bi]
            base = self.ex.base
            ctx = torch.cuda.stream(base) if base is not None else _null()
            with ctx:
                torch._foreach_copy_(self.fviews[a:b], [p.grad for p in self.params[a:b]])
            self.ex.launch(f"b{bi}")

    def arm(self) -> None:
        self.armed = True
        self._left = [b - a for a, b in self.ranges]
        if self.flat.is_cuda:
            self.ex.base = torch.cuda.current_stream(self.flat.device)

    def wait(self) -> None:
        """Join; every bucket must have been launched by this backward."""
        if not self.armed:
            return
        if any(self._left):
            raise RuntimeError(f"gradient buckets not complete after backward: {self._left}")
        self.ex.wait()
        self.ex.base = None
        if self.copy_back:
            torch._foreach_copy_([p.grad for p in self.params], self.fviews)
        self.armed = False

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def even_buckets(n: int, k: int) -> List[Tuple[int, int]]:
    """k contiguous runs of n parameters, the last run first in backward order."""
    k = max(1, min(k, n))
    cuts = [round(i * n / k) for i in range(k + 1)]
    return [(cuts[i], cuts[i + 1]) for i in range(k)]


def broadcast_arena(flat: torch.Tensor, src: int = 0, group=None) -> None:
    """Identical start on every rank: rank `src`'s parameters overwrite the others."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)
