"""Recorded C-ABI programs.

A `Ctx` is the launch context the network builders (net.py) talk to.  In *eager* mode
each C-ABI call runs immediately on the current HIP stream; in *record* mode the calls
are appended to a program (with every tensor they touch kept alive) that `run()` replays
on any stream -- which is what makes a whole forward/backward capturable in one hipGraph.
Buffers come from the PyTorch HIP caching allocator (the library allocates nothing).
"""
from __future__ import annotations

import ctypes
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import lib as L


def current_stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


class Ctx:
    def __init__(self, dtype: torch.dtype, device, record: bool = False, shared: Optional[dict] = None):
        self.tdtype = dtype
        self.code = L.dtype_code(dtype)
        self.device = torch.device(device)
        self.record = record
        self.ops: List[Tuple[str, Callable, tuple]] = []
        self._scratch: Dict[str, torch.Tensor] = {}
        self._hold: List[torch.Tensor] = []   # replaced scratch buffers still referenced by ops
        self.lib = L.load()
        # long-lived state shared by short-lived eager contexts
        self._shared = {} if shared is None else shared

    # ---- memory ----
    def alloc(self, shape, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        t = torch.empty(tuple(shape), dtype=dtype or self.tdtype, device=self.device)
        if self.record:   # a recorded program owns every buffer its launches touch
            self._hold.append(t)
        return t

    def zeros(self, shape, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        return torch.zeros(tuple(shape), dtype=dtype or self.tdtype, device=self.device)

    def scratch(self, tag: str, shape, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """A buffer re-used across layers in record mode (tags encode lifetimes)."""
        dtype = dtype or self.tdtype
        n = 1
        for s in shape:
            n *= int(s)
        if not self.record:
            return self.alloc(shape, dtype)
        key = f"{tag}/{dtype}"
        buf = self._scratch.get(key)
        if buf is None or buf.numel() < n:
            if buf is not None:
                self._hold.append(buf)
            buf = torch.empty(n, dtype=dtype, device=self.device)
            self._scratch[key] = buf
        return buf[:n].view(tuple(shape))

    def zero_scratch(self, tag: str, shape, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """A persistent zero-initialised buffer (e.g. self-cleaning sync words), one per tag."""
        dtype = dtype or self.tdtype
        key = f"zero:{tag}/{dtype}"
        buf = self._scratch.get(key)
        n = 1
        for s in shape:
            n *= int(s)
        if buf is None or buf.numel() < n:
            if buf is not None:
                self._hold.append(buf)
            buf = torch.zeros(n, dtype=dtype, device=self.device)
            self._scratch[key] = buf
        return buf[:n].view(tuple(shape))

    def persistent_zeros(self, tag: str, nbytes: int) -> torch.Tensor:
        """A zero-initialised byte buffer that outlives this context (kept in the shared state of
        the eager contexts, or in the program): self-resetting sync workspaces."""
        key = f"pz:{tag}"
        buf = self._shared.get(key)
        if buf is None or buf.numel() < nbytes:
            if buf is not None:
                self._hold.append(buf)
            buf = torch.zeros(int(nbytes), dtype=torch.uint8, device=self.device)
            self._shared[key] = buf
        return buf

    def keep(self, obj) -> None:
        """Keep a host object (e.g. a ctypes job table) alive as long as the program."""
        self._hold.append(obj)

    # ---- launches ----
    def emit(self, name: str, fn: Callable, *args) -> None:
        if self.record:
            self.ops.append((name, fn, args))
        else:
            L.check(fn(*args, current_stream_handle()), name)

    def mark(self, name: str, callback: Callable[[], None]) -> None:
        """A host-side hook inside a program (e.g. issue a bucket all-reduce)."""
        if self.record:
            self.ops.append((name, None, (callback,)))
        else:
            callback()

    def run(self, stream: Optional[int] = None) -> None:
        s = current_stream_handle() if stream is None else stream
        for name, fn, args in self.ops:
            if fn is None:
                args[0]()
                continue
            code = fn(*args, s)
            if code:
                L.check(code, name)

    def __len__(self):
        return len(self.ops)


def ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def byref(desc):
    return ctypes.byref(desc)
