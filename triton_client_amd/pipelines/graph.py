"""hipGraph capture of a whole pipeline step.

The per-frame work is dozens of short kernels (preprocess, ~60 convs,
decode, sort, NMS...).  Eager launch costs ≈3-4 µs of host time per kernel
(MI355X_MICROARCH.md price list, row graph-replay-floor), so a step is
captured once and replayed: static input buffers are written (H2D copy or
RCCL receive) before ``replay()``, outputs are read from static buffers
after it.  Every op in this package is capture-safe by construction (no
allocation, no host sync, device-side counts).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphRunner:
    def __init__(self, fn: Callable[[], object], warmup: int = 3, enabled: bool = True,
                 pool=None, capture_error_mode: str = "global"):
        self.fn = fn
        self.enabled = enabled and torch.cuda.is_available()
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.warmup = warmup
        self.pool = pool
        # "thread_local": other host threads may keep issuing HIP calls (event
        # waits, pinned allocations) while this thread captures (live drivers)
        self.capture_error_mode = capture_error_mode

    def capture(self) -> None:
        if not self.enabled:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.out = self.fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool, capture_error_mode=self.capture_error_mode):
            self.out = self.fn()
        self.graph = g

    def __call__(self):
        if self.graph is None:
            if self.enabled:
                self.capture()
            else:
                self.out = self.fn()
                return self.out
        self.graph.replay()
        return self.out
