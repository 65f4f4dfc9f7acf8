"""Sub-batched, multi-stream execution of the per-frame pipelines.

A step of B frames can run as S sub-pipelines of B/S frames each, every one
captured as its own hipGraph and replayed on its own stream (one HW queue
each; ``GPU_MAX_HW_QUEUES`` is 4).  The sub-pipelines share one model and
one set of input buffers (views of a [B, ...] parent), so ingest is
unchanged.  What it buys: each pipeline has low-occupancy phases (point
cloud unpack, voxeliser scans, top-k, the single-wave NMS reduce) that leave
most of the 256 CUs idle; with several independent graphs in flight those
phases overlap another graph's convolutions instead of sitting on the
critical path.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch

from .graph import GraphRunner


class SubBatched:
    """``make(batch, model)`` builds one pipeline (``model=None`` → a fresh
    one).  Sub-pipeline 0 owns the model; the others share it, so calibrating
    sub-pipeline 0 (before the first step builds the fused plans) calibrates
    all of them."""

    def __init__(self, make: Callable[[int, Optional[torch.nn.Module]], object], batch: int, splits: int):
        if splits < 1 or batch % splits:
            raise ValueError(f"batch {batch} must split evenly into {splits}")
        bs = batch // splits
        p0 = make(bs, None)
        self.pipes = [p0] + [make(bs, p0.model) for _ in range(splits - 1)]
        self.B, self.splits, self.model = batch, splits, p0.model
        dev = p0.device
        if hasattr(p0, "frames"):  # camera: [B, H, W, 3] uint8
            self.frames = torch.zeros((batch, *p0.frames.shape[1:]), dtype=p0.frames.dtype, device=dev)
            for s, p in enumerate(self.pipes):
                p.frames = self.frames[s * bs:(s + 1) * bs]
        if hasattr(p0, "data"):  # LiDAR: B payload slots + point counts
            self.frame_bytes = fb = p0.frame_bytes
            self.data = torch.zeros(batch * fb, dtype=torch.uint8, device=dev)
            self.frame_n = torch.zeros(batch, dtype=torch.int32, device=dev)
            for s, p in enumerate(self.pipes):
                p.data = self.data[s * bs * fb:(s + 1) * bs * fb]
                p.frame_n = self.frame_n[s * bs:(s + 1) * bs]

    @property
    def device(self):
        return self.pipes[0].device

    def calibrate_detection_density(self, *args, **kw):
        return self.pipes[0].calibrate_detection_density(*args, **kw)


class MultiStreamRunner:
    """Replays one step function per stream: fns[0] on the current stream, the
    rest on their own streams forked from / joined back to it.  Launch order
    follows ``fns`` (put the critical path first)."""

    def __init__(self, fns: Sequence[Callable[[], object]], enabled: bool = True):
        self.runners = [GraphRunner(f, enabled=enabled) for f in fns]
        self.streams: List[Optional[torch.cuda.Stream]] = [None] + [torch.cuda.Stream() for _ in fns[1:]]

    def __call__(self) -> list:
        main = torch.cuda.current_stream()
        for s in self.streams[1:]:  # fork every branch before any replay is enqueued on main
            s.wait_stream(main)
        outs: list = [None] * len(self.runners)
        for i, (r, s) in enumerate(zip(self.runners, self.streams)):
            if s is None:
                outs[i] = r()
                continue
            with torch.cuda.stream(s):
                outs[i] = r()
        for s in self.streams[1:]:
            main.wait_stream(s)
        return outs
