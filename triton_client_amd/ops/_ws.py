"""Persistent device workspaces.

Every GPU op owns its scratch through a :class:`Workspace`: buffers are
allocated once per (name, shape, dtype) and reused, so a captured hipGraph
sees stable addresses and no allocation ever happens on the hot path
(cdna_hip_programming.md Guideline 9).  Buffers that must start in a given
state (the voxeliser's self-resetting grids) take an ``init`` value that is
applied only at allocation time.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import torch


class Workspace:
    def __init__(self, device: torch.device | str):
        self.device = torch.device(device)
        self._bufs: Dict[str, torch.Tensor] = {}

    def get(self, name: str, shape: Sequence[int], dtype: torch.dtype, init: Optional[float] = None) -> torch.Tensor:
        shape = tuple(int(s) for s in shape)
        t = self._bufs.get(name)
        if t is None or t.shape != shape or t.dtype != dtype:
            if init is None:
                t = torch.empty(shape, dtype=dtype, device=self.device)
            else:
                t = torch.full(shape, init, dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self._bufs.values())


DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.uint8: 3, torch.int32: 4}


def dtype_code(t: torch.Tensor) -> int:
    try:
        return DTYPE_CODE[t.dtype]
    except KeyError as e:
        raise TypeError(f"unsupported dtype {t.dtype}") from e


def is_nhwc(t: torch.Tensor) -> bool:
    """True if a 4-D tensor is channels_last-contiguous (and not also NCHW-contiguous
    in a way that makes the distinction moot)."""
    if t.dim() != 4:
        return False
    if t.is_contiguous():
        return False
    return t.is_contiguous(memory_format=torch.channels_last)


def layout_of(t: torch.Tensor) -> Tuple[int, torch.Tensor]:
    """(layout code, tensor in that layout): 0 NCHW, 1 NHWC."""
    if t.is_contiguous():
        return 0, t
    if t.is_contiguous(memory_format=torch.channels_last):
        return 1, t
    return 0, t.contiguous()
