"""K4 / K10 — top-k + sort + bitmask NMS over per-image candidate buffers.

GPU: ``csrc/kernels/nms.hip`` (three launches, static shapes, device-side
counts).  CPU: the same semantics through :func:`golden.nms_greedy`.

Candidate buffer contract (produced by the YOLO / anchor decode kernels):
``box [B, cap, D]`` fp32, ``score [B, cap]``, ``cls [B, cap]`` int32,
``key [B, cap]`` uint64 (score-major, ~index-minor), ``count [B]`` int32.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from . import golden
from ._ws import Workspace

SORT_CAP = 8192  # must match kSortCap in nms.hip


@dataclass
class Candidates:
    box: torch.Tensor    # [B, cap, D]
    score: torch.Tensor  # [B, cap]
    cls: torch.Tensor    # [B, cap] int32
    key: torch.Tensor    # [B, cap] int64 (bit pattern of the uint64 key)
    count: torch.Tensor  # [B] int32

    @staticmethod
    def alloc(ws: Workspace, prefix: str, batch: int, cap: int, dim: int) -> "Candidates":
        return Candidates(ws.get(prefix + "box", (batch, cap, dim), torch.float32),
                          ws.get(prefix + "score", (batch, cap), torch.float32),
                          ws.get(prefix + "cls", (batch, cap), torch.int32),
                          ws.get(prefix + "key", (batch, cap), torch.int64),
                          ws.get(prefix + "count", (batch,), torch.int32))


@dataclass
class NmsResult:
    box: torch.Tensor    # [B, max_out, D]
    score: torch.Tensor  # [B, max_out]
    cls: torch.Tensor    # [B, max_out] int32
    count: torch.Tensor  # [B]

    def per_image(self) -> List[dict]:
        cnt = self.count.cpu().numpy()
        box, score, cls = self.box.cpu().numpy(), self.score.cpu().numpy(), self.cls.cpu().numpy()
        return [dict(box=box[b, :cnt[b]], score=score[b, :cnt[b]], cls=cls[b, :cnt[b]]) for b in range(len(cnt))]


def sort_and_nms(ws: Workspace, cand: Candidates, mode: int, iou_thr: float, pre_max: int, max_out: int,
                 agnostic: bool, xform: Optional[Sequence[float]] = None, prefix: str = "nms_",
                 stream=None) -> NmsResult:
    """mode 0: axis-aligned xyxy (class-aware unless agnostic); 1: rotated BEV (box dim >= 7)."""
    B, cap, D = cand.box.shape
    pre_max = min(pre_max, SORT_CAP, cap)
    words = (pre_max + 63) // 64
    order = ws.get(prefix + "order", (B, pre_max), torch.int32)
    nsorted = ws.get(prefix + "nsorted", (B,), torch.int32)
    mask = ws.get(prefix + "mask", (B, pre_max, words), torch.int64)
    res = NmsResult(ws.get(prefix + "out_box", (B, max_out, D), torch.float32),
                    ws.get(prefix + "out_score", (B, max_out), torch.float32),
                    ws.get(prefix + "out_cls", (B, max_out), torch.int32),
                    ws.get(prefix + "out_count", (B,), torch.int32))
    s = _native.stream_ptr(stream)
    _native.call("tca_topk_sort", _native.ptr(cand.key), _native.ptr(cand.count), B, cap, pre_max,
                 _native.ptr(order), _native.ptr(nsorted), s)
    if mode == 1:
        soa = ws.get(prefix + "soa", (B, 9, (pre_max + 3) // 4 * 4), torch.float32)
        _native.call("tca_nms_mask_rot", _native.ptr(cand.box), D, _native.ptr(cand.cls), _native.ptr(order),
                     _native.ptr(nsorted), B, cap, pre_max, float(iou_thr), int(agnostic), _native.ptr(soa),
                     _native.ptr(mask), s)
    else:
        _native.call("tca_nms_mask", mode, _native.ptr(cand.box), D, _native.ptr(cand.cls), _native.ptr(order),
                     _native.ptr(nsorted), B, cap, pre_max, float(iou_thr), int(agnostic), _native.ptr(mask), 0, s)
    xf_arr = None
    if xform is not None:
        import ctypes
        xf_arr = (ctypes.c_float * 6)(*[float(v) for v in xform])
    _native.call("tca_nms_reduce", _native.ptr(order), _native.ptr(nsorted), _native.ptr(mask), B, pre_max,
                 _native.ptr(cand.box), D, _native.ptr(cand.score), _native.ptr(cand.cls), cap, max_out,
                 xf_arr, _native.ptr(res.box), _native.ptr(res.score), _native.ptr(res.cls),
                 _native.ptr(res.count), s)
    return res


def sort_and_nms_cpu(box: np.ndarray, score: np.ndarray, cls: np.ndarray, tie: np.ndarray, mode: int,
                     iou_thr: float, pre_max: int, max_out: int, agnostic: bool):
    """One image on the CPU; same ordering/tie rules as the GPU path.
    Returns kept indices into the inputs (score order)."""
    n = len(score)
    if n == 0:
        return np.zeros((0,), np.int64)
    order = np.lexsort((tie, -score.astype(np.float64)))[:min(pre_max, SORT_CAP)]
    b, s, c, t = box[order], score[order], cls[order], tie[order]
    if mode == 0:
        iou_fn = None
    else:
        iou_fn = lambda a, bs: golden.rotated_iou_bev(a, bs)  # noqa: E731
    keep = golden.nms_greedy(b, s, iou_thr, None if agnostic else c, order_key=t, iou_fn=iou_fn, max_out=max_out)
    return order[np.asarray(keep, np.int64)]
