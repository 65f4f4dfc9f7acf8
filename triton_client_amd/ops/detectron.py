"""Detectron2 RetinaNet / FCOS postprocess and GroupNorm (``csrc/kernels/detectron.hip``).

GPU chain per step:

1. Per FPN level, a decode kernel writes multi-label candidates into
   (image, level) segments.
2. ``tca_topk_sort`` keeps the top 1000 per segment (Detectron2's
   ``topk_candidates``).
3. ``tca_segment_merge`` concatenates the levels of each image.
4. The class-aware bitmask NMS (K4) keeps 100 and maps the boxes back to the
   original frame.

The CPU path is :func:`triton_client_amd.models.detectron.decode_reference`.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from ..config.detectron import DetectronConfig
from ._ws import Workspace, dtype_code
from .conv import NHWC
from .image import FrameXform
from .nms import Candidates, NmsResult, SORT_CAP, sort_and_nms


def group_norm_nhwc(x: NHWC, gamma: torch.Tensor, beta: torch.Tensor, groups: int = 32, eps: float = 1e-5,
                    relu: bool = True, out: Optional[NHWC] = None, ws: Optional[Workspace] = None,
                    stream=None) -> NHWC:
    """GroupNorm + affine (+ ReLU) over an NHWC slice; ``out`` may be ``x`` (in place)."""
    out = out or x
    B, H, W, C = x.shape
    if x.t.device.type != "cuda":
        y = torch.nn.functional.group_norm(x.nchw().float(), groups, gamma.float().cpu(), beta.float().cpu(), eps)
        if relu:
            y = torch.relu(y)
        out.tensor().copy_(y.permute(0, 2, 3, 1).to(out.t.dtype))
        return out
    ws = ws or Workspace(x.t.device)
    stats = ws.get(f"gn_stats_{B}_{groups}", (B, groups, 2), torch.float32)
    if x.t.dtype != out.t.dtype or x.t.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError(f"group_norm_nhwc: bf16 or fp32 NHWC, got {x.t.dtype} -> {out.t.dtype}")
    _native.call("tca_group_norm_nhwc_dt", _native.ptr(x.t), B, H * W, C, x.t.shape[-1], x.off, groups, float(eps),
                 _native.ptr(gamma), _native.ptr(beta), int(relu), _native.ptr(stats), _native.ptr(out.t),
                 out.t.shape[-1], out.off, dtype_code(x.t), _native.stream_ptr(stream))
    return out


class DetectronPostprocess:
    """Per-level head outputs → NmsResult [B, max_det, 4] (original-frame pixels
    when an xform is given), class ids, scores."""

    def __init__(self, cfg: DetectronConfig, batch: int, device="cuda", seg_cap: int = 32768):
        self.cfg, self.B = cfg, batch
        self.device = torch.device(device)
        self.L = len(cfg.strides)
        self.seg_cap = seg_cap
        self.pre = min(cfg.topk_per_level, SORT_CAP)
        self.merged_cap = min(self.L * self.pre, SORT_CAP)
        self._anchors = []
        if cfg.arch == "retinanet":
            for lvl in range(self.L):
                tab = [v for wh in cfg.anchor_table(lvl) for v in wh]
                self._anchors.append((ctypes.c_float * len(tab))(*tab))
        if self.device.type == "cuda":
            self.ws = Workspace(self.device)

    def __call__(self, outs: Sequence, xform: Optional[FrameXform] = None, stream=None) -> NmsResult:
        """outs[level] = (cls, box) (RetinaNet) or (cls, box, ctr) (FCOS): NHWC slices."""
        cfg = self.cfg
        if outs[0][0].t.device.type != "cuda":
            return self.cpu(outs, xform)
        B, L = self.B, self.L
        cand = Candidates.alloc(self.ws, "dt_seg_", B * L, self.seg_cap, 4)
        s = _native.stream_ptr(stream)
        H_in, W_in = cfg.input_hw
        for lvl, o in enumerate(outs):
            cls, box = o[0], o[1]
            es = cls.t.element_size()
            pc = _native.ptr(cls.t) + cls.off * es
            pb = _native.ptr(box.t) + box.off * es
            _, H, W, _ = cls.shape
            if cfg.arch == "retinanet":
                _native.call("tca_retina_decode", pc, pb, dtype_code(cls.t), B, H, W, cfg.num_anchors, cfg.num_classes,
                             cls.t.shape[-1], box.t.shape[-1], cfg.strides[lvl], self._anchors[lvl],
                             float(cfg.score_thresh), float(cfg.scale_clamp), float(H_in), float(W_in), lvl, L,
                             _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls),
                             _native.ptr(cand.key), _native.ptr(cand.count), self.seg_cap, int(lvl == 0), s)
            else:
                ctr = o[2]
                pt = _native.ptr(ctr.t) + ctr.off * es
                _native.call("tca_fcos_decode", pc, pb, pt, dtype_code(cls.t), B, H, W, cfg.num_classes,
                             cls.t.shape[-1], box.t.shape[-1], ctr.t.shape[-1], cfg.strides[lvl],
                             float(cfg.score_thresh), float(H_in), float(W_in), lvl, L, _native.ptr(cand.box),
                             _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key),
                             _native.ptr(cand.count), self.seg_cap, int(lvl == 0), s)
        order = self.ws.get("dt_seg_order", (B * L, self.pre), torch.int32)
        nsorted = self.ws.get("dt_seg_nsorted", (B * L,), torch.int32)
        _native.call("tca_topk_sort", _native.ptr(cand.key), _native.ptr(cand.count), B * L, self.seg_cap, self.pre,
                     _native.ptr(order), _native.ptr(nsorted), s)
        merged = Candidates.alloc(self.ws, "dt_img_", B, self.merged_cap, 4)
        _native.call("tca_segment_merge", _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls),
                     _native.ptr(cand.key), 4, self.seg_cap, _native.ptr(order), _native.ptr(nsorted), self.pre, B, L,
                     _native.ptr(merged.box), _native.ptr(merged.score), _native.ptr(merged.cls),
                     _native.ptr(merged.key), _native.ptr(merged.count), self.merged_cap, s)
        return sort_and_nms(self.ws, merged, 0, cfg.nms_thresh, self.merged_cap, cfg.max_detections, False,
                            xform.as_list() if xform is not None else None, prefix="dt_nms_", stream=stream)

    def cpu(self, outs, xform: Optional[FrameXform] = None) -> NmsResult:
        from ..models.detectron import decode_reference

        per = decode_reference([tuple(t.nchw().float() for t in o) for o in outs], self.cfg)
        B, md = len(per), self.cfg.max_detections
        box = np.zeros((B, md, 4), np.float32)
        score = np.zeros((B, md), np.float32)
        cls = np.zeros((B, md), np.int32)
        cnt = np.zeros((B,), np.int32)
        for b, (bx, sc, cl) in enumerate(per):
            k = min(len(sc), md)
            if xform is not None and k:
                bx = xform.unmap_boxes(bx)
            box[b, :k], score[b, :k], cls[b, :k], cnt[b] = bx[:k], sc[:k], cl[:k], k
        return NmsResult(torch.from_numpy(box), torch.from_numpy(score), torch.from_numpy(cls), torch.from_numpy(cnt))
