"""YOLOv5 postprocess: Detect decode + candidate filter (K3) + top-k/NMS (K4)
+ box rescale to the original frame, as one device-resident chain.

Reference: ``clients/postprocess/yolov5_postprocess.py:28-125`` and the box
rescale at ``communicator/ros_inference.py:100-115``.  Fixes (SURVEY
Appendix A5/A10): an empty result is an empty detection set (the reference
returns the AssertionError object); output dtypes follow the data.

Deviations, documented: candidates beyond 8192 per image are cut to the top
8192 by score before NMS (reference: 30000).  Merge-NMS (``merge=True``; off by
default, as in the reference's ``merge = False``) follows
``yolov5_postprocess.py:111-117``: each kept box becomes the score-weighted mean
of its class's candidates with IoU > iou_thres, and with ``redundant`` (the
reference's default) kept boxes overlapping no other candidate are dropped;
only when 1 < n < 3000 candidates.  GPU: ``tca_nms_merge`` (csrc/kernels/nms.hip).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from ..models.yolov5 import STRIDES
from . import golden
from ._ws import Workspace, dtype_code, layout_of
from .image import FrameXform
from .nms import Candidates, NmsResult, SORT_CAP, sort_and_nms


def _on_gpu(t) -> bool:
    from .conv import NHWC
    if isinstance(t, NHWC):
        t = t.t
    return t.device.type == "cuda"


class YoloPostprocess:
    def __init__(self, nc: int, anchors: torch.Tensor | Sequence, img_hw=(640, 640), conf_thres: float = 0.3,
                 iou_thres: float = 0.45, max_det: int = 300, max_nms: int = 8192, agnostic: bool = False,
                 multi_label: bool = False, classes: Optional[Sequence[int]] = None, device="cuda",
                 merge: bool = False, redundant: bool = True):
        self.nc = nc
        self.merge, self.redundant = merge, redundant
        a = torch.as_tensor(anchors, dtype=torch.float32).reshape(3, -1, 2)
        self.anchors = a.cpu()
        self.na = a.shape[1]
        self.img_hw = tuple(img_hw)
        self.conf_thres, self.iou_thres = conf_thres, iou_thres
        self.max_det, self.max_nms = max_det, min(max_nms, SORT_CAP)
        self.agnostic, self.multi_label = agnostic, multi_label
        self.classes = None if classes is None else list(classes)
        self.device = torch.device(device)
        self.ws = Workspace(self.device) if self.device.type == "cuda" else None
        grids = [(self.img_hw[0] // s, self.img_hw[1] // s) for s in STRIDES]
        self.hw = (ctypes.c_int * 6)(*[v for g in grids for v in g])
        self.strides = (ctypes.c_int * 3)(*STRIDES)
        self.anc = (ctypes.c_float * a.numel())(*a.flatten().tolist())
        self.num_anchors_total = sum(self.na * gh * gw for gh, gw in grids)
        self._class_mask = None
        if self.classes is not None and self.ws is not None:
            words = (nc + 31) // 32
            m = np.zeros(words, np.uint32)
            for c in self.classes:
                m[c >> 5] |= np.uint32(1 << (c & 31))
            self._class_mask = torch.from_numpy(m.view(np.int32)).to(self.device)

    # -------------------------------------------------------------- GPU
    def __call__(self, heads: List[torch.Tensor], xform: Optional[FrameXform] = None, decoded_out: bool = False,
                 stream=None):
        """heads: 3 raw head maps [B, na*(5+nc), H, W] (NCHW or channels_last).
        Returns NmsResult with box [B, max_det, 4] (xyxy, original-frame pixels if
        xform given), score, cls, count — and the decoded [B, N, 5+nc] tensor
        when decoded_out (KServe contract)."""
        if not _on_gpu(heads[0]):
            return self.cpu(heads, xform)
        cand, decoded = self._filter(heads, decoded_out, stream)
        xf = xform.as_list() if xform is not None else None
        res = sort_and_nms(self.ws, cand, 0, self.iou_thres, self.max_nms, self.max_det, self.agnostic,
                           None if self.merge else xf, prefix="yolo_nms_", stream=stream)
        if self.merge:
            res = self._merge(cand, res, xf, stream)
        return (res, decoded) if decoded_out else res

    def detect_fused_ok(self, plan) -> bool:
        """The plan's Detect convs can run fused with this filter (single-label, head width
        na * (5 + nc) <= 256)."""
        return (not self.multi_label and self.na * (self.nc + 5) <= 256 and self.na <= 4
                and self.device.type == "cuda" and plan.detect_fused_ok() and plan.no_real == self.na * (self.nc + 5))

    def detect_fused(self, plan, feats, xform: Optional[FrameXform] = None, stream=None):
        """Detect convs + decode + filter in one kernel (yolo_detect.hip) from the head inputs
        ``feats`` (plan.forward(heads=False)), then sort / NMS as :meth:`__call__`.  The logits
        are bit-identical to the plan's convs, so the candidates are those of the unfused path."""
        B = feats[0].t.shape[0]
        cap = min(self.num_anchors_total, 1 << 20)
        cand = Candidates.alloc(self.ws, "yolo_", B, cap, 4)
        args = getattr(plan, "_detect_args", None)
        if args is None:
            P = ctypes.c_void_p
            args = plan._detect_args = dict(
                x=(P * 3)(*[_native.ptr(o.t) + o.off * o.t.element_size() for o in feats]),
                ldx=(ctypes.c_int * 3)(*[o.t.shape[-1] for o in feats]),
                xoff=(ctypes.c_int * 3)(0, 0, 0),
                cin=(ctypes.c_int * 3)(*[d.cin_p for d in plan.det]),
                w=(P * 3)(*[_native.ptr(d.w_gemm) for d in plan.det]),
                b=(P * 3)(*[_native.ptr(d.b_gemm) for d in plan.det]),
                key=tuple(_native.ptr(o.t) + o.off * o.t.element_size() for o in feats))
        assert args["key"] == tuple(_native.ptr(o.t) + o.off * o.t.element_size() for o in feats)
        _native.call("tca_yolo_detect_filter", ctypes.addressof(args["x"]), args["ldx"], args["xoff"], args["cin"],
                     self.hw, ctypes.addressof(args["w"]), ctypes.addressof(args["b"]), self.strides, self.anc, B,
                     self.na, self.nc, float(self.conf_thres), _native.ptr(self._class_mask), _native.ptr(cand.box),
                     _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key), _native.ptr(cand.count),
                     cap, _native.stream_ptr(stream))
        xf = xform.as_list() if xform is not None else None
        res = sort_and_nms(self.ws, cand, 0, self.iou_thres, self.max_nms, self.max_det, self.agnostic,
                           None if self.merge else xf, prefix="yolo_nms_", stream=stream)
        if self.merge:
            res = self._merge(cand, res, xf, stream)
        return res

    def _merge(self, cand, kept: NmsResult, xf, stream=None) -> NmsResult:
        B, md = kept.score.shape
        out = NmsResult(self.ws.get("yolo_merge_box", (B, md, 4), torch.float32),
                        self.ws.get("yolo_merge_score", (B, md), torch.float32),
                        self.ws.get("yolo_merge_cls", (B, md), torch.int32),
                        self.ws.get("yolo_merge_count", (B,), torch.int32))
        xf_arr = (ctypes.c_float * 6)(*[float(v) for v in xf]) if xf is not None else None
        _native.call("tca_nms_merge", _native.ptr(kept.box), _native.ptr(kept.score), _native.ptr(kept.cls),
                     _native.ptr(kept.count), _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls),
                     _native.ptr(cand.count), B, cand.box.shape[1], md, float(self.iou_thres), int(self.agnostic),
                     int(self.redundant), xf_arr, _native.ptr(out.box), _native.ptr(out.score), _native.ptr(out.cls),
                     _native.ptr(out.count), _native.stream_ptr(stream))
        return out

    def _heads(self, heads):
        """-> (head pointers, NHWC channel strides or None, layout, dtype code, batch)."""
        from .conv import NHWC
        ldc = None
        if isinstance(heads[0], NHWC):  # slices of padded NHWC buffers (fused-conv plan)
            ptrs = [_native.ptr(h.t) + h.off * h.t.element_size() for h in heads]
            ldc = (ctypes.c_int * 3)(*[h.t.shape[-1] for h in heads])
            lay, dt, B = 1, dtype_code(heads[0].t), heads[0].t.shape[0]
        else:
            lay, h0 = layout_of(heads[0])
            hs = [h0] + [layout_of(h)[1] for h in heads[1:]]
            if any(layout_of(h)[0] != lay for h in hs):
                hs = [h.contiguous() for h in hs]
                lay = 0
            ptrs = [_native.ptr(h) for h in hs]
            dt, B = dtype_code(hs[0]), hs[0].shape[0]
        return ptrs, ldc, lay, dt, B

    def _filter(self, heads, decoded_out: bool, stream=None):
        ptrs, ldc, lay, dt, B = self._heads(heads)
        cap = self.num_anchors_total * (self.nc if self.multi_label else 1)
        cap = min(cap, 1 << 20)
        cand = Candidates.alloc(self.ws, "yolo_", B, cap, 4)
        decoded = None
        if decoded_out:
            decoded = self.ws.get("decoded", (B, self.num_anchors_total, self.nc + 5), torch.float32)
        _native.call("tca_yolo_decode_filter", ptrs[0], ptrs[1], ptrs[2],
                     dt, lay, B, self.na, self.nc, self.hw, self.strides, ldc, self.anc,
                     float(self.conf_thres), int(self.multi_label), _native.ptr(self._class_mask),
                     _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key),
                     _native.ptr(cand.count), cap, _native.ptr(decoded), _native.stream_ptr(stream))
        return cand, decoded

    def filter_decoded(self, pred: torch.Tensor, xform: Optional[FrameXform] = None, stream=None) -> NmsResult:
        """K3 + K4 on a *decoded* prediction already on the GPU: pred [B, N, >=5+nc] fp32
        (a KServe YOLOv5 response uploaded by the remote client) -> NmsResult on the
        device, boxes in original-frame pixels if ``xform`` is given, else model pixels.
        Same kept sets as :meth:`postprocess_decoded` (the CPU path of ``--device cpu``)."""
        if pred.device.type != "cuda":
            return self.postprocess_decoded(pred.numpy(), xform)
        if pred.dim() != 3 or pred.dtype != torch.float32 or pred.stride(2) != 1 or pred.shape[2] < self.nc + 5:
            raise ValueError(f"pred must be fp32 [B, N, >= {self.nc + 5}] with unit inner stride, "
                             f"got {tuple(pred.shape)} {pred.dtype}")
        pred = pred if pred.stride(1) == pred.shape[2] and pred.stride(0) == pred.shape[1] * pred.shape[2] \
            else pred.contiguous()
        B, N, ld = pred.shape
        cap = min(N * (self.nc if self.multi_label else 1), 1 << 20)
        cand = Candidates.alloc(self.ws, "yolod_", B, cap, 4)
        _native.call("tca_yolo_filter_decoded", _native.ptr(pred), None, 0, B, N, ld, self.nc, float(self.conf_thres),
                     int(self.multi_label), _native.ptr(self._class_mask), 0.0, 0.0, _native.ptr(cand.box),
                     _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key), _native.ptr(cand.count),
                     cap, _native.stream_ptr(stream))
        xf = xform.as_list() if xform is not None else None
        res = sort_and_nms(self.ws, cand, 0, self.iou_thres, self.max_nms, self.max_det, self.agnostic,
                           None if self.merge else xf, prefix="yolod_nms_", stream=stream)
        if self.merge:
            res = self._merge(cand, res, xf, stream)
        return res

    def decode(self, heads: List[torch.Tensor], stream=None) -> torch.Tensor:
        """Decoded [B, N, 5+nc] fp32 (the ONNX YOLOv5 output contract)."""
        if not _on_gpu(heads[0]):
            return self.decode_cpu(heads)
        ptrs, ldc, lay, dt, B = self._heads(heads)
        decoded = self.ws.get("decoded", (B, self.num_anchors_total, self.nc + 5), torch.float32)
        _native.call("tca_yolo_decode", ptrs[0], ptrs[1], ptrs[2], dt, lay, B, self.na, self.nc, self.hw, self.strides,
                     ldc, self.anc, _native.ptr(decoded), _native.stream_ptr(stream))
        return decoded

    # -------------------------------------------------------------- CPU
    def decode_cpu(self, heads: List[torch.Tensor]) -> torch.Tensor:
        from ..models.yolov5 import yolo_decode_reference
        from .conv import NHWC
        C = self.na * (self.nc + 5)
        hs = [h.nchw()[:, :C] if isinstance(h, NHWC) else h for h in heads]
        return yolo_decode_reference([h.float().contiguous() for h in hs], self.anchors)

    def cpu(self, heads, xform: Optional[FrameXform] = None) -> NmsResult:
        return self.postprocess_decoded(self.decode_cpu(heads).numpy(), xform)

    def postprocess_decoded(self, pred: np.ndarray, xform: Optional[FrameXform] = None) -> NmsResult:
        """Reference-semantics postprocess of a decoded [B, N, 5+nc] array (what
        a KServe YOLOv5 returns).  Vectorised NumPy, class-aware greedy NMS."""
        B, N, no = pred.shape
        nc = no - 5
        outs = []
        for b in range(B):
            x = pred[b]
            idx = np.nonzero(x[:, 4] > self.conf_thres)[0]
            x = x[idx]
            if self.classes is not None:
                allowed = np.zeros(nc, bool)
                allowed[self.classes] = True
            cls_conf = x[:, 5:] * x[:, 4:5]
            box = np.stack([x[:, 0] - x[:, 2] / 2, x[:, 1] - x[:, 3] / 2, x[:, 0] + x[:, 2] / 2,
                            x[:, 1] + x[:, 3] / 2], 1).astype(np.float32)
            if self.multi_label:
                ii, jj = np.nonzero(cls_conf > self.conf_thres)
                if self.classes is not None:
                    keep = allowed[jj]
                    ii, jj = ii[keep], jj[keep]
                bx, sc, cl, tie = box[ii], cls_conf[ii, jj].astype(np.float32), jj, idx[ii] * nc + jj
            else:
                # best over all classes, then the class filter (yolov5_postprocess.py:87-92)
                j = cls_conf.argmax(1) if len(cls_conf) else np.zeros((0,), np.int64)
                conf = cls_conf[np.arange(len(j)), j].astype(np.float32)
                sel = conf > self.conf_thres
                if self.classes is not None:
                    sel &= allowed[j]
                bx, sc, cl, tie = box[sel], conf[sel], j[sel], idx[sel]
            from .nms import sort_and_nms_cpu
            keep = sort_and_nms_cpu(bx, sc, cl.astype(np.int32), tie, 0, self.iou_thres, self.max_nms,
                                    self.max_det, self.agnostic)
            kb = bx[keep]
            if self.merge and 1 < len(sc) < 3000 and len(keep):
                kb, keep = merge_nms(bx, sc, cl, keep, self.iou_thres, self.agnostic, self.redundant)
            if xform is not None:
                kb = xform.unmap_boxes(kb)
            outs.append((kb, sc[keep], cl[keep].astype(np.int32)))
        md = self.max_det
        box = np.zeros((B, md, 4), np.float32)
        score = np.zeros((B, md), np.float32)
        cls = np.zeros((B, md), np.int32)
        count = np.zeros((B,), np.int32)
        for b, (kb, ks, kc) in enumerate(outs):
            n = len(ks)
            box[b, :n], score[b, :n], cls[b, :n], count[b] = kb, ks, kc, n
        return NmsResult(torch.from_numpy(box), torch.from_numpy(score), torch.from_numpy(cls), torch.from_numpy(count))


def merge_nms(box: np.ndarray, score: np.ndarray, cls: np.ndarray, keep: np.ndarray, iou_thr: float,
              agnostic: bool = False, redundant: bool = True):
    """Merge-NMS of one image (reference yolov5_postprocess.py:111-117): kept
    box i -> sum_j w_ij box_j / sum_j w_ij with w_ij = score_j [IoU(i, j) > thr,
    same class unless agnostic] over all candidates j; with ``redundant`` a kept
    box with no other such candidate is dropped.  Returns (merged boxes, keep)."""
    iou = golden.box_iou_np(box[keep].astype(np.float64), box.astype(np.float64)) > iou_thr
    if not agnostic:
        iou &= cls[keep][:, None] == cls[None, :]
    w = iou * score[None, :].astype(np.float64)
    merged = (w @ box.astype(np.float64)) / w.sum(1, keepdims=True)
    if redundant:
        r = iou.sum(1) > 1
        return merged[r].astype(np.float32), keep[r]
    return merged.astype(np.float32), keep


def detections_nx6(res: NmsResult) -> List[np.ndarray]:
    """Reference output format: per image [n, 6] = x1, y1, x2, y2, conf, cls."""
    out = []
    for d in res.per_image():
        out.append(np.concatenate([d["box"], d["score"][:, None], d["cls"][:, None].astype(np.float32)], 1))
    return out
