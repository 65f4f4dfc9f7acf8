"""YOLOv4 decode + post-processing (K5 → K4), reference ``tools/yolo_layer.py`` /
``tools/utils.py:166-233`` / ``utils/postprocess.py:201-260``."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from ..models.yolov4 import ANCHORS, MASKS, STRIDES
from ._ws import Workspace, dtype_code
from .conv import NHWC
from .image import FrameXform
from .nms import Candidates, NmsResult, SORT_CAP, sort_and_nms


class Yolov4Postprocess:
    """Three NHWC head slices → per-class NMS detections (model pixels, or the
    original frame with an xform), optionally also the served model's full
    ``boxes`` [B, N, 1, 4] / ``confs`` [B, N, nc] tensors."""

    def __init__(self, nc: int = 80, img_hw=(512, 512), conf_thres: float = 0.4, nms_thres: float = 0.6,
                 max_out: int = 1000, scale_x_y: float = 1.0, device="cuda", cap: int = 8192):
        self.nc, self.img_hw = nc, tuple(img_hw)
        self.conf_thres, self.nms_thres, self.max_out, self.sxy = conf_thres, nms_thres, max_out, scale_x_y
        self.device = torch.device(device)
        self.cap = min(cap, SORT_CAP)
        H, W = self.img_hw
        self.grids = [(H // s, W // s) for s in STRIDES]
        self.N = sum(3 * h * w for h, w in self.grids)
        anc = [ANCHORS[2 * m + k] / STRIDES[l] for l, ms in enumerate(MASKS) for m in ms for k in range(2)]
        self._anc = (ctypes.c_float * 18)(*anc)
        self._hw = (ctypes.c_int * 6)(*[v for g in self.grids for v in g])
        self.ws = Workspace(self.device) if self.device.type == "cuda" else None

    def __call__(self, heads: Sequence[NHWC], xform: Optional[FrameXform] = None, full: bool = False,
                 stream=None):
        if heads[0].t.device.type != "cuda":
            return self.cpu([h.nchw()[:, :3 * (5 + self.nc)] for h in heads], xform, full)
        B = heads[0].t.shape[0]
        cand = Candidates.alloc(self.ws, "y4_", B, self.cap, 4)
        ob = oc = None
        if full:
            ob = self.ws.get("y4_boxes", (B, self.N, 1, 4), torch.float32)
            oc = self.ws.get("y4_confs", (B, self.N, self.nc), torch.float32)
        es = heads[0].t.element_size()
        ptrs = [_native.ptr(h.t) + h.off * es for h in heads]
        ldc = (ctypes.c_int * 3)(*[h.t.shape[-1] for h in heads])
        H, W = self.img_hw
        _native.call("tca_yolov4_decode", ptrs[0], ptrs[1], ptrs[2], dtype_code(heads[0].t), B, self.nc, self._hw,
                     ldc, self._anc, float(self.sxy), float(self.conf_thres), H, W, _native.ptr(ob),
                     _native.ptr(oc), _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls),
                     _native.ptr(cand.key), _native.ptr(cand.count), self.cap, _native.stream_ptr(stream))
        res = sort_and_nms(self.ws, cand, 0, self.nms_thres, self.cap, self.max_out, False,
                           xform.as_list() if xform is not None else None, prefix="y4_nms_", stream=stream)
        return (res, ob, oc) if full else res

    def filter_decoded(self, boxes: torch.Tensor, confs: torch.Tensor, xform: Optional[FrameXform] = None,
                       stream=None) -> NmsResult:
        """The served model's decoded outputs (``boxes`` [B, N, 1, 4] normalised x1y1x2y2,
        ``confs`` [B, N, nc]) already on the GPU -> per-class NMS detections on the device
        (the remote client's postprocess, ``tools/utils.py:166-233``); CPU tensors take
        :meth:`decoded_cpu`."""
        if boxes.device.type != "cuda":
            return self.decoded_cpu(boxes.numpy(), confs.numpy(), xform)
        B, N = confs.shape[:2]
        if confs.shape[2] != self.nc or boxes.numel() != B * N * 4:
            raise ValueError(f"boxes {tuple(boxes.shape)} / confs {tuple(confs.shape)} do not match nc={self.nc}")
        boxes, confs = boxes.float().contiguous(), confs.float().contiguous()
        cand = Candidates.alloc(self.ws, "y4d_", B, self.cap, 4)
        H, W = self.img_hw
        _native.call("tca_yolo_filter_decoded", _native.ptr(boxes), _native.ptr(confs), 1, B, N, 4, self.nc,
                     float(self.conf_thres), 0, None, float(W), float(H), _native.ptr(cand.box), _native.ptr(cand.score),
                     _native.ptr(cand.cls), _native.ptr(cand.key), _native.ptr(cand.count), self.cap,
                     _native.stream_ptr(stream))
        return sort_and_nms(self.ws, cand, 0, self.nms_thres, self.cap, self.max_out, False,
                            xform.as_list() if xform is not None else None, prefix="y4d_nms_", stream=stream)

    def decoded_cpu(self, boxes: np.ndarray, confs: np.ndarray, xform=None) -> NmsResult:
        from ..models.yolov4 import post_processing

        B = confs.shape[0]
        return self._pack(post_processing(np.asarray(boxes).reshape(B, -1, 1, 4), np.asarray(confs), self.conf_thres,
                                          self.nms_thres), xform)

    def cpu(self, heads, xform=None, full=False):
        from ..models.yolov4 import decode_reference, post_processing

        boxes, confs = decode_reference(heads, self.nc, self.sxy)
        res = self._pack(post_processing(boxes.numpy(), confs.numpy(), self.conf_thres, self.nms_thres), xform)
        return (res, boxes, confs) if full else res

    def _pack(self, per, xform=None) -> NmsResult:
        B, mo = len(per), self.max_out
        H, W = self.img_hw
        box = np.zeros((B, mo, 4), np.float32)
        score = np.zeros((B, mo), np.float32)
        cls = np.zeros((B, mo), np.int32)
        cnt = np.zeros((B,), np.int32)
        for b, d in enumerate(per):
            d = d[np.argsort(-d[:, 4], kind="stable")][:mo]
            bx = d[:, :4] * np.array([W, H, W, H], np.float32)
            if xform is not None and len(bx):
                bx = xform.unmap_boxes(bx)
            k = len(d)
            box[b, :k], score[b, :k], cls[b, :k], cnt[b] = bx, d[:, 4], d[:, 5], k
        return NmsResult(torch.from_numpy(box), torch.from_numpy(score), torch.from_numpy(cls), torch.from_numpy(cnt))
