"""YOLOv5 client (reference ``clients/yolov5_client.py``,
``clients/preprocess/yolov5_preprocess.py``, ``clients/postprocess/yolov5_postprocess.py``)."""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops.yolo import YoloPostprocess, detections_nx6
from .base_client import Client
from .postprocess.base_postprocess import Postprocess

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "data")


class Yolov5preprocess:
    """HWC uint8 RGB → [1, 3, H, W] fp32 in [0, 1] (reference :12-24).  Frames
    already resized by the caller; :meth:`image_adjust_device` does resize +
    normalise in one HIP kernel for a whole batch."""

    scaling = "COCO"

    def preprocess(self):
        pass

    def image_adjust(self, cv_image: np.ndarray) -> np.ndarray:
        if cv_image is None:
            return None
        x = np.ascontiguousarray(cv_image.transpose(2, 0, 1)).astype(np.float32)
        x = x[None]
        if self.scaling == "COCO":
            x *= np.float32(1.0 / 255.0)
        return x

    def image_adjust_device(self, frames: torch.Tensor, hw, mode="stretch", dtype=torch.float32, layout="NCHW"):
        from ..ops.image import preprocess
        return preprocess(frames, hw, mode, self.scaling, dtype, layout)


class Yolov5postprocess(Postprocess):
    """``extract_boxes`` of a YOLOv5 response (reference :28-125).  ``device="cpu"``:
    vectorised NumPy + greedy NMS (config 1, the CPU-only client).  A GPU device:
    the response bytes go to the GPU (one pinned H2D per batch of responses) and the
    filter (K3, ``tca_yolo_filter_decoded``) + sort + bitmask NMS (K4) run there —
    the same kept sets (``tests/test_remote_device_gpu.py``)."""

    def __init__(self, device="cpu"):
        self.device = torch.device(device)
        self._pp = {}
        self._up = None
        # the device path's workspaces (candidates, NMS buffers) are reused: one caller at a time,
        # held until its results have been read (RemoteLiveCamera holds it across the annotation)
        self.lock = threading.RLock()

    def load_class_names(self, namesfile: Optional[str] = None) -> List[str]:
        return Postprocess.load_class_names(namesfile or os.path.join(DATA, "coco.names"))

    def _post(self, nc: int, conf_thres, iou_thres, classes, agnostic, multi_label, max_det, device):
        key = (nc, float(conf_thres), float(iou_thres), None if classes is None else tuple(classes), bool(agnostic),
               bool(multi_label), int(max_det), str(device))
        pp = self._pp.get(key)
        if pp is None:
            pp = self._pp[key] = YoloPostprocess(nc, np.zeros((3, 3, 2), np.float32), conf_thres=conf_thres,
                                                 iou_thres=iou_thres, max_det=max_det, agnostic=agnostic,
                                                 multi_label=multi_label, classes=classes, device=device)
        return pp

    @staticmethod
    def _pred(prediction) -> np.ndarray:
        if hasattr(prediction, "raw_output_contents") or hasattr(prediction, "order"):
            pred = Postprocess.output_array(prediction, 0)
        else:
            pred = prediction
        pred = np.asarray(pred, np.float32)
        return pred[None] if pred.ndim == 2 else pred

    def extract_boxes(self, prediction, conf_thres: float = 0.6, iou_thres: float = 0.45, classes=None,
                      agnostic: bool = False, multi_label: bool = False, labels=(), max_det: int = 300):
        """ModelInferResponse (decoded [B, N, 5+nc] output 0) → list of [n, 6]
        arrays (x1, y1, x2, y2, conf, cls) in model-input pixels.  An empty
        list entry means no detections (the reference returned the exception)."""
        pred = self._pred(prediction)
        if self.device.type == "cuda":
            with self.lock:
                res = self.extract_boxes_device([pred], conf_thres, iou_thres, classes=classes, agnostic=agnostic,
                                                multi_label=multi_label, max_det=max_det)
                return detections_nx6(res)
        pp = self._post(pred.shape[2] - 5, conf_thres, iou_thres, classes, agnostic, multi_label, max_det, "cpu")
        return detections_nx6(pp.postprocess_decoded(pred))

    def extract_boxes_device(self, responses: Sequence, conf_thres: float = 0.3, iou_thres: float = 0.45,
                             xform=None, classes=None, agnostic: bool = False, multi_label: bool = False,
                             max_det: int = 300, stream=None):
        """Several responses (one frame each, or decoded arrays) -> one device NmsResult
        [n, max_det]: boxes in original-frame pixels when ``xform`` (the frames' common
        preprocess transform) is given, else model-input pixels."""
        from .postprocess.device import ResponseUpload

        preds = [self._pred(r) for r in responses]
        rows = [p.reshape(-1, p.shape[-1]) for p in preds] if all(p.shape[0] == 1 for p in preds) else \
            [row for p in preds for row in p]
        if self._up is None:
            self._up = ResponseUpload(self.device)
        dev = self._up(rows, np.float32, stream)
        pp = self._post(dev.shape[2] - 5, conf_thres, iou_thres, classes, agnostic, multi_label, max_det, self.device)
        return pp.filter_decoded(dev, xform, stream)


class Yolov5client(Client):
    def __init__(self, device="cpu"):
        super().__init__()
        self.device = device

    def get_preprocess(self):
        return Yolov5preprocess()

    def get_postprocess(self):
        return Yolov5postprocess(self.device)
