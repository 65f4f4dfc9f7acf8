"""YOLOv5 client (reference ``clients/yolov5_client.py``,
``clients/preprocess/yolov5_preprocess.py``, ``clients/postprocess/yolov5_postprocess.py``)."""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops.yolo import YoloPostprocess
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
    def load_class_names(self, namesfile: Optional[str] = None) -> List[str]:
        return Postprocess.load_class_names(namesfile or os.path.join(DATA, "coco.names"))

    def extract_boxes(self, prediction, conf_thres: float = 0.6, iou_thres: float = 0.45, classes=None,
                      agnostic: bool = False, multi_label: bool = False, labels=(), max_det: int = 300):
        """ModelInferResponse (decoded [B, N, 5+nc] output 0) → list of [n, 6]
        arrays (x1, y1, x2, y2, conf, cls) in model-input pixels.  An empty
        list entry means no detections (the reference returned the exception)."""
        if hasattr(prediction, "raw_output_contents") or hasattr(prediction, "order"):
            pred = self.output_array(prediction, 0)
        else:
            pred = prediction
        pred = np.asarray(pred, np.float32)
        if pred.ndim == 2:
            pred = pred[None]
        pp = YoloPostprocess(pred.shape[2] - 5, np.zeros((3, 3, 2), np.float32), conf_thres=conf_thres,
                             iou_thres=iou_thres, max_det=max_det, agnostic=agnostic, multi_label=multi_label,
                             classes=classes, device="cpu")
        res = pp.postprocess_decoded(pred)
        out = []
        for d in res.per_image():
            out.append(np.concatenate([d["box"], d["score"][:, None], d["cls"][:, None].astype(np.float32)], 1))
        return out


class Yolov5client(Client):
    def get_preprocess(self):
        return Yolov5preprocess()

    def get_postprocess(self):
        return Yolov5postprocess()
