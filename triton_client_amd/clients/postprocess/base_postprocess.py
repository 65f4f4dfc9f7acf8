"""Postprocess base helpers (reference ``clients/postprocess/base_postprocess.py:11-111``).

The reference decodes response tensors with a per-element
``struct.unpack_from`` loop into object arrays (501 ms for a YOLOv5-640
output).  Here decoding is a zero-copy ``np.frombuffer`` typed by
the response's declared datatype (fixes Appendix A10: ``'l'`` vs ``'i'``).
"""
from __future__ import annotations

from abc import ABC
from typing import List, Optional

import numpy as np
import torch

from ...ops import golden

_DT = {"FP32": np.float32, "FP16": np.float16, "FP64": np.float64, "INT32": np.int32, "INT64": np.int64,
       "INT16": np.int16, "INT8": np.int8, "UINT8": np.uint8, "BOOL": np.bool_}


class Postprocess(ABC):
    def postprocess(self):
        pass

    @staticmethod
    def load_class_names(namesfile: str) -> List[str]:
        with open(namesfile) as fp:
            return [ln.rstrip() for ln in fp.read().splitlines() if ln.strip()]

    @staticmethod
    def output_names(response) -> List[str]:
        if hasattr(response, "order"):  # channel.wire.ParsedResponse
            return list(response.order)
        return [t.name for t in response.outputs]

    @staticmethod
    def output_array(response, i) -> np.ndarray:
        """Output i (index or name) of a ModelInferResponse — or of the C++
        codec's ParsedResponse — as a typed, shaped array (no copy)."""
        if hasattr(response, "order"):
            return response[i]
        if isinstance(i, str):
            i = [t.name for t in response.outputs].index(i)
        t = response.outputs[i]
        dt = _DT.get(t.datatype, np.float32)
        return np.frombuffer(response.raw_output_contents[i], dtype=dt).reshape(tuple(t.shape))

    @staticmethod
    def deserialize_bytes_float(encoded: bytes) -> np.ndarray:
        return np.frombuffer(encoded, dtype=np.float32)

    @staticmethod
    def deserialize_bytes_int(encoded: bytes, dtype=np.int64) -> np.ndarray:
        return np.frombuffer(encoded, dtype=dtype)

    @staticmethod
    def xywh2xyxy(x):
        y = x.clone() if isinstance(x, torch.Tensor) else np.copy(x)
        y[:, 0] = x[:, 0] - x[:, 2] / 2
        y[:, 1] = x[:, 1] - x[:, 3] / 2
        y[:, 2] = x[:, 0] + x[:, 2] / 2
        y[:, 3] = x[:, 1] + x[:, 3] / 2
        return y

    @staticmethod
    def box_iou(box1, box2):
        """IoU matrix [N, M] of xyxy boxes (torch or numpy)."""
        if isinstance(box1, torch.Tensor):
            a, b = box1.float(), box2.float()
            area1 = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
            area2 = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
            lt = torch.max(a[:, None, :2], b[:, :2])
            rb = torch.min(a[:, None, 2:], b[:, 2:])
            inter = (rb - lt).clamp(min=0).prod(2)
            return inter / (area1[:, None] + area2 - inter)
        return golden.box_iou_np(np.asarray(box1, np.float64), np.asarray(box2, np.float64))

    @staticmethod
    def nms_cpu(boxes, confs, nms_thresh: float = 0.5, min_mode: bool = False) -> np.ndarray:
        """Greedy NMS; ``min_mode`` uses intersection / min(area) (reference :72-106)."""
        boxes = np.asarray(boxes, np.float64)
        order = np.argsort(-np.asarray(confs), kind="stable")
        x1, y1, x2, y2 = boxes.T
        areas = (x2 - x1) * (y2 - y1)
        keep = []
        while order.size > 0:
            i = order[0]
            keep.append(i)
            xx1 = np.maximum(x1[i], x1[order[1:]])
            yy1 = np.maximum(y1[i], y1[order[1:]])
            xx2 = np.minimum(x2[i], x2[order[1:]])
            yy2 = np.minimum(y2[i], y2[order[1:]])
            inter = np.maximum(0.0, xx2 - xx1) * np.maximum(0.0, yy2 - yy1)
            if min_mode:
                over = inter / np.minimum(areas[i], areas[order[1:]])
            else:
                over = inter / (areas[i] + areas[order[1:]] - inter)
            order = order[1:][over <= nms_thresh]
        return np.asarray(keep, np.int64)
