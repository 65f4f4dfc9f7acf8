"""YOLOv4 client (reference ``examples/YOLOv4/config.pbtxt`` model; decode in
``tools/yolo_layer.py``, post-processing ``tools/utils.py:166-233`` and the
(broken) legacy ``utils/postprocess.py:201-260`` ``extract_boxes_triton``,
re-implemented here per SURVEY Appendix A13)."""
from __future__ import annotations

import os
import threading
from typing import List, Optional

import numpy as np
import torch

from .base_client import Client
from .postprocess.base_postprocess import Postprocess
from .yolov5_client import DATA, Yolov5preprocess


class Yolov4preprocess(Yolov5preprocess):
    scaling = "COCO"  # RGB / 255, NCHW (tools/torch_utils.py:do_detect)


class Yolov4postprocess(Postprocess):
    def __init__(self, input_hw=(512, 512), device="cpu"):
        self.input_hw = tuple(input_hw)
        self.device = torch.device(device)
        self._pp, self._up = {}, None
        self.lock = threading.RLock()  # the device path's workspaces: one caller at a time

    def load_class_names(self, namesfile: Optional[str] = None) -> List[str]:
        return Postprocess.load_class_names(namesfile or os.path.join(DATA, "coco.names"))

    def extract_boxes(self, prediction, conf_thres: float = 0.4, iou_thres: float = 0.6):
        """Response with ``confs`` [1, N, nc] and ``boxes`` [1, N, 1, 4] (normalised)
        → list (per image) of [n, 6] x1, y1, x2, y2 (model-input pixels), conf, cls."""
        from ..models.yolov4 import post_processing

        names = self.output_names(prediction)
        ci = names.index("confs") if "confs" in names else 0
        bi = names.index("boxes") if "boxes" in names else 1
        confs = np.asarray(self.output_array(prediction, ci), np.float32)
        boxes = np.asarray(self.output_array(prediction, bi), np.float32)
        per = post_processing(boxes.reshape(boxes.shape[0], -1, 1, 4), confs, conf_thres, iou_thres)
        H, W = self.input_hw
        out = []
        for d in per:
            d = d.copy()
            d[:, :4] *= np.array([W, H, W, H], np.float32)
            out.append(d)
        return out

    def extract_boxes_device(self, responses, conf_thres: float = 0.4, iou_thres: float = 0.6, xform=None,
                             stream=None, **_):
        """Several responses -> one device NmsResult: ``boxes`` / ``confs`` of every
        response uploaded by one pinned H2D each, then the filter (K3,
        ``tca_yolo_filter_decoded`` kind 1) and per-class NMS (K4) on the GPU."""
        from ..ops.yolov4 import Yolov4Postprocess
        from .postprocess.device import ResponseUpload

        names = self.output_names(responses[0])
        ci = names.index("confs") if "confs" in names else 0
        bi = names.index("boxes") if "boxes" in names else 1
        confs = [np.asarray(self.output_array(r, ci), np.float32) for r in responses]
        boxes = [np.asarray(self.output_array(r, bi), np.float32) for r in responses]
        nc = confs[0].shape[-1]
        confs = [c.reshape(-1, nc) for c in confs]
        boxes = [b.reshape(-1, 4) for b in boxes]
        if self._up is None:
            self._up = (ResponseUpload(self.device), ResponseUpload(self.device))
        dc, db = self._up[0](confs, np.float32, stream), self._up[1](boxes, np.float32, stream)
        key = (nc, float(conf_thres), float(iou_thres))
        pp = self._pp.get(key)
        if pp is None:
            pp = self._pp[key] = Yolov4Postprocess(nc, self.input_hw, conf_thres, iou_thres, device=self.device)
        return pp.filter_decoded(db, dc, xform, stream)


class Yolov4client(Client):
    def __init__(self, device="cpu"):
        super().__init__()
        self.input_hw = (512, 512)
        self.device = device

    def parse_model(self, model_metadata, model_config):
        r = super().parse_model(model_metadata, model_config)
        self.input_hw = (r[3], r[4])
        return r

    def get_preprocess(self):
        return Yolov4preprocess()

    def get_postprocess(self):
        return Yolov4postprocess(self.input_hw, self.device)
