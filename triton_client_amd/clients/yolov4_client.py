"""YOLOv4 client (reference ``examples/YOLOv4/config.pbtxt`` model; decode in
``tools/yolo_layer.py``, post-processing ``tools/utils.py:166-233`` and the
(broken) legacy ``utils/postprocess.py:201-260`` ``extract_boxes_triton``,
re-implemented here per SURVEY Appendix A13)."""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

from .base_client import Client
from .postprocess.base_postprocess import Postprocess
from .yolov5_client import DATA, Yolov5preprocess


class Yolov4preprocess(Yolov5preprocess):
    scaling = "COCO"  # RGB / 255, NCHW (tools/torch_utils.py:do_detect)


class Yolov4postprocess(Postprocess):
    def __init__(self, input_hw=(512, 512)):
        self.input_hw = tuple(input_hw)

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


class Yolov4client(Client):
    def __init__(self):
        super().__init__()
        self.input_hw = (512, 512)

    def parse_model(self, model_metadata, model_config):
        r = super().parse_model(model_metadata, model_config)
        self.input_hw = (r[3], r[4])
        return r

    def get_preprocess(self):
        return Yolov4preprocess()

    def get_postprocess(self):
        return Yolov4postprocess(self.input_hw)
