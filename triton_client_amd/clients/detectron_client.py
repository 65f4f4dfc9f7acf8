"""Detectron2 FCOS / RetinaNet client (reference ``clients/detectron_client.py``,
``clients/preprocess/detectron_preprocess.py``, ``clients/postprocess/detectron_postprocess.py``).

The server returns final detections (boxes ``[-1, 4]``, class ids INT64,
scores, image dims — ``examples/RetinaNet_detectron/config.pbtxt``), so the
client only decodes; inputs are un-normalised 0..255 (Detectron normalises
inside the model)."""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

from .base_client import Client
from .postprocess.base_postprocess import Postprocess
from .yolov5_client import DATA, Yolov5preprocess


class FCOSpreprocess(Yolov5preprocess):
    scaling = "NONE"


class FCOSpostprocess(Postprocess):
    def load_class_names(self, namesfile: Optional[str] = None) -> List[str]:
        return Postprocess.load_class_names(namesfile or os.path.join(DATA, "coco.names"))

    def extract_boxes(self, prediction, conf_thres: float = 0.0):
        boxes = self.output_array(prediction, 0).reshape(-1, 4)
        classes = self.output_array(prediction, 1).reshape(-1)
        scores = self.output_array(prediction, 2).reshape(-1)
        keep = scores >= conf_thres
        return [np.concatenate([boxes[keep], scores[keep, None], classes[keep, None].astype(np.float32)], 1)]

    def extract_boxes_device(self, responses, conf_thres: float = 0.0, iou_thres=None, xform=None, device="cuda",
                             **_):
        """Final server detections of several responses -> one device NmsResult (boxes
        in original-frame pixels with ``xform``) for the GPU annotator."""
        from .postprocess.device import pack_host_detections

        per = []
        for r in responses:
            d = self.extract_boxes(r, conf_thres)[0]
            if xform is not None and len(d):
                d[:, :4] = xform.unmap_boxes(d[:, :4])
            per.append(d)
        return pack_host_detections(per, device)


class FCOS_client(Client):
    def __init__(self, device="cpu"):
        super().__init__()
        self.device = device

    def get_preprocess(self):
        return FCOSpreprocess()

    def get_postprocess(self):
        return FCOSpostprocess()
