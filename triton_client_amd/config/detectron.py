"""Detectron2 one-stage detectors served behind ``examples/RetinaNet_detectron/config.pbtxt``.

The reference only has the served contract (``input__00`` FP32 NCHW
[3, 640, 480] un-normalised 0..255 → ``bboxex__0`` [-1, 4], ``classes__1``
INT64, ``scores__2``, ``dims__3`` INT64 [1, 2]) and the client decode
(``clients/postprocess/detectron_postprocess.py:26-38``).  The networks are
Detectron2's defaults (``RetinaNet R50-FPN 1x`` / ``FCOS R50-FPN 1x``); there
are no configs in the reference, so these numbers are Detectron2's defaults
("parity unpinned": no reference outputs exist to compare against).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Tuple


@dataclass
class DetectronConfig:
    arch: str = "retinanet"                  # "retinanet" | "fcos"
    num_classes: int = 80
    input_hw: Tuple[int, int] = (800, 1344)  # model input (multiple of 32; 1333x800 class, BASELINE config 3)
    depth_blocks: Tuple[int, ...] = (3, 4, 6, 3)  # ResNet-50
    stride_in_1x1: bool = True               # Detectron2 MSRA ResNet default
    fpn_channels: int = 256
    strides: Tuple[int, ...] = (8, 16, 32, 64, 128)  # P3..P7
    # input normalisation (RGB order; the reference clients send RGB 0..255)
    pixel_mean: Tuple[float, float, float] = (123.675, 116.28, 103.53)
    pixel_std: Tuple[float, float, float] = (58.395, 57.12, 57.375)
    # RetinaNet anchors: per level size 32 * 2^l * {2^0, 2^(1/3), 2^(2/3)}, ratios {0.5, 1, 2}
    anchor_sizes: Tuple[float, ...] = (32.0, 64.0, 128.0, 256.0, 512.0)
    anchor_scales: Tuple[float, ...] = (1.0, 2 ** (1 / 3), 2 ** (2 / 3))
    anchor_ratios: Tuple[float, ...] = (0.5, 1.0, 2.0)
    head_convs: int = 4
    score_thresh: float = -1.0               # -1: 0.05 RetinaNet / 0.2 FCOS
    topk_per_level: int = 1000
    nms_thresh: float = -1.0                 # -1: 0.5 RetinaNet / 0.6 FCOS
    max_detections: int = 100
    scale_clamp: float = math.log(1000.0 / 16)

    def __post_init__(self):
        if self.score_thresh < 0:
            self.score_thresh = 0.05 if self.arch == "retinanet" else 0.2
        if self.nms_thresh < 0:
            self.nms_thresh = 0.5 if self.arch == "retinanet" else 0.6

    @property
    def num_anchors(self) -> int:
        return len(self.anchor_scales) * len(self.anchor_ratios) if self.arch == "retinanet" else 1

    def level_hw(self):
        """(H, W) of P3..P7: stem conv7 s2 p3 → maxpool3 s2 p1 → res3/res4/res5 (stride-2
        1x1 or 3x3) → P6/P7 conv3 s2 p1."""
        def conv(n, k, s, p):
            return (n + 2 * p - k) // s + 1

        out = []
        hw = [conv(conv(x, 7, 2, 3), 3, 2, 1) for x in self.input_hw]  # res2
        for _ in range(3):  # res3, res4, res5
            hw = [conv(x, 1, 2, 0) for x in hw]
            out.append(tuple(hw))
        for _ in range(2):  # P6, P7
            hw = [conv(x, 3, 2, 1) for x in hw]
            out.append(tuple(hw))
        return out

    def anchor_table(self, level: int):
        """[A, 2] (w, h) of the level's anchors, Detectron2 DefaultAnchorGenerator order
        (sizes outer, aspect ratios inner)."""
        res = []
        base = self.anchor_sizes[level]
        for sc in self.anchor_scales:
            size = base * sc
            area = size * size
            for r in self.anchor_ratios:
                w = math.sqrt(area / r)
                res.append((w, r * w))
        return res
