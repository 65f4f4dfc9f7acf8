"""YOLOv5 (v6.x topology) — the 2D detector the reference serves as
``YOLOv5nCROP`` / ``YOLOv5nCOCO`` through Triton's onnxruntime backend
(reference ``examples/YOLOv5/config.pbtxt:1-19``, ``.vscode/launch.json:12``).

The reference only ever sees the model's *decoded* output tensor
``[B, N, 5+nc]`` (rows: cx, cy, w, h, obj, cls...; N = 3·(S/8)²+3·(S/16)²+3·(S/32)²,
e.g. 25200 at 640).  Here the network returns the three raw head maps and the
decode (sigmoid, grid offset, anchor scaling) is a separate op:
``triton_client_amd.ops.yolo.decode`` — on the GPU that decode is fused into
the candidate-filter kernel (``csrc/kernels/yolo.hip``), so the 8.5 MB decoded
tensor is never materialised on the hot path; for the KServe server contract
the same kernel can write the full decoded tensor.

Random-init weights, deterministic by seed; the detection-head biases get the
standard YOLO prior initialisation so objectness starts near the prior rather
than at 0.5 (matters for how many candidates reach NMS).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .common import ConvBNAct, kaiming_init


VARIANTS = {  # name: (depth_multiple, width_multiple)
    "n": (0.33, 0.25),
    "s": (0.33, 0.50),
    "m": (0.67, 0.75),
    "l": (1.0, 1.0),
    "x": (1.33, 1.25),
}

DEFAULT_ANCHORS = (
    (10, 13, 16, 30, 33, 23),
    (30, 61, 62, 45, 59, 119),
    (116, 90, 156, 198, 373, 326),
)
STRIDES = (8, 16, 32)


@dataclass
class YoloConfig:
    variant: str = "n"
    nc: int = 80
    img_size: Tuple[int, int] = (640, 640)  # (H, W)
    anchors: Sequence[Sequence[int]] = field(default_factory=lambda: DEFAULT_ANCHORS)

    @property
    def no(self) -> int:
        return self.nc + 5

    @property
    def na(self) -> int:
        return len(self.anchors[0]) // 2

    def grid_sizes(self) -> List[Tuple[int, int]]:
        h, w = self.img_size
        return [(h // s, w // s) for s in STRIDES]

    def num_predictions(self) -> int:
        return sum(self.na * gh * gw for gh, gw in self.grid_sizes())


def _ch(c: int, width: float) -> int:
    return int(math.ceil(c * width / 8) * 8)


def _n(n: int, depth: float) -> int:
    return max(round(n * depth), 1) if n > 1 else n


class Bottleneck(nn.Module):
    def __init__(self, c1: int, c2: int, shortcut: bool = True):
        super().__init__()
        self.cv1 = ConvBNAct(c1, c2, 1)
        self.cv2 = ConvBNAct(c2, c2, 3)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return x + y if self.add else y


class C3(nn.Module):
    """CSP block with 3 convolutions."""

    def __init__(self, c1: int, c2: int, n: int = 1, shortcut: bool = True):
        super().__init__()
        c_ = c2 // 2
        self.cv1 = ConvBNAct(c1, c_, 1)
        self.cv2 = ConvBNAct(c1, c_, 1)
        self.cv3 = ConvBNAct(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut) for _ in range(n)))

    def forward(self, x):
        return self.cv3(torch.cat((self.m(self.cv1(x)), self.cv2(x)), 1))


class SPPF(nn.Module):
    def __init__(self, c1: int, c2: int, k: int = 5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = ConvBNAct(c1, c_, 1)
        self.cv2 = ConvBNAct(c_ * 4, c2, 1)
        self.k = k

    def forward(self, x):
        x = self.cv1(x)
        p = self.k // 2
        y1 = F.max_pool2d(x, self.k, 1, p)
        y2 = F.max_pool2d(y1, self.k, 1, p)
        y3 = F.max_pool2d(y2, self.k, 1, p)
        return self.cv2(torch.cat((x, y1, y2, y3), 1))


class YOLOv5(nn.Module):
    """Backbone (CSP-Darknet + SPPF) + PANet neck + 3 detection convs.

    ``forward`` returns the three raw head maps ``[B, na*(5+nc), H_l, W_l]``.
    """

    def __init__(self, cfg: YoloConfig | None = None):
        super().__init__()
        cfg = cfg or YoloConfig()
        self.cfg = cfg
        d, w = VARIANTS[cfg.variant]
        c = lambda x: _ch(x, w)  # noqa: E731
        n = lambda x: _n(x, d)  # noqa: E731
        # backbone
        self.b0 = ConvBNAct(3, c(64), 6, 2, 2)
        self.b1 = ConvBNAct(c(64), c(128), 3, 2)
        self.b2 = C3(c(128), c(128), n(3))
        self.b3 = ConvBNAct(c(128), c(256), 3, 2)
        self.b4 = C3(c(256), c(256), n(6))
        self.b5 = ConvBNAct(c(256), c(512), 3, 2)
        self.b6 = C3(c(512), c(512), n(9))
        self.b7 = ConvBNAct(c(512), c(1024), 3, 2)
        self.b8 = C3(c(1024), c(1024), n(3))
        self.b9 = SPPF(c(1024), c(1024), 5)
        # head
        self.h10 = ConvBNAct(c(1024), c(512), 1, 1)
        self.h13 = C3(c(512) * 2, c(512), n(3), shortcut=False)
        self.h14 = ConvBNAct(c(512), c(256), 1, 1)
        self.h17 = C3(c(256) * 2, c(256), n(3), shortcut=False)
        self.h18 = ConvBNAct(c(256), c(256), 3, 2)
        self.h20 = C3(c(256) * 2, c(512), n(3), shortcut=False)
        self.h21 = ConvBNAct(c(512), c(512), 3, 2)
        self.h23 = C3(c(512) * 2, c(1024), n(3), shortcut=False)
        na, no = cfg.na, cfg.no
        self.detect = nn.ModuleList(nn.Conv2d(ch, na * no, 1) for ch in (c(256), c(512), c(1024)))
        kaiming_init(self)
        self._init_head_bias()
        self.register_buffer("anchors", torch.tensor(cfg.anchors, dtype=torch.float32).view(3, -1, 2))

    @torch.no_grad()
    def _init_head_bias(self) -> None:
        h, w = self.cfg.img_size
        for conv, s in zip(self.detect, STRIDES):
            b = conv.bias.view(self.cfg.na, -1)
            b[:, 4] += math.log(8 / (h / s * w / s))  # ~8 objects per image prior
            b[:, 5:] += math.log(0.6 / (self.cfg.nc - 0.99)) if self.cfg.nc > 1 else 0.0

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        x = self.b2(self.b1(self.b0(x)))
        p3 = self.b4(self.b3(x))
        p4 = self.b6(self.b5(p3))
        x = self.b9(self.b8(self.b7(p4)))
        h10 = self.h10(x)
        x = self.h13(torch.cat((F.interpolate(h10, scale_factor=2.0, mode="nearest"), p4), 1))
        h14 = self.h14(x)
        o3 = self.h17(torch.cat((F.interpolate(h14, scale_factor=2.0, mode="nearest"), p3), 1))
        o4 = self.h20(torch.cat((self.h18(o3), h14), 1))
        o5 = self.h23(torch.cat((self.h21(o4), h10), 1))
        return [m(o) for m, o in zip(self.detect, (o3, o4, o5))]


def yolo_decode_reference(heads: Sequence[torch.Tensor], anchors: torch.Tensor,
                          strides: Sequence[int] = STRIDES) -> torch.Tensor:
    """fp32 PyTorch reference of the YOLOv5 Detect decode.

    heads[l]: [B, na*no, H, W] (NCHW) or any layout convertible to it.
    Returns [B, sum(na*H*W), no] with rows (cx, cy, w, h, obj, cls...) in input
    pixels, ordered (level, anchor, y, x) like the exported ONNX model.
    """
    outs = []
    for l, h in enumerate(heads):
        h = h.float()
        b, _, ny, nx = h.shape
        na = anchors.shape[1]
        no = h.shape[1] // na
        y = h.view(b, na, no, ny, nx).permute(0, 1, 3, 4, 2).sigmoid()
        gy, gx = torch.meshgrid(torch.arange(ny, device=h.device), torch.arange(nx, device=h.device), indexing="ij")
        grid = torch.stack((gx, gy), -1).view(1, 1, ny, nx, 2).float()
        ag = (anchors[l].to(h.device).float()).view(1, na, 1, 1, 2)
        xy = (y[..., 0:2] * 2 - 0.5 + grid) * strides[l]
        wh = (y[..., 2:4] * 2) ** 2 * ag
        outs.append(torch.cat((xy, wh, y[..., 4:]), -1).view(b, -1, no))
    return torch.cat(outs, 1)


def build_yolov5(variant: str = "n", nc: int = 80, img_size: int | Tuple[int, int] = 640,
                 seed: int = 0) -> YOLOv5:
    if isinstance(img_size, int):
        img_size = (img_size, img_size)
    torch.manual_seed(seed)
    return YOLOv5(YoloConfig(variant=variant, nc=nc, img_size=tuple(img_size)))
