"""2D YOLOv4 pipeline on one GPU (reference ``examples/YOLOv4/config.pbtxt`` model):
raw uint8 frames → K1 (resize, /255) → CSPDarknet53-SPP-PANet (fused MFMA
convs, Mish / Leaky epilogues, in-place routes) → K5 decode + filter → K4
per-class NMS (0.6) with the box rescale → detections.  One hipGraph.
``precision="fp32"`` (default; the served model is FP32, ``examples/YOLOv4/config.pbtxt``):
fp32 activations with split-product MFMA convs; ``"bf16"`` is the secondary mode."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..models.common import fuse_model, lsuv_rescale
from ..models.yolov4 import YOLOV4_OUTPUTS, YOLOv4, build_yolov4
from ..ops.image import frame_xform, preprocess
from ..ops.yolov4 import Yolov4Postprocess


class Yolov4Pipeline:
    def __init__(self, model: Optional[YOLOv4] = None, batch: int = 16, src_hw: Tuple[int, int] = (720, 1280),
                 img: int = 512, nc: int = 80, mode: str = "stretch", conf_thres: float = 0.4,
                 nms_thres: float = 0.6, device="cuda", seed: int = 0, precision: str = "fp32",
                 max_out: int = 1000):
        self.device = torch.device(device)
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision {precision!r}")
        self.precision = precision
        self.dtype = torch.float32 if precision == "fp32" else torch.bfloat16
        if self.device.type != "cuda":
            raise ValueError("Yolov4Pipeline runs on the GPU; use models.yolov4 on the CPU")
        if model is None:
            model = build_yolov4(nc, img, seed)
        model = fuse_model(model.eval())
        self.model = model.to(device=self.device, dtype=self.dtype, memory_format=torch.channels_last)
        self.cfg = model.cfg
        self.B, self.src_hw, self.mode = batch, tuple(src_hw), mode
        self.img_hw = self.cfg.img
        self.frames = torch.zeros((batch, *self.src_hw, 3), dtype=torch.uint8, device=self.device)
        self.xform, _ = frame_xform(self.src_hw, self.img_hw, mode)
        self.post = Yolov4Postprocess(self.cfg.nc, self.img_hw, conf_thres, nms_thres,
                                      max_out=max_out, device=self.device)
        self.fast = None

    def build_fast(self):
        from ..models.fast import FastGraph

        self.fast = FastGraph(self.model, self.B, self.img_hw, self.device, outputs=YOLOV4_OUTPUTS,
                              precision=self.precision)
        return self.fast

    @torch.no_grad()
    def calibrate_detection_density(self, target_per_frame: float = 100.0, lsuv: bool = True) -> float:
        """LSUV on the current frames, then one logit shift on objectness and
        class biases so ~target rows per frame pass conf > conf_thres."""
        x, _ = preprocess(self.frames, self.img_hw, self.mode, "COCO", self.dtype, "NHWC", 3)
        heads = [self.model.layers[n] for n in YOLOV4_OUTPUTS]
        if lsuv:
            lsuv_rescale(self.model, lambda: self.model(x), head_modules=heads, head_std=1.5)
        outs = self.model(x)
        nc, t = self.cfg.nc, self.post.conf_thres
        obj, cls = [], []
        for o in outs:
            v = o.float().view(o.shape[0], 3, 5 + nc, -1)
            obj.append(v[:, :, 4].flatten(1))
            cls.append(v[:, :, 5:].max(2).values.flatten(1))
        obj, cls = torch.cat(obj, 1), torch.cat(cls, 1)

        def count(d):
            return (torch.sigmoid(obj + d) * torch.sigmoid(cls + d) > t).float().sum(1).mean().item()

        lo, hi = -30.0, 30.0
        for _ in range(50):
            mid = 0.5 * (lo + hi)
            if count(mid) > target_per_frame:
                hi = mid
            else:
                lo = mid
        d = 0.5 * (lo + hi)
        for m in heads:
            b = m.conv.bias.view(3, 5 + nc)
            b[:, 4:] += d
        self.calibration_shift = d
        self.fast = None
        return d

    @torch.no_grad()
    def step(self):
        f = self.fast or self.build_fast()
        preprocess(self.frames, self.img_hw, self.mode, "COCO", self.dtype, "NHWC", f.IN_CHANNELS,
                   out=f.input_view())
        return self.post(f.forward(), self.xform)
