"""2D Detectron2 RetinaNet / FCOS pipeline on one GPU: raw uint8 frames → detections.

    frames u8 [B,H0,W0,3] ─K1 letterbox + (x-mean)/std→ NHWC×8 bf16 [B,800,1344,8]
    ─ResNet-50-FPN + head (fused MFMA convs, GN kernels for FCOS)→ per-level maps
    ─K-R / K-F decode → per-level top-1000 → segment merge → class-aware NMS
    (K4, box rescale to the frame) → boxes [B,100,4], scores, classes

The reference serves these networks behind Triton's libtorch backend
(``examples/RetinaNet_detectron/config.pbtxt``) and only decodes the final
detections on the client (``clients/postprocess/detectron_postprocess.py``).
Here the whole step is one captured hipGraph (BASELINE config 3: 1333×800
class, batched, data-parallel).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..config.detectron import DetectronConfig
from ..models.common import fuse_model, lsuv_rescale
from ..models.detectron import DetectronDetector, build_detectron
from ..ops.detectron import DetectronPostprocess
from ..ops.image import frame_xform, preprocess


class DetectronPipeline:
    def __init__(self, model: Optional[DetectronDetector] = None, batch: int = 16,
                 src_hw: Tuple[int, int] = (720, 1280), cfg: Optional[DetectronConfig] = None, device="cuda",
                 seed: int = 0, mode: str = "letterbox", precision: str = "fp32"):
        """precision "fp32": the reference's serving precision (libtorch fp32,
        examples/RetinaNet_detectron/config.pbtxt) — fp32 activations and
        split-product convs; "bf16" the faster secondary mode."""
        self.device = torch.device(device)
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision {precision!r}")
        self.precision = precision
        self.dtype = torch.float32 if precision == "fp32" else torch.bfloat16
        if self.device.type != "cuda":
            raise ValueError("DetectronPipeline runs on the GPU; use models.detectron on the CPU")
        if model is None:
            model = build_detectron(cfg, seed)
        model = fuse_model(model.eval())
        self.cfg = model.cfg
        self.model = model.to(device=self.device, dtype=self.dtype, memory_format=torch.channels_last)
        self.B, self.src_hw, self.mode = batch, tuple(src_hw), mode
        self.frames = torch.zeros((batch, *self.src_hw, 3), dtype=torch.uint8, device=self.device)
        self.xform, _ = frame_xform(self.src_hw, self.cfg.input_hw, mode)
        mean, std = self.cfg.pixel_mean, self.cfg.pixel_std
        # K1 computes v * scale + bias on 0..255 pixels: fold (v - mean) / std into it
        self.scaling = ([1.0 / s for s in std], [-m / s for m, s in zip(mean, std)])
        self.post = DetectronPostprocess(self.cfg, batch, self.device)
        self.fast = None

    def build_fast(self):
        from ..models.fast import FastDetectron

        self.fast = FastDetectron(self.model, self.B, self.device, precision=self.precision)
        return self.fast

    def _input_nchw(self):
        """Un-normalised 0..255 NCHW input (the mode's dtype) for the module path (calibration)."""
        x, _ = preprocess(self.frames, self.cfg.input_hw, self.mode, ([1.0] * 3, [0.0] * 3), self.dtype,
                          "NHWC", 3)
        return x

    @torch.no_grad()
    def calibrate_detection_density(self, target_per_frame: float = 300.0, lsuv: bool = True) -> float:
        """LSUV-rescale the random network on the current frames, then shift
        the class-logit bias so ~target (location, class) pairs per frame pass
        the score threshold, as a trained detector would hand to NMS.  Returns
        the shift."""
        x = self._input_nchw()
        hd = self.model.head
        finals = [hd.cls_score, hd.bbox_pred] + ([hd.ctrness] if self.cfg.arch == "fcos" else [])
        if lsuv:
            lsuv_rescale(self.model, lambda: self.model(x), head_modules=finals, head_std=1.5)
            hd.bbox_pred.weight.mul_(0.2)
            hd.bbox_pred.bias.mul_(0.2)
            if self.cfg.arch == "retinanet":
                hd.cls_score.bias.fill_(-4.595)
            else:
                hd.cls_score.bias.fill_(-4.595)
                hd.bbox_pred.bias.add_(1.0)  # positive ltrb distances (~2.7 strides)
        outs = self.model(x)
        t = self.cfg.score_thresh
        if self.cfg.arch == "retinanet":
            logits = torch.cat([o[0].float().flatten(1) for o in outs], 1)

            def count(d):
                return (torch.sigmoid(logits + d) > t).float().sum(1).mean().item()
        else:
            cls = torch.cat([o[0].float().flatten(2) for o in outs], 2)  # [B, C, N]
            ctr = torch.sigmoid(torch.cat([o[2].float().flatten(2) for o in outs], 2))

            def count(d):
                return (torch.sqrt(torch.sigmoid(cls + d) * ctr) > t).float().sum((1, 2)).mean().item()

        lo, hi = -30.0, 30.0
        for _ in range(50):
            mid = 0.5 * (lo + hi)
            if count(mid) > target_per_frame:
                hi = mid
            else:
                lo = mid
        d = 0.5 * (lo + hi)
        hd.cls_score.bias += d
        self.calibration_shift = d
        self.fast = None
        return d

    @torch.no_grad()
    def step(self):
        f = self.fast or self.build_fast()
        preprocess(self.frames, self.cfg.input_hw, self.mode, self.scaling, self.dtype, "NHWC",
                   f.IN_CHANNELS, out=f.input_view())
        return self.post(f.forward(), self.xform)
