"""K1 — camera frame preprocessing (resize/letterbox + normalise + layout).

Reference: ``communicator/ros_inference.py:131-141`` (decode, BGR→RGB flip,
``cv2.resize`` stretch to the model size) and
``clients/preprocess/yolov5_preprocess.py:20-24`` (HWC→CHW, fp32, /255);
``clients/preprocess/detectron_preprocess.py:20-24`` (no /255);
``utils/preprocess.py:147-157`` (INCEPTION / VGG / COCO scaling — the only
implementation of the CLI's ``-s`` flag).

Fixes vs reference: the reference passes (H, W) to
``cv2.resize``'s (W, H) — wrong for non-square models; here dst is always
(H, W).  ``mode="letterbox"`` adds the aspect-preserving YOLOv5 letterbox.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence, Tuple

import numpy as np
import torch

from .. import _native
from . import golden
from ._ws import DTYPE_CODE

SCALING_PRESETS = {
    # name: (scale per channel, bias per channel)
    "COCO": ((1 / 255.0,) * 3, (0.0,) * 3),
    "YOLO": ((1 / 255.0,) * 3, (0.0,) * 3),
    "NONE": ((1.0,) * 3, (0.0,) * 3),
    "INCEPTION": ((1 / 127.5,) * 3, (-1.0,) * 3),
    "VGG": ((1.0,) * 3, (-123.0, -117.0, -104.0)),
}


@dataclass
class FrameXform:
    """How model-input pixels map back to the original frame (for boxes)."""
    gain_x: float
    gain_y: float
    pad_x: float
    pad_y: float
    orig_w: int
    orig_h: int

    def as_list(self):
        return [self.gain_x, self.gain_y, self.pad_x, self.pad_y, float(self.orig_w), float(self.orig_h)]

    def unmap_boxes(self, boxes: np.ndarray) -> np.ndarray:
        b = boxes.astype(np.float32).copy()
        b[:, [0, 2]] = np.clip((b[:, [0, 2]] - self.pad_x) / self.gain_x, 0, self.orig_w)
        b[:, [1, 3]] = np.clip((b[:, [1, 3]] - self.pad_y) / self.gain_y, 0, self.orig_h)
        return b


def frame_xform(src_hw: Tuple[int, int], dst_hw: Tuple[int, int], mode: str) -> Tuple[FrameXform, tuple]:
    top, left, nh, nw, gx, gy = golden.letterbox_params(src_hw, dst_hw, mode)
    return FrameXform(gx, gy, float(left), float(top), src_hw[1], src_hw[0]), (top, left, nh, nw)


def preprocess(frames: torch.Tensor, dst_hw: Tuple[int, int], mode: str = "stretch",
               scaling: str | Tuple[Sequence[float], Sequence[float]] = "COCO", dtype: torch.dtype = torch.float32,
               layout: str = "NCHW", out_channels: int = 3, swap_rb: bool = False, pad_value: float = 114.0,
               quantize_u8: bool = True, out: torch.Tensor | None = None, stream=None):
    """frames: [B, H, W, C>=3] uint8 (or [H, W, C]). Returns (tensor, FrameXform).

    layout "NCHW" → [B, C, H, W] contiguous; "NHWC" → [B, C, H, W] view of a
    channels_last buffer (C = out_channels, 3 or 4; the 4th channel is 0);
    "S2D" → [B, H/2, W/2, 16] space-to-depth (bf16 or fp32, see :func:`space_to_depth2`).
    """
    if frames.dim() == 3:
        frames = frames.unsqueeze(0)
    B, h0, w0, c0 = frames.shape
    H, W = dst_hw
    scale, bias = SCALING_PRESETS[scaling.upper()] if isinstance(scaling, str) else scaling
    xf, (top, left, nh, nw) = frame_xform((h0, w0), (H, W), mode)
    if layout == "S2D":
        return _preprocess_s2d(frames, (H, W), mode, scale, bias, swap_rb, pad_value, quantize_u8, out, stream,
                               xf, (top, left, nh, nw), dtype)
    if frames.device.type == "cuda":
        frames = frames.contiguous()
        if out is None:
            if layout == "NCHW":
                out = torch.empty((B, out_channels, H, W), dtype=dtype, device=frames.device)
            else:
                out = torch.empty((B, H, W, out_channels), dtype=dtype, device=frames.device).permute(0, 3, 1, 2)
        _native.call(
            "tca_image_preprocess", _native.ptr(frames), h0 * w0 * c0, h0, w0, w0 * c0, c0, int(swap_rb),
            _native.ptr(out), DTYPE_CODE[dtype], 0 if layout == "NCHW" else 1, out_channels, H, W, B, top, left,
            nh, nw, float(pad_value), int(quantize_u8), float(scale[0]), float(scale[1]), float(scale[2]),
            float(bias[0]), float(bias[1]), float(bias[2]), _native.stream_ptr(stream))
        return out, xf
    # CPU path (config 1 / GPU-less host): the C++ preprocess when the runtime
    # library is built, else the NumPy golden (bit-identical results)
    if out_channels == 3 and frames.dtype == torch.uint8 and dtype == torch.float32 and layout in ("NCHW", "NHWC"):
        rt = _cpu_runtime()
        if rt is not None:
            return _preprocess_cpu_native(rt, frames, (H, W), layout, swap_rb, pad_value, quantize_u8, scale, bias,
                                          (top, left, nh, nw), out, xf)
    res = []
    for b in range(B):
        img = frames[b].numpy()
        o = golden.preprocess_image(img, (H, W), mode, scale, bias, swap_rb, pad_value, "NHWC")
        if out_channels > 3:
            o = np.concatenate([o, np.zeros(o.shape[:-1] + (out_channels - 3,), o.dtype)], -1)
        res.append(o)
    arr = torch.from_numpy(np.stack(res)).to(dtype)
    if layout == "NCHW":
        t = arr.permute(0, 3, 1, 2).contiguous()
    else:
        t = arr.permute(0, 3, 1, 2)
    if out is not None:
        out.copy_(t)
        return out, xf
    return t, xf


def _cpu_runtime():
    try:
        return _native.runtime()
    except _native.NativeError:
        return None


def _preprocess_cpu_native(rt, frames, dst_hw, layout, swap_rb, pad_value, quantize_u8, scale, bias, region, out, xf):
    import ctypes
    import os

    B, h0, w0, c0 = frames.shape
    H, W = dst_hw
    top, left, nh, nw = region
    frames = frames.contiguous()
    res = torch.empty((B, 3, H, W) if layout == "NCHW" else (B, H, W, 3), dtype=torch.float32)
    sc = (ctypes.c_float * 3)(*[float(v) for v in scale])
    bi = (ctypes.c_float * 3)(*[float(v) for v in bias])
    threads = min(8, os.cpu_count() or 1)
    for b in range(B):
        rt.tca_cpu_preprocess(frames[b].data_ptr(), h0, w0, c0, int(swap_rb), res[b].data_ptr(),
                              0 if layout == "NCHW" else 1, H, W, top, left, nh, nw, float(pad_value),
                              int(quantize_u8), sc, bi, threads)
    t = res if layout == "NCHW" else res.permute(0, 3, 1, 2)
    if out is not None:
        out.copy_(t)
        return out, xf
    return t, xf


def planar_affine(x: torch.Tensor, out: torch.Tensor, scale=(1.0, 1.0, 1.0), bias=(0.0, 0.0, 0.0),
                  stream=None) -> torch.Tensor:
    """A model-sized fp32 NCHW request tensor ``x`` [B, 3, H, W] (the served contracts'
    input) -> ``out``: NHWC [B, H, W, 8] (3 channels + zero pad) or space-to-depth
    [B, H/2, W/2, 16], fp32 or bf16, with ``x * scale[c] + bias[c]`` — one kernel
    (image.hip tca_planar_affine), capturable, instead of a normalise + permute +
    pad chain of PyTorch element-wise ops."""
    B, C, H, W = x.shape
    assert C == 3 and x.dtype == torch.float32 and x.is_contiguous(), (x.shape, x.dtype)
    if tuple(out.shape) == (B, H, W, 8):
        layout = 1
    elif tuple(out.shape) == (B, H // 2, W // 2, 16):
        layout = 2
    else:
        raise ValueError(f"planar_affine: output {tuple(out.shape)} is neither NHWC x 8 nor S2D x 16 of {tuple(x.shape)}")
    if not x.is_cuda:
        y = x * torch.tensor(scale).view(1, 3, 1, 1) + torch.tensor(bias).view(1, 3, 1, 1)
        y = y.permute(0, 2, 3, 1)
        if layout == 2:
            y = space_to_depth2(y)
        else:
            y = torch.cat([y, torch.zeros(B, H, W, 5)], -1)
        out.copy_(y.to(out.dtype))
        return out
    assert out.is_contiguous() and out.dtype in (torch.float32, torch.bfloat16)
    _native.call("tca_planar_affine", _native.ptr(x), B, H, W, _native.ptr(out), 0 if out.dtype == torch.float32 else 2,
                 layout, *[float(v) for v in scale], *[float(v) for v in bias], _native.stream_ptr(stream))
    return out


def space_to_depth2(x: torch.Tensor) -> torch.Tensor:
    """[B, H, W, 3] -> [B, H/2, W/2, 16]: channel (dy*2 + dx)*3 + c = x[2Y+dy, 2X+dx, c];
    channels 12..15 are zero.  A k=6, s=2, p=2 conv over x equals a 3x3, s=1,
    p=1 conv over this tensor (weights: :func:`s2d_stem_weight`)."""
    B, H, W, C = x.shape
    assert C == 3 and H % 2 == 0 and W % 2 == 0
    y = x.view(B, H // 2, 2, W // 2, 2, 3).permute(0, 1, 3, 2, 4, 5).reshape(B, H // 2, W // 2, 12)
    return torch.cat([y, y.new_zeros(B, H // 2, W // 2, 4)], -1)


def s2d_stem_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, 3, 6, 6] (stride 2, pad 2) -> [Cout, 16, 3, 3] (stride 1, pad 1) over space_to_depth2 input:
    W'[o, (dy*2+dx)*3 + c, a, b] = W[o, c, 2a + dy, 2b + dx]."""
    co, ci, kh, kw = w.shape
    assert ci == 3 and kh == 6 and kw == 6
    v = w.view(co, 3, 3, 2, 3, 2)                # o, c, a, dy, b, dx
    v = v.permute(0, 3, 5, 1, 2, 4).reshape(co, 12, 3, 3)  # o, (dy, dx, c), a, b
    return torch.cat([v, v.new_zeros(co, 4, 3, 3)], 1)


def _preprocess_s2d(frames, dst_hw, mode, scale, bias, swap_rb, pad_value, quantize_u8, out, stream, xf, region,
                    dtype=torch.bfloat16):
    B, h0, w0, c0 = frames.shape
    H, W = dst_hw
    top, left, nh, nw = region
    if out is None:
        out = torch.zeros((B, H // 2, W // 2, 16), dtype=dtype, device=frames.device)
    if frames.device.type == "cuda":
        frames = frames.contiguous()
        _native.call(
            "tca_image_preprocess", _native.ptr(frames), h0 * w0 * c0, h0, w0, w0 * c0, c0, int(swap_rb),
            _native.ptr(out), DTYPE_CODE[out.dtype], 2, 16, H, W, B, top, left, nh, nw, float(pad_value),
            int(quantize_u8), float(scale[0]), float(scale[1]), float(scale[2]), float(bias[0]), float(bias[1]),
            float(bias[2]), _native.stream_ptr(stream))
        return out, xf
    res = [golden.preprocess_image(frames[b].numpy(), (H, W), mode, scale, bias, swap_rb, pad_value, "NHWC")
           for b in range(B)]
    out.copy_(space_to_depth2(torch.from_numpy(np.stack(res))).to(out.dtype))
    return out, xf


def yolo_stem_fused(frames: torch.Tensor, dst_hw: Tuple[int, int], mode: str, stem, b1, out,
                    scaling: str = "COCO", swap_rb: bool = False, pad_value: float = 114.0, quantize_u8: bool = True,
                    stream=None):
    """K1 + the YOLOv5 s2d stem + its first 3x3 stride-2 conv in one kernel
    (``tca_yolo_stem_fused``, ``csrc/kernels/image.hip``): uint8 frames [B, h0, w0, 3] ->
    ``out`` (an fp32 NHWC view, 32 channels) at dst_hw / 4.  ``stem`` / ``b1`` are the plan's
    fp32 FusedConvs (split weights).  Same values as preprocess(S2D) -> stem -> b1."""
    B, h0, w0, c0 = frames.shape
    H, W = dst_hw
    scale, bias = SCALING_PRESETS[scaling.upper()] if isinstance(scaling, str) else scaling
    xf, (top, left, nh, nw) = frame_xform((h0, w0), (H, W), mode)
    frames = frames.contiguous()
    _native.call("tca_yolo_stem_fused", _native.ptr(frames), h0 * w0 * c0, h0, w0, w0 * c0, c0, int(swap_rb), H, W, B,
                 top, left, nh, nw, float(pad_value), int(quantize_u8), float(scale[0]), float(scale[1]),
                 float(scale[2]), float(bias[0]), float(bias[1]), float(bias[2]), _native.ptr(stem.w_gemm),
                 _native.ptr(stem.b_gemm), stem.act, _native.ptr(b1.w_gemm), _native.ptr(b1.b_gemm), b1.act,
                 _native.ptr(out.t), out.t.shape[-1], out.off, _native.stream_ptr(stream))
    return out, xf


def draw_boxes_(frames: torch.Tensor, box: torch.Tensor, cls: torch.Tensor, count: torch.Tensor,
                thickness: int = 2, stream=None) -> torch.Tensor:
    """K15: draw result boxes onto uint8 frames in place (``csrc/kernels/draw.hip``).

    frames [B, H, W, 3] uint8 (row-contiguous), box [B, K, D>=4] fp32 x1,y1,x2,y2
    in frame pixels, cls [B, K] int32, count [B] int32.  Boxes 0..count-1 are
    drawn in order (a later box wins where boxes overlap), pixel-identical to
    :func:`triton_client_amd.utils.draw.draw_rect` with ``class_color``
    (reference ``ros_inference.py:149-169``)."""
    B, H, W, C = frames.shape
    if C != 3 or frames.dtype != torch.uint8 or frames.stride(2) != 3 or frames.stride(1) != 3 * W:
        raise ValueError("frames must be [B, H, W, 3] uint8 with contiguous rows")
    if box.dim() != 3 or box.shape[0] != B or box.shape[2] < 4 or not box.is_contiguous():
        raise ValueError("box must be contiguous [B, K, >=4]")
    if tuple(cls.shape) != tuple(box.shape[:2]) or cls.dtype != torch.int32 or count.dtype != torch.int32:
        raise ValueError("cls [B, K] int32 and count [B] int32")
    if frames.is_cuda:
        _native.call("tca_draw_boxes", _native.ptr(frames), frames.stride(0), B, H, W, frames.stride(1),
                     _native.ptr(box), box.shape[1], box.shape[2], _native.ptr(cls.contiguous()),
                     _native.ptr(count), thickness, _native.stream_ptr(stream))
        return frames
    from ..utils.draw import class_color, draw_rect

    cnt = count.numpy()
    for b in range(B):
        img = frames[b].numpy()
        for k in range(min(int(cnt[b]), box.shape[1])):
            x = box[b, k].tolist()
            draw_rect(img, x[0], x[1], x[2], x[3], class_color(int(cls[b, k])), thickness)
    return frames


def draw_annotations_(frames: torch.Tensor, box: torch.Tensor, score: torch.Tensor, cls: torch.Tensor,
                      count: torch.Tensor, names_dev: torch.Tensor | None = None, names=None, thickness: int = 2,
                      stream=None) -> torch.Tensor:
    """K15 with labels: every result box's rectangle, then its ``"<name> <conf>"``
    label, drawn in place on uint8 frames [B, H, W, 3] (``tca_draw_annotations``;
    capture-safe).  ``names_dev``: the [n, 32] uint8 device table of
    :func:`triton_client_amd.utils.draw.names_table` (None: numeric class ids).
    Pixel-identical to :func:`triton_client_amd.utils.draw.draw_detections`
    (``names``: the same class names, used by the CPU path)."""
    B, H, W, C = frames.shape
    if C != 3 or frames.dtype != torch.uint8 or frames.stride(2) != 3 or frames.stride(1) != 3 * W:
        raise ValueError("frames must be [B, H, W, 3] uint8 with contiguous rows")
    if box.dim() != 3 or box.shape[0] != B or box.shape[2] < 4 or not box.is_contiguous():
        raise ValueError("box must be contiguous [B, K, >=4]")
    if (tuple(cls.shape) != tuple(box.shape[:2]) or cls.dtype != torch.int32 or count.dtype != torch.int32
            or tuple(score.shape) != tuple(box.shape[:2]) or score.dtype != torch.float32):
        raise ValueError("score [B, K] fp32, cls [B, K] int32 and count [B] int32")
    if frames.is_cuda:
        if names_dev is not None and (names_dev.dtype != torch.uint8 or names_dev.dim() != 2
                                      or names_dev.shape[1] != 32 or not names_dev.is_cuda):
            raise ValueError("names_dev must be a [n, 32] uint8 device table")
        nn = 0 if names_dev is None else names_dev.shape[0]
        _native.call("tca_draw_annotations", _native.ptr(frames), frames.stride(0), B, H, W, frames.stride(1),
                     _native.ptr(box), box.shape[1], box.shape[2], _native.ptr(score.contiguous()),
                     _native.ptr(cls.contiguous()), _native.ptr(count), thickness,
                     _native.ptr(names_dev) if nn else 0, nn, _native.stream_ptr(stream))
        return frames
    from ..utils.draw import draw_detections

    cnt = count.numpy()
    for b in range(B):
        k = min(int(cnt[b]), box.shape[1])
        d = np.concatenate([box[b, :k, :4].numpy(), score[b, :k, None].numpy(),
                            cls[b, :k, None].numpy().astype(np.float32)], 1)
        draw_detections(frames[b].numpy(), d, names, thickness)
    return frames
