"""Golden (sequential, obviously-correct) NumPy references for every per-frame
op.  They re-state the reference's semantics — not its code — and are what
the HIP kernels and the vectorised CPU paths are tested against:

* ``resize_bilinear_u8``     — OpenCV INTER_LINEAR pixel-centre convention
  (reference ``communicator/ros_inference.py:140``, cv2 is not installed here,
  so bit-exactness with cv2's fixed point is "parity unpinned"; we match the
  float formula and round to uint8 like cv2's u8 output).
* ``letterbox_params``       — YOLOv5 letterbox geometry.
* ``nms_greedy``             — torchvision.ops.nms semantics (score-desc,
  suppress IoU > thr), class-aware like the reference's class-offset trick.
* ``voxelize_sequential``    — spconv ``points_to_voxel`` loop.
* ``rotated_iou_bev``        — polygon clipping IoU (OpenPCDet iou_bev).
* ``pc2_read_points``        — ``sensor_msgs.point_cloud2.read_points(skip_nans)``.
"""
from __future__ import annotations

import math
import struct
from typing import List, Sequence, Tuple

import numpy as np


# ----------------------------------------------------------------------------- image
def _axis_coords(n_dst: int, n_src: int):
    scale = np.float32(n_src) / np.float32(n_dst)  # fp32 like the kernel
    f = (np.arange(n_dst, dtype=np.float32) + np.float32(0.5)) * scale - np.float32(0.5)
    s = np.floor(f).astype(np.int64)
    a = f - s.astype(np.float32)
    a = np.where(s < 0, 0.0, a)
    s = np.where(s < 0, 0, s)
    hi = s >= n_src - 1
    a = np.where(hi, 0.0, a)
    s = np.where(hi, n_src - 1, s)
    s1 = np.minimum(s + 1, n_src - 1)
    return s, s1, a.astype(np.float32)


def resize_bilinear_u8(img: np.ndarray, out_h: int, out_w: int, quantize: bool = True) -> np.ndarray:
    """img [H, W, C] uint8 → [out_h, out_w, C] (uint8 if quantize else float32)."""
    H, W = img.shape[:2]
    y0, y1, ay = _axis_coords(out_h, H)
    x0, x1, ax = _axis_coords(out_w, W)
    f = img.astype(np.float32)
    ax_ = ax[None, :, None]
    top = f[y0][:, x0] + ax_ * (f[y0][:, x1] - f[y0][:, x0])
    bot = f[y1][:, x0] + ax_ * (f[y1][:, x1] - f[y1][:, x0])
    out = top + ay[:, None, None] * (bot - top)
    if quantize:
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)
    return out


def letterbox_params(src_hw: Tuple[int, int], dst_hw: Tuple[int, int], mode: str = "letterbox"):
    """Returns (reg_top, reg_left, reg_h, reg_w, gain_x, gain_y).

    stretch  : the whole dst is the resized region (reference behaviour,
               ``cv2.resize(img, (W, H))``).
    letterbox: keep aspect ratio, centre, pad 114 (YOLOv5 ``letterbox``).
    """
    h0, w0 = src_hw
    H, W = dst_hw
    if mode == "stretch":
        return 0, 0, H, W, W / w0, H / h0
    r = min(H / h0, W / w0)
    nw, nh = int(round(w0 * r)), int(round(h0 * r))
    dw, dh = (W - nw) / 2.0, (H - nh) / 2.0
    top, left = int(round(dh - 0.1)), int(round(dw - 0.1))
    return top, left, nh, nw, nw / w0, nh / h0


def preprocess_image(img: np.ndarray, dst_hw, mode="stretch", scale=(1 / 255.0,) * 3, bias=(0.0,) * 3,
                     swap_rb=False, pad=114.0, layout="NCHW") -> np.ndarray:
    H, W = dst_hw
    top, left, nh, nw, _, _ = letterbox_params(img.shape[:2], dst_hw, mode)
    canvas = np.full((H, W, 3), pad, np.float32)
    canvas[top:top + nh, left:left + nw] = resize_bilinear_u8(img[..., :3], nh, nw).astype(np.float32)
    if swap_rb:
        canvas = canvas[..., ::-1]
    out = canvas * np.asarray(scale, np.float32) + np.asarray(bias, np.float32)
    return out.transpose(2, 0, 1).copy() if layout == "NCHW" else out


# ----------------------------------------------------------------------------- 2D NMS
def box_iou_np(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    ix1 = np.maximum(a[:, None, 0], b[None, :, 0])
    iy1 = np.maximum(a[:, None, 1], b[None, :, 1])
    ix2 = np.minimum(a[:, None, 2], b[None, :, 2])
    iy2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(ix2 - ix1, 0, None) * np.clip(iy2 - iy1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    with np.errstate(invalid="ignore", divide="ignore"):
        return inter / (aa[:, None] + ab[None, :] - inter)


def nms_greedy(boxes: np.ndarray, scores: np.ndarray, thr: float, classes=None, order_key=None,
               iou_fn=None, max_out: int | None = None) -> List[int]:
    """Greedy NMS; returns kept indices in score order.

    order_key: optional int array used to break score ties (ascending), the
    same (score desc, index asc) order the GPU sort uses."""
    n = len(scores)
    if n == 0:
        return []
    if order_key is None:
        order_key = np.arange(n)
    order = np.lexsort((order_key, -scores.astype(np.float64)))
    iou_fn = iou_fn or (lambda a, b: box_iou_np(a[None], b)[0])
    removed = np.zeros(n, bool)
    keep = []
    for oi, i in enumerate(order):
        if removed[i]:
            continue
        keep.append(int(i))
        if max_out is not None and len(keep) >= max_out:
            break
        rest = order[oi + 1:]
        rest = rest[~removed[rest]]
        if len(rest) == 0:
            continue
        ious = iou_fn(boxes[i], boxes[rest])
        sup = ious > thr
        if classes is not None:
            sup &= classes[rest] == classes[i]
        removed[rest[sup]] = True
    return keep


# ----------------------------------------------------------------------------- rotated IoU
def _corners(b):
    c, s = math.cos(b[6]), math.sin(b[6])
    hx, hy = b[3] / 2, b[4] / 2
    pts = []
    for ox, oy in ((-hx, -hy), (hx, -hy), (hx, hy), (-hx, hy)):
        pts.append((b[0] + c * ox - s * oy, b[1] + s * ox + c * oy))
    return pts


def _clip(poly, a, b):
    out = []
    n = len(poly)
    def side(p):
        return (b[0] - a[0]) * (p[1] - a[1]) - (b[1] - a[1]) * (p[0] - a[0])
    for i in range(n):
        cur, nxt = poly[i], poly[(i + 1) % n]
        dc, dn = side(cur), side(nxt)
        if dc >= 0:
            out.append(cur)
        if (dc >= 0) != (dn >= 0):
            t = dc / (dc - dn)
            out.append((cur[0] + t * (nxt[0] - cur[0]), cur[1] + t * (nxt[1] - cur[1])))
    return out


def rotated_overlap(a, b) -> float:
    poly = _corners(a)
    cb = _corners(b)
    for i in range(4):
        if not poly:
            break
        poly = _clip(poly, cb[i], cb[(i + 1) % 4])
    if len(poly) < 3:
        return 0.0
    area = 0.0
    for i in range(len(poly)):
        p, q = poly[i], poly[(i + 1) % len(poly)]
        area += p[0] * q[1] - q[0] * p[1]
    return abs(area) / 2


def rotated_iou_bev(a, bs) -> np.ndarray:
    out = np.zeros(len(bs), np.float64)
    if len(bs) == 0:
        return out
    bs_ = np.asarray(bs, np.float64)
    # exact prefilter: boxes whose bounding circles do not meet have no overlap (IoU 0)
    ra = 0.5 * math.hypot(a[3], a[4])
    rb = 0.5 * np.hypot(bs_[:, 3], bs_[:, 4])
    near = np.hypot(bs_[:, 0] - a[0], bs_[:, 1] - a[1]) <= ra + rb
    for k in np.nonzero(near)[0]:
        b = bs_[k]
        ov = rotated_overlap(a, b)
        out[k] = ov / max(a[3] * a[4] + b[3] * b[4] - ov, 1e-8)
    return out


# ----------------------------------------------------------------------------- point clouds
PF_FMT = {1: "b", 2: "B", 3: "h", 4: "H", 5: "i", 6: "I", 7: "f", 8: "d"}


def pc2_read_points(data: bytes, n: int, point_step: int, offsets: Sequence[int], dtypes: Sequence[int]):
    """Sequential read_points(skip_nans=True) over 4 fields → [M, 4] float32."""
    out = []
    for i in range(n):
        rec = i * point_step
        vals = [struct.unpack_from("<" + PF_FMT[dt], data, rec + off)[0] for off, dt in zip(offsets, dtypes)]
        if any(isinstance(v, float) and math.isnan(v) for v in vals):
            continue
        out.append(vals)
    return np.asarray(out, np.float32).reshape(-1, 4)


def voxelize_sequential(points: np.ndarray, pc_range, voxel_size, max_points: int, max_voxels: int):
    """spconv points_to_voxel loop (continue-on-full semantics).

    Returns voxels [V, P, F], coords [V, 3] (z, y, x), num_points [V]."""
    r = np.asarray(pc_range, np.float32)
    vs = np.asarray(voxel_size, np.float32)
    grid = np.round((r[3:] - r[:3]) / vs).astype(np.int64)
    F = points.shape[1]
    coor_to_vid = {}
    voxels, coords, num = [], [], []
    for i in range(points.shape[0]):
        p = points[i]
        c = np.floor((p[:3] - r[:3]) / vs).astype(np.int64)
        if np.any(c < 0) or np.any(c >= grid):
            continue
        key = (int(c[2]), int(c[1]), int(c[0]))
        vid = coor_to_vid.get(key, -1)
        if vid == -1:
            if len(voxels) >= max_voxels:
                continue
            vid = len(voxels)
            coor_to_vid[key] = vid
            voxels.append(np.zeros((max_points, F), np.float32))
            coords.append(key)
            num.append(0)
        if num[vid] < max_points:
            voxels[vid][num[vid]] = p
            num[vid] += 1
    if not voxels:
        return np.zeros((0, max_points, F), np.float32), np.zeros((0, 3), np.int32), np.zeros((0,), np.int32)
    return np.stack(voxels), np.asarray(coords, np.int32), np.asarray(num, np.int32)
