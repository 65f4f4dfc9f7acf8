"""Headless 3D visualisation (reference ``clients/postprocess/visualize_open3d.py``,
``visualize_mayavi.py`` — Open3D / Mayavi are not available here and a
production client has no display).

* :func:`rotate_points_along_z`, :func:`boxes_to_corners_3d` — same geometry as
  the reference's Mayavi helpers (``visualize_mayavi.py:19-69``): 8 corners of
  (x, y, z, dx, dy, dz, heading) boxes;
* :func:`render_bev` — bird's-eye-view PNG of a point cloud with predicted and
  ground-truth boxes (NumPy raster + PIL), for bag replay inspection where the
  reference used rviz / Open3D windows.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np


def rotate_points_along_z(points: np.ndarray, angle: np.ndarray) -> np.ndarray:
    """points [B, N, 3+C], angle [B] (rad, counter-clockwise about +z)."""
    c, s = np.cos(angle), np.sin(angle)
    rot = np.stack([np.stack([c, s, np.zeros_like(c)], -1), np.stack([-s, c, np.zeros_like(c)], -1),
                    np.stack([np.zeros_like(c), np.zeros_like(c), np.ones_like(c)], -1)], 1)  # [B,3,3]
    out = points.copy()
    out[..., :3] = points[..., :3] @ rot
    return out


def boxes_to_corners_3d(boxes: np.ndarray) -> np.ndarray:
    """boxes [N, 7+] (x, y, z, dx, dy, dz, heading) → corners [N, 8, 3]
    (order: 4 bottom then 4 top, counter-clockwise from (+x, +y))."""
    boxes = np.asarray(boxes, np.float64).reshape(-1, boxes.shape[-1] if np.ndim(boxes) else 7)
    t = np.array([[1, 1, -1], [1, -1, -1], [-1, -1, -1], [-1, 1, -1],
                  [1, 1, 1], [1, -1, 1], [-1, -1, 1], [-1, 1, 1]], np.float64) / 2
    corners = boxes[:, None, 3:6] * t[None]
    corners = rotate_points_along_z(corners, boxes[:, 6])
    return corners + boxes[:, None, 0:3]


def _line(img, x0, y0, x1, y1, color):
    n = int(max(abs(x1 - x0), abs(y1 - y0))) + 1
    xs = np.clip(np.round(np.linspace(x0, x1, n)).astype(int), 0, img.shape[1] - 1)
    ys = np.clip(np.round(np.linspace(y0, y1, n)).astype(int), 0, img.shape[0] - 1)
    img[ys, xs] = color


def render_bev(points: np.ndarray, boxes: Optional[np.ndarray] = None, gt_boxes: Optional[np.ndarray] = None,
               x_range: Tuple[float, float] = (0.0, 69.12), y_range: Tuple[float, float] = (-39.68, 39.68),
               res: float = 0.1, labels: Optional[Sequence[int]] = None, path: Optional[str] = None) -> np.ndarray:
    """Top-down raster: +x up, +y left (the LiDAR convention).  Points grey by
    height, predicted boxes green (heading edge highlighted), ground truth blue."""
    H = int(round((x_range[1] - x_range[0]) / res))
    W = int(round((y_range[1] - y_range[0]) / res))
    img = np.zeros((H, W, 3), np.uint8)

    def to_px(x, y):
        return (y_range[1] - y) / res, (x_range[1] - x) / res  # col, row

    if points is not None and len(points):
        p = np.asarray(points)
        c, r = to_px(p[:, 0], p[:, 1])
        ok = (r >= 0) & (r < H) & (c >= 0) & (c < W)
        z = p[ok, 2]
        g = np.clip((z - z.min()) / max(np.ptp(z), 1e-6) * 200 + 55, 0, 255).astype(np.uint8) if ok.any() else []
        img[r[ok].astype(int), c[ok].astype(int)] = np.stack([g, g, g], -1) if ok.any() else 0
    for bxs, color in ((gt_boxes, (60, 120, 255)), (boxes, (40, 230, 60))):
        if bxs is None or len(bxs) == 0:
            continue
        b = np.asarray(bxs, np.float64)
        if b.shape[1] >= 9:  # det3d 9-d: yaw at index 8
            b = b[:, [0, 1, 2, 3, 4, 5, 8]]
        for k, cor in enumerate(boxes_to_corners_3d(b)):
            pts = [to_px(cor[i, 0], cor[i, 1]) for i in range(4)]
            for i in range(4):
                (c0, r0), (c1, r1) = pts[i], pts[(i + 1) % 4]
                _line(img, c0, r0, c1, r1, (255, 80, 40) if i == 0 else color)
    if path:
        from PIL import Image
        Image.fromarray(img).save(path)
    return img
