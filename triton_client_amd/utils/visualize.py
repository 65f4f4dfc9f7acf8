"""Headless 3D visualisation (reference ``clients/postprocess/visualize_open3d.py``,
``visualize_mayavi.py`` — Open3D / Mayavi are not available here and a
production client has no display).

* :func:`rotate_points_along_z`, :func:`boxes_to_corners_3d` — same geometry as
  the reference's Mayavi helpers (``visualize_mayavi.py:19-69``): 8 corners of
  (x, y, z, dx, dy, dz, heading) boxes;
* :func:`render_bev` — bird's-eye-view PNG of a point cloud with predicted and
  ground-truth boxes (NumPy raster + PIL), for bag replay inspection where the
  reference used rviz / Open3D windows;
* :func:`draw_scenes` — the reference's ``draw_scenes`` (Open3D / Mayavi 3D
  view: cloud, origin axes, ground truth and predictions coloured by label)
  rendered headless through a pinhole camera;
* :func:`project_boxes_to_image` — the corners view (Mayavi ``draw_corners3d``)
  drawn into a camera image with a LiDAR->camera transform.
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


# ----------------------------------------------------------------------------- 3D scene
# Reference draw_scenes (visualize_open3d.py:38-80, visualize_mayavi.py:142-200):
# an interactive window with the cloud, an origin frame, ground-truth boxes in blue
# and predictions coloured by label.  Here the same scene is rendered headless
# through a pinhole camera into an image (painter's order, far points first).

BOX_COLORS = np.array([[255, 255, 255], [0, 255, 0], [0, 255, 255], [255, 255, 0], [255, 128, 0],
                       [255, 0, 255], [128, 128, 255], [255, 96, 96], [160, 255, 160], [96, 160, 255]], np.uint8)
# the 12 edges of boxes_to_corners_3d's corner order (bottom 0-3, top 4-7)
BOX_EDGES = ((0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6), (3, 7))


def label_colors(labels: np.ndarray) -> np.ndarray:
    """Per-point / per-box RGB from integer labels (reference get_coor_colors)."""
    return BOX_COLORS[np.asarray(labels, np.int64) % len(BOX_COLORS)]


def look_at(eye: Sequence[float], target: Sequence[float], up: Sequence[float] = (0.0, 0.0, 1.0)) -> np.ndarray:
    """World -> camera rotation-translation [3, 4] (camera looks along +z, y down)."""
    eye, target, up = (np.asarray(v, np.float64) for v in (eye, target, up))
    f = target - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    R = np.stack([r, d, f])
    return np.concatenate([R, -(R @ eye)[:, None]], 1)


def project(pts: np.ndarray, Rt: np.ndarray, K: np.ndarray):
    """World points [N, 3] -> (pixel [N, 2], depth [N])."""
    cam = pts @ Rt[:, :3].T + Rt[:, 3]
    z = cam[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        uv = (cam @ K.T)[:, :2] / z[:, None]
    return uv, z


def draw_box_edges(img: np.ndarray, corners: np.ndarray, Rt: np.ndarray, K: np.ndarray, color, near: float = 0.1):
    """Wireframes of boxes given as corners [M, 8, 3]; edges behind the camera
    are clipped at the near plane; the heading face (0-1-5-4) is marked."""
    for cor in corners:
        cam = cor @ Rt[:, :3].T + Rt[:, 3]
        for k, (i, j) in enumerate(BOX_EDGES):
            a, b = cam[i].copy(), cam[j].copy()
            if a[2] < near and b[2] < near:
                continue
            if a[2] < near or b[2] < near:  # clip to the near plane
                t = (near - a[2]) / (b[2] - a[2])
                p = a + t * (b - a)
                a, b = (p, b) if a[2] < near else (a, p)
            ua, ub = K @ a, K @ b
            _line(img, ua[0] / ua[2], ua[1] / ua[2], ub[0] / ub[2], ub[1] / ub[2],
                  (255, 80, 40) if k in (0, 8, 9) else color)
    # a diagonal across the heading face (reference draw_corners3d marks it too)
    for cor in corners:
        uv, z = project(cor[[0, 5]], Rt, K)
        if (z > near).all():
            _line(img, uv[0, 0], uv[0, 1], uv[1, 0], uv[1, 1], (255, 80, 40))


def draw_scenes(points: np.ndarray, gt_boxes: Optional[np.ndarray] = None, ref_boxes: Optional[np.ndarray] = None,
                ref_labels: Optional[np.ndarray] = None, ref_scores: Optional[np.ndarray] = None,
                point_colors: Optional[np.ndarray] = None, draw_origin: bool = True,
                eye: Sequence[float] = (-12.0, 0.0, 14.0), target: Sequence[float] = (22.0, 0.0, 0.0),
                size: Tuple[int, int] = (720, 1280), fov_deg: float = 70.0, score_thresh: float = 0.0,
                path: Optional[str] = None) -> np.ndarray:
    """Headless equivalent of the reference's draw_scenes: points (grey by
    height, or ``point_colors`` [N, 3] uint8 / labels), ground truth in blue,
    predictions coloured by label (heading edges orange), origin axes (x red,
    y green, z blue).  Boxes: [M, 7] (x, y, z, dx, dy, dz, heading) or det3d
    [M, 9] (yaw at index 8).  Returns the HxWx3 uint8 image (saved to ``path``)."""
    H, W = size
    fpx = 0.5 * W / np.tan(np.radians(fov_deg) / 2)
    K = np.array([[fpx, 0, W / 2], [0, fpx, H / 2], [0, 0, 1]], np.float64)
    Rt = look_at(eye, target)
    img = np.zeros((H, W, 3), np.uint8)
    if points is not None and len(points):
        p = np.asarray(points, np.float64)
        uv, z = project(p[:, :3], Rt, K)
        ok = (z > 0.1) & (uv[:, 0] >= 0) & (uv[:, 0] < W) & (uv[:, 1] >= 0) & (uv[:, 1] < H)
        if point_colors is not None:
            pc = np.asarray(point_colors)
            col = label_colors(pc) if pc.ndim == 1 else pc.astype(np.uint8)
        else:
            zz = p[:, 2]
            g = np.clip((zz - zz.min()) / max(np.ptp(zz), 1e-6) * 200 + 55, 0, 255).astype(np.uint8)
            col = np.stack([g, g, g], -1)
        idx = np.nonzero(ok)[0]
        idx = idx[np.argsort(-z[idx], kind="stable")]  # far first: near points win
        img[uv[idx, 1].astype(int), uv[idx, 0].astype(int)] = col[idx]
    if draw_origin:
        o = np.zeros(3)
        for axis, color in ((np.array([1.0, 0, 0]), (255, 0, 0)), (np.array([0, 1.0, 0]), (0, 255, 0)),
                            (np.array([0, 0, 1.0]), (0, 0, 255))):
            uv, z = project(np.stack([o, axis * 2.0]), Rt, K)
            if (z > 0.1).all():
                _line(img, uv[0, 0], uv[0, 1], uv[1, 0], uv[1, 1], color)

    def as7(b):
        b = np.asarray(b, np.float64).reshape(-1, np.shape(b)[-1] if len(np.shape(b)) > 1 else 7)
        return b[:, [0, 1, 2, 3, 4, 5, 8]] if b.shape[1] >= 9 else b[:, :7]

    if gt_boxes is not None and len(gt_boxes):
        draw_box_edges(img, boxes_to_corners_3d(as7(gt_boxes)), Rt, K, (60, 120, 255))
    if ref_boxes is not None and len(ref_boxes):
        rb = as7(ref_boxes)
        keep = np.ones(len(rb), bool) if ref_scores is None else np.asarray(ref_scores) >= score_thresh
        labels = np.ones(len(rb), np.int64) if ref_labels is None else np.asarray(ref_labels, np.int64)
        cors = boxes_to_corners_3d(rb)
        for k in np.nonzero(keep)[0]:
            draw_box_edges(img, cors[k:k + 1], Rt, K, tuple(int(v) for v in label_colors(labels[k:k + 1])[0]))
    if path:
        from PIL import Image
        Image.fromarray(img).save(path)
    return img


def project_boxes_to_image(img: np.ndarray, boxes: np.ndarray, P: np.ndarray, Tr: Optional[np.ndarray] = None,
                           labels: Optional[np.ndarray] = None) -> np.ndarray:
    """Draw 3D boxes (LiDAR frame) onto a camera image: ``Tr`` [3|4, 4] LiDAR ->
    camera (identity if None), ``P`` [3, 3|4] camera projection (KITTI
    P2-style).  The corners view of the reference's Mayavi draw_corners3d, in
    the image instead of a 3D window.  Modifies and returns ``img``."""
    Tr = np.eye(4) if Tr is None else np.vstack([np.asarray(Tr, np.float64)[:3], [0, 0, 0, 1]])
    P = np.asarray(P, np.float64)
    K = P[:, :3]
    Rt = np.linalg.inv(K) @ P if P.shape[1] == 4 else np.concatenate([np.eye(3), np.zeros((3, 1))], 1)
    Rt = (np.vstack([Rt, [0, 0, 0, 1]]) @ Tr)[:3]
    b = np.asarray(boxes, np.float64)
    b = b[:, [0, 1, 2, 3, 4, 5, 8]] if b.shape[1] >= 9 else b[:, :7]
    labels = np.ones(len(b), np.int64) if labels is None else np.asarray(labels)
    cors = boxes_to_corners_3d(b)
    for k in range(len(b)):
        draw_box_edges(img, cors[k:k + 1], Rt, K, tuple(int(v) for v in label_colors(labels[k:k + 1])[0]))
    return img
