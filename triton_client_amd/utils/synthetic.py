"""Synthetic sensors (no datasets are reachable): a camera producing uint8
RGB frames and a spinning LiDAR producing PointCloud2-style byte payloads.

The LiDAR is a vectorised ray caster: ``rings`` beams (HDL-64-like elevation
fan) x ``azimuth_steps`` columns against a ground plane and a handful of
box-shaped obstacles (cars/pedestrians), with range noise, random dropouts
(NaN returns — the reference skips them with ``skip_nans=True``) and an
intensity channel.  64 x 1875 ≈ 120k points per sweep, 16 B per point
(x, y, z, intensity float32) — the KITTI velodyne layout.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np


@dataclass
class LidarSpec:
    rings: int = 64
    azimuth_steps: int = 1875
    elev_min_deg: float = -24.9
    elev_max_deg: float = 2.0
    max_range: float = 90.0
    sensor_height: float = 1.73  # ground at z = -sensor_height in the sensor frame
    dropout: float = 0.02
    n_objects: int = 24
    point_step: int = 16

    @property
    def points_per_sweep(self) -> int:
        return self.rings * self.azimuth_steps


def lidar_sweep(spec: LidarSpec, seed: int = 0) -> np.ndarray:
    """Returns [N, 4] float32 (x, y, z, intensity); NaN rows for dropouts."""
    rng = np.random.default_rng(seed)
    el = np.deg2rad(np.linspace(spec.elev_min_deg, spec.elev_max_deg, spec.rings))
    az = np.linspace(-np.pi, np.pi, spec.azimuth_steps, endpoint=False) + rng.uniform(0, 2 * np.pi / spec.azimuth_steps)
    E, A = np.meshgrid(el, az, indexing="ij")
    d = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], -1).reshape(-1, 3)
    t = np.full(d.shape[0], np.inf)
    # ground plane z = -h
    down = d[:, 2] < -1e-6
    t[down] = -spec.sensor_height / d[down, 2]
    # axis-aligned box obstacles (slab test)
    for _ in range(spec.n_objects):
        r = rng.uniform(4, 60)
        th = rng.uniform(-np.pi, np.pi)
        c = np.array([r * np.cos(th), r * np.sin(th), 0.0])
        if rng.random() < 0.7:
            size = np.array([rng.uniform(3.5, 4.8), rng.uniform(1.5, 2.0), rng.uniform(1.4, 1.8)])
        else:
            size = np.array([rng.uniform(0.5, 0.9), rng.uniform(0.5, 0.9), rng.uniform(1.5, 1.9)])
        lo = c - size / 2
        lo[2] = -spec.sensor_height
        hi = lo + size
        with np.errstate(divide="ignore", invalid="ignore"):
            t1 = (lo[None] - 0) / d
            t2 = (hi[None] - 0) / d
        tmin = np.nanmax(np.minimum(t1, t2), 1)
        tmax = np.nanmin(np.maximum(t1, t2), 1)
        hit = (tmax >= tmin) & (tmin > 0)
        t = np.where(hit & (tmin < t), tmin, t)
    t = t + rng.normal(0, 0.02, t.shape)
    valid = np.isfinite(t) & (t < spec.max_range)
    pts = d * t[:, None]
    inten = np.clip(rng.normal(0.3, 0.15, t.shape) * 255.0, 0, 255)
    out = np.concatenate([pts, inten[:, None]], 1).astype(np.float32)
    drop = (~valid) | (rng.random(t.shape) < spec.dropout)
    out[drop] = np.nan
    return out


def camera_frame(h: int, w: int, seed: int = 0) -> np.ndarray:
    """A cheap structured RGB frame: gradient background + random rectangles."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)),
                    ((xx + yy) * 127 // max(h + w - 2, 1))], -1).astype(np.uint8)
    for _ in range(12):
        x0, y0 = rng.integers(0, w - 8), rng.integers(0, h - 8)
        x1, y1 = min(w, x0 + rng.integers(8, w // 3)), min(h, y0 + rng.integers(8, h // 3))
        img[y0:y1, x0:x1] = rng.integers(0, 256, 3, dtype=np.uint8)
    noise = rng.integers(0, 16, img.shape, dtype=np.uint8)
    return img + noise


def sensor_batch(n: int, cam_hw: Tuple[int, int], lidar: LidarSpec, seed: int = 0):
    """n (camera frame, lidar sweep) pairs."""
    cams = np.stack([camera_frame(cam_hw[0], cam_hw[1], seed + i) for i in range(n)])
    clouds: List[np.ndarray] = [lidar_sweep(lidar, seed + 1000 + i) for i in range(n)]
    return cams, clouds
