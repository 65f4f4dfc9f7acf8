"""Typed configuration for the LiDAR pipelines.

The numbers are the reference's (cited per field) so that they are *data*,
not code: PointPillars/KITTI (``data/pointpillar.yaml``), the SECOND-style
client voxeliser (``data/kitti_dataset.yaml``), and CenterPoint-PointPillars
on nuScenes (``data/nusc_centerpoint_pp_02voxel_two_pfn_10sweep.py``).
``from_openpcdet_yaml`` reads an OpenPCDet model YAML so a user can point the
pipeline at their own config file.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import yaml


@dataclass
class VoxelConfig:
    """Point → voxel parameters (spconv ``VoxelGenerator`` semantics)."""
    point_cloud_range: Tuple[float, float, float, float, float, float]
    voxel_size: Tuple[float, float, float]
    max_points_per_voxel: int
    max_voxels: int
    num_point_features: int = 4  # x, y, z, intensity (+ time lag for nuScenes)

    @property
    def grid_size(self) -> Tuple[int, int, int]:
        """(nx, ny, nz), rounded like OpenPCDet/spconv."""
        r, v = self.point_cloud_range, self.voxel_size
        return tuple(int(round((r[i + 3] - r[i]) / v[i])) for i in range(3))  # type: ignore

    @property
    def num_cells(self) -> int:
        nx, ny, nz = self.grid_size
        return nx * ny * nz


# SECOND-style client voxeliser: data/kitti_dataset.yaml:4 (range), :64-70 (voxel/limits)
KITTI_SECOND_VOXELS = VoxelConfig((0.0, -40.0, -3.0, 70.4, 40.0, 1.0), (0.05, 0.05, 0.1), 5, 40000, 4)
# PointPillars: data/pointpillar.yaml:5 (range), :16-22 (voxel/limits)
KITTI_PILLARS = VoxelConfig((0.0, -39.68, -3.0, 69.12, 39.68, 1.0), (0.16, 0.16, 4.0), 32, 40000, 4)
# CenterPoint-PP nuScenes: nusc_…py:138-143 (generator), clients/preprocess/voxelize.py:19-24 (20000 voxels)
NUSC_PILLARS = VoxelConfig((-51.2, -51.2, -5.0, 51.2, 51.2, 3.0), (0.2, 0.2, 8.0), 20, 20000, 5)


@dataclass
class AnchorClass:
    name: str
    size: Tuple[float, float, float]  # dx, dy, dz (l, w, h)
    rotations: Tuple[float, ...]
    bottom_height: float


@dataclass
class PointPillarsConfig:
    """OpenPCDet PointPillar (data/pointpillar.yaml:50-142)."""
    voxel: VoxelConfig = field(default_factory=lambda: KITTI_PILLARS)
    class_names: Tuple[str, ...] = ("Car", "Pedestrian", "Cyclist")  # pointpillar.yaml:1
    vfe_filters: int = 64  # :53-58
    bev_features: int = 64  # :60-62
    layer_nums: Tuple[int, ...] = (3, 5, 5)  # :64-70
    layer_strides: Tuple[int, ...] = (2, 2, 2)
    num_filters: Tuple[int, ...] = (64, 128, 256)
    upsample_strides: Tuple[float, ...] = (1, 2, 4)
    num_upsample_filters: Tuple[int, ...] = (128, 128, 128)
    anchors: Tuple[AnchorClass, ...] = (  # :84-112
        AnchorClass("Car", (3.9, 1.6, 1.56), (0.0, 1.57), -1.78),
        AnchorClass("Pedestrian", (0.8, 0.6, 1.73), (0.0, 1.57), -0.6),
        AnchorClass("Cyclist", (1.76, 0.6, 1.73), (0.0, 1.57), -0.6),
    )
    feature_map_stride: int = 2
    dir_offset: float = 0.78539  # :77
    dir_limit_offset: float = 0.0
    num_dir_bins: int = 2
    score_thresh: float = 0.1  # :132
    nms_thresh: float = 0.01  # :139
    nms_pre_max: int = 4096  # :140
    nms_post_max: int = 500  # :141

    @property
    def num_anchors_per_loc(self) -> int:
        return sum(len(a.rotations) for a in self.anchors)

    @property
    def num_classes(self) -> int:
        return len(self.class_names)

    @property
    def feature_map_size(self) -> Tuple[int, int]:
        """(ny, nx) of the head feature map."""
        nx, ny, _ = self.voxel.grid_size
        return ny // self.feature_map_stride, nx // self.feature_map_stride

    @staticmethod
    def from_openpcdet_yaml(path: str) -> "PointPillarsConfig":
        with open(path) as f:
            y = yaml.safe_load(f)
        cfg = PointPillarsConfig()
        dc = y.get("DATA_CONFIG", {})
        rng = dc.get("POINT_CLOUD_RANGE")
        vox = None
        for p in dc.get("DATA_PROCESSOR", []):
            if p.get("NAME") == "transform_points_to_voxels":
                vox = p
        if rng is not None and vox is not None:
            mv = vox["MAX_NUMBER_OF_VOXELS"]
            mv = mv.get("test", mv) if isinstance(mv, dict) else mv
            cfg.voxel = VoxelConfig(tuple(rng), tuple(vox["VOXEL_SIZE"]), int(vox["MAX_POINTS_PER_VOXEL"]), int(mv), 4)
        m = y.get("MODEL", {})
        if "CLASS_NAMES" in y:
            cfg.class_names = tuple(y["CLASS_NAMES"])
        bb = m.get("BACKBONE_2D", {})
        if bb:
            cfg.layer_nums = tuple(bb["LAYER_NUMS"])
            cfg.layer_strides = tuple(bb["LAYER_STRIDES"])
            cfg.num_filters = tuple(bb["NUM_FILTERS"])
            cfg.upsample_strides = tuple(bb["UPSAMPLE_STRIDES"])
            cfg.num_upsample_filters = tuple(bb["NUM_UPSAMPLE_FILTERS"])
        dh = m.get("DENSE_HEAD", {})
        if dh:
            cfg.dir_offset = float(dh.get("DIR_OFFSET", cfg.dir_offset))
            cfg.dir_limit_offset = float(dh.get("DIR_LIMIT_OFFSET", cfg.dir_limit_offset))
            cfg.num_dir_bins = int(dh.get("NUM_DIR_BINS", cfg.num_dir_bins))
            ags = dh.get("ANCHOR_GENERATOR_CONFIG")
            if ags:
                cfg.anchors = tuple(AnchorClass(a["class_name"], tuple(a["anchor_sizes"][0]),
                                                tuple(a["anchor_rotations"]), float(a["anchor_bottom_heights"][0]))
                                    for a in ags)
                cfg.feature_map_stride = int(ags[0].get("feature_map_stride", 2))
        pp = m.get("POST_PROCESSING", {})
        if pp:
            cfg.score_thresh = float(pp.get("SCORE_THRESH", cfg.score_thresh))
            nms = pp.get("NMS_CONFIG", {})
            cfg.nms_thresh = float(nms.get("NMS_THRESH", cfg.nms_thresh))
            cfg.nms_pre_max = int(nms.get("NMS_PRE_MAXSIZE", cfg.nms_pre_max))
            cfg.nms_post_max = int(nms.get("NMS_POST_MAXSIZE", cfg.nms_post_max))
        return cfg


@dataclass
class CenterPointTask:
    class_names: Tuple[str, ...]


@dataclass
class CenterPointConfig:
    """det3d CenterPoint-PointPillars (nusc_centerpoint_pp_02voxel_two_pfn_10sweep.py)."""
    voxel: VoxelConfig = field(default_factory=lambda: NUSC_PILLARS)
    tasks: Tuple[CenterPointTask, ...] = (  # :6-13
        CenterPointTask(("car",)),
        CenterPointTask(("truck", "construction_vehicle")),
        CenterPointTask(("bus", "trailer")),
        CenterPointTask(("barrier",)),
        CenterPointTask(("motorcycle", "bicycle")),
        CenterPointTask(("pedestrian", "traffic_cone")),
    )
    pfn_filters: Tuple[int, ...] = (64, 64)  # :27-34
    layer_nums: Tuple[int, ...] = (3, 5, 5)  # :36-45
    ds_strides: Tuple[int, ...] = (2, 2, 2)
    ds_filters: Tuple[int, ...] = (64, 128, 256)
    us_strides: Tuple[float, ...] = (0.5, 1, 2)
    us_filters: Tuple[int, ...] = (128, 128, 128)
    share_conv: int = 64
    head_conv: int = 64
    common_heads: Tuple[Tuple[str, int], ...] = (("reg", 2), ("height", 1), ("dim", 3), ("rot", 2), ("vel", 2))
    out_size_factor: int = 4
    post_center_range: Tuple[float, ...] = (-61.2, -61.2, -10.0, 61.2, 61.2, 10.0)  # :70
    score_thresh: float = 0.1  # :78
    nms_iou: float = 0.2  # :75
    nms_pre_max: int = 1000  # :73
    nms_post_max: int = 83  # :74

    @property
    def class_names(self) -> List[str]:
        return [c for t in self.tasks for c in t.class_names]

    @property
    def feature_map_size(self) -> Tuple[int, int]:
        nx, ny, _ = self.voxel.grid_size
        return ny // self.out_size_factor, nx // self.out_size_factor


def anchor_grid(cfg: PointPillarsConfig):
    """Analytic anchor layout (OpenPCDet AnchorGenerator, align_center=False).

    Returns (x0, dx, y0, dy, per-anchor table [A, 7 + 1(rotation)]).  Anchor
    index order is (y, x, class, rotation) — the same order the head's
    ``[B, H, W, A*C]`` permute produces.  Anchors are never materialised on
    the GPU; the decode kernel evaluates them from this table.
    """
    r = cfg.voxel.point_cloud_range
    ny, nx = cfg.feature_map_size
    x_stride = (r[3] - r[0]) / (nx - 1)
    y_stride = (r[4] - r[1]) / (ny - 1)
    table = []
    for a in cfg.anchors:
        for rot in a.rotations:
            dxa, dya, dza = a.size
            table.append((dxa, dya, dza, a.bottom_height + dza / 2.0, rot, math.sqrt(dxa * dxa + dya * dya)))
    return r[0], x_stride, r[1], y_stride, table
