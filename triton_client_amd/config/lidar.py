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
class SparseConvSpec:
    """One layer of the VoxelBackBone8x sparse 3D CNN (OpenPCDet
    ``backbones_3d/spconv_backbone.py``, named by ``second_iou.yaml:13-14``):
    ``subm`` = SubMConv3d (output sites = input sites, 3x3x3, pad 1);
    otherwise SparseConv3d with per-(z, y, x) kernel / stride / padding.
    Every layer is conv (no bias) + BatchNorm1d(eps 1e-3) + ReLU."""
    cin: int
    cout: int
    subm: bool = True
    kernel: Tuple[int, int, int] = (3, 3, 3)
    stride: Tuple[int, int, int] = (1, 1, 1)
    padding: Tuple[int, int, int] = (1, 1, 1)

    @property
    def taps(self) -> int:
        return self.kernel[0] * self.kernel[1] * self.kernel[2]


def voxel_backbone_8x(c_in: int = 4) -> Tuple[SparseConvSpec, ...]:
    """VoxelBackBone8x: conv_input + conv1 at 1x, conv2 at 2x, conv3 at 4x,
    conv4 at 8x (z padding 0), conv_out (3,1,1)/(2,1,1): 16, 16, 32, 64, 64,
    128 channels."""
    S = SparseConvSpec
    return (
        S(c_in, 16), S(16, 16),                                                       # conv_input, conv1
        S(16, 32, False, stride=(2, 2, 2)), S(32, 32), S(32, 32),                       # conv2
        S(32, 64, False, stride=(2, 2, 2)), S(64, 64), S(64, 64),                       # conv3
        S(64, 64, False, stride=(2, 2, 2), padding=(0, 1, 1)), S(64, 64), S(64, 64),    # conv4
        S(64, 128, False, kernel=(3, 1, 1), stride=(2, 1, 1), padding=(0, 0, 0)),       # conv_out
    )


@dataclass
class SecondIoUConfig(PointPillarsConfig):
    """OpenPCDet SECONDNetIoU (reference ``examples/second_iou/1/second_iou.yaml``)
    on the client's KITTI voxels (``data/kitti_dataset.yaml:4,64-70``):
    MeanVFE → VoxelBackBone8x → HeightCompression (256) → BaseBEVBackbone
    [5,5] / [1,2] / [128,256] / up [1,2] / [256,256] → AnchorHeadSingle
    (stride 8) → proposal NMS (pre 1024, post 100, IoU 0.7) → SECONDHead
    (7x7 RoI grid pool on the 512-channel BEV map, shared FC [256,256], IoU FC
    [256,256]) → rotated NMS on sigmoid(IoU) (score 0.1, IoU 0.01, 4096 → 500)."""
    voxel: VoxelConfig = field(default_factory=lambda: KITTI_SECOND_VOXELS)
    sparse: Tuple[SparseConvSpec, ...] = field(default_factory=voxel_backbone_8x)  # second_iou.yaml:13-14
    bev_features: int = 256  # :16-18 (HeightCompression: 128 channels x 2 z-levels)
    layer_nums: Tuple[int, ...] = (5, 5)  # :20-27
    layer_strides: Tuple[int, ...] = (1, 2)
    num_filters: Tuple[int, ...] = (128, 256)
    upsample_strides: Tuple[float, ...] = (1, 2)
    num_upsample_filters: Tuple[int, ...] = (256, 256)
    feature_map_stride: int = 8  # :45
    # ROI_HEAD (:87-112)
    roi_grid: int = 7
    roi_shared_fc: Tuple[int, ...] = (256, 256)
    roi_iou_fc: Tuple[int, ...] = (256, 256)
    proposal_nms_thresh: float = 0.7
    proposal_pre_max: int = 1024
    proposal_post_max: int = 100
    # POST_PROCESSING (:136-148) = the inherited score 0.1, NMS 0.01, 4096 → 500

    @property
    def sparse_shape(self) -> Tuple[int, int, int]:
        """spconv input shape (z, y, x) = grid[::-1] + [1, 0, 0]."""
        nx, ny, nz = self.voxel.grid_size
        return nz + 1, ny, nx

    def level_shapes(self) -> List[Tuple[int, int, int]]:
        """(z, y, x) shape of the input and of every sparse layer's output."""
        shp = [self.sparse_shape]
        for s in self.sparse:
            z = shp[-1]
            shp.append(z if s.subm else
                       tuple((z[d] + 2 * s.padding[d] - s.kernel[d]) // s.stride[d] + 1 for d in range(3)))
        return shp

    @property
    def bev_shape(self) -> Tuple[int, int, int]:
        """(channels, ny, nx) of HeightCompression's output."""
        z, y, x = self.level_shapes()[-1]
        return self.sparse[-1].cout * z, y, x

    @property
    def feature_map_size(self) -> Tuple[int, int]:
        _, y, x = self.bev_shape
        s = self.layer_strides[0]
        return y // s, x // s


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
