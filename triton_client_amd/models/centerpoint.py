"""CenterPoint-PointPillars, nuScenes (det3d topology).

Reference: ``data/nusc_centerpoint_pp_02voxel_two_pfn_10sweep.py:24-56``
(model) and ``:69-81`` (test config).  The reference client voxelises with
det3d's ``VoxelGenerator`` (``clients/preprocess/voxelize.py:11-49``).  Its
Detection3DArray branch reads 9-d boxes with yaw at index 8
(``communicator/ros_inference3d.py:179-205``).  The network itself ran behind
a server that is not in the repository.

Stages and where they run here:

* PillarFeatureNet, two PFN layers [64, 64] over 10-d point features: x, y, z,
  r, t, the offset to the pillar mean, and the x/y offset to the pillar centre.
  Layer 1 is Linear(10→32)+BN+ReLU, then concat with the pillar max (64).
  Layer 2 is Linear(64→64)+BN+ReLU, then max over points.
  HIP kernel K8b ``pfn2`` (``csrc/kernels/centerpoint.hip``, MFMA); the
  module below is the fp32 definition.
* PointPillarsScatter: fused into the PFN kernel's epilogue (NHWC canvas).
* RPN neck (3 down blocks, deblocks with strides 0.5 / 1 / 2, concat 384).
  :class:`~.pointpillars.BEVBackbone` with ``up_strides=(0.5, 1, 2)``.
* CenterHead: a shared 3×3 conv 384→64, then per task a SepHead.  Each of its
  heads (reg 2, height 1, dim 3, rot 2, vel 2, hm num_classes) is
  conv3×3(64→64)+BN+ReLU then conv3×3(64→out).
* Decode: K12 (``centerhead_decode``), then per-task top-1000, rotated BEV
  NMS at 0.2, keep 83.

Box layout of the outputs (det3d, nuScenes): ``x, y, z, w, l, h, vx, vy,
yaw`` with ``w`` along x and ``l`` along y (the BEV IoU uses
``[0, 1, 2, 3, 4, 5, 8]``).  Labels are 0-based global class indices
(``data/nuScenes.names``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config.lidar import CenterPointConfig, VoxelConfig
from .common import ConvBNAct, kaiming_init
from .pointpillars import BEVBackbone, scatter_to_bev

HEAD_ORDER = ("reg", "height", "dim", "rot", "vel")  # channel order of a task's merged output (then hm)


def pfn_point_features(voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor,
                       vcfg: VoxelConfig) -> torch.Tensor:
    """[V, P, 5] voxels (x, y, z, r, t) → [V, P, 10] det3d PillarFeatureNet
    features (points, cluster offset xyz, centre offset xy), padded slots zero."""
    vx, vy = vcfg.voxel_size[0], vcfg.voxel_size[1]
    r = vcfg.point_cloud_range
    pts = voxels[:, :, :5] if voxels.shape[-1] >= 5 else F.pad(voxels, (0, 5 - voxels.shape[-1]))
    xyz = pts[:, :, :3]
    n = num_points.clamp(min=1).to(pts.dtype).view(-1, 1, 1)
    f_cluster = xyz - xyz.sum(dim=1, keepdim=True) / n
    c = coords.to(pts.dtype)
    f_center = torch.stack((xyz[:, :, 0] - (c[:, 3:4] * vx + (vx / 2 + r[0])),
                            xyz[:, :, 1] - (c[:, 2:3] * vy + (vy / 2 + r[1]))), dim=-1)
    f = torch.cat([pts, f_cluster, f_center], dim=-1)
    P = pts.shape[1]
    mask = (torch.arange(P, device=pts.device).view(1, -1) < num_points.view(-1, 1)).to(f.dtype)
    return f * mask.unsqueeze(-1)


class PFNLayer(nn.Module):
    def __init__(self, c_in: int, c_out: int, last: bool):
        super().__init__()
        self.last = last
        self.units = c_out if last else c_out // 2
        self.linear = nn.Linear(c_in, self.units, bias=False)
        self.norm = nn.BatchNorm1d(self.units, eps=1e-3, momentum=0.01)
        self.fused_weight = None
        self.fused_bias = None

    @torch.no_grad()
    def fuse_bn(self) -> None:
        if self.fused_weight is not None:  # idempotent: a shared model is fused (fp32) once
            return
        s = self.norm.weight / torch.sqrt(self.norm.running_var + self.norm.eps)
        self.fused_weight = (self.linear.weight * s.view(-1, 1)).detach().clone()
        self.fused_bias = (self.norm.bias - self.norm.running_mean * s).detach().clone()

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # [V, P, c_in]
        if self.fused_weight is not None:
            y = F.relu(x @ self.fused_weight.t().to(x.dtype) + self.fused_bias.to(x.dtype))
        else:
            y = F.relu(self.norm(self.linear(x).permute(0, 2, 1)).permute(0, 2, 1))
        m = y.max(dim=1, keepdim=True).values
        if self.last:
            return m.squeeze(1)
        return torch.cat([y, m.expand_as(y)], dim=-1)


class PillarFeatureNet(nn.Module):
    def __init__(self, filters=(64, 64), c_in: int = 10):
        super().__init__()
        chans = [c_in] + list(filters)
        self.layers = nn.ModuleList(PFNLayer(chans[i], chans[i + 1], i == len(filters) - 1)
                                    for i in range(len(filters)))

    def fuse_bn(self) -> None:
        for lyr in self.layers:
            lyr.fuse_bn()

    def forward(self, feats: torch.Tensor) -> torch.Tensor:  # [V, P, 10] → [V, C]
        x = feats
        for lyr in self.layers:
            x = lyr(x)
        return x


class SepHead(nn.Module):
    """det3d SepHead: per output head, (num_conv-1) × conv3x3+BN+ReLU, then a conv3x3."""

    def __init__(self, c_in: int, heads: Dict[str, int], head_conv: int = 64, final_kernel: int = 3):
        super().__init__()
        self.names = list(heads)
        self.pre = nn.ModuleDict()
        self.out = nn.ModuleDict()
        for name, c in heads.items():
            self.pre[name] = ConvBNAct(c_in, head_conv, final_kernel, 1, final_kernel // 2, act="relu")
            self.out[name] = nn.Conv2d(head_conv, c, final_kernel, 1, final_kernel // 2, bias=True)

    def forward(self, x):
        return {n: self.out[n](self.pre[n](x)) for n in self.names}


class CenterHead(nn.Module):
    def __init__(self, cfg: CenterPointConfig, c_in: int):
        super().__init__()
        self.cfg = cfg
        self.shared = ConvBNAct(c_in, cfg.share_conv, 3, 1, 1, act="relu")
        self.tasks = nn.ModuleList()
        for t in cfg.tasks:
            heads = dict(cfg.common_heads)
            heads["hm"] = len(t.class_names)
            self.tasks.append(SepHead(cfg.share_conv, heads, cfg.head_conv))

    def forward(self, x) -> List[Dict[str, torch.Tensor]]:
        x = self.shared(x)
        return [t(x) for t in self.tasks]


class CenterPoint(nn.Module):
    def __init__(self, cfg: CenterPointConfig | None = None):
        super().__init__()
        cfg = cfg or CenterPointConfig()
        self.cfg = cfg
        self.pfn = PillarFeatureNet(cfg.pfn_filters, 10)
        self.backbone = BEVBackbone(cfg.pfn_filters[-1], cfg.layer_nums, cfg.ds_strides, cfg.ds_filters,
                                    cfg.us_strides, cfg.us_filters)
        self.head = CenterHead(cfg, self.backbone.out_channels)
        kaiming_init(self)
        for t in self.head.tasks:  # det3d init: heatmap prior -2.19, other final convs default
            nn.init.constant_(t.out["hm"].bias, -2.19)

    def fuse_bn(self) -> None:
        self.pfn.fuse_bn()

    def bev_forward(self, canvas: torch.Tensor) -> List[Dict[str, torch.Tensor]]:
        return self.head(self.backbone(canvas))

    def forward(self, voxels, num_points, coords, batch_size: int):
        f = pfn_point_features(voxels, num_points, coords, self.cfg.voxel)
        pf = self.pfn(f)
        nx, ny, _ = self.cfg.voxel.grid_size
        canvas = scatter_to_bev(pf, coords, batch_size, ny, nx, channels_last=True)
        return self.bev_forward(canvas)


def build_centerpoint(cfg: CenterPointConfig | None = None, seed: int = 0) -> CenterPoint:
    torch.manual_seed(seed)
    return CenterPoint(cfg)


def merged_task_outputs(preds: List[Dict[str, torch.Tensor]]) -> List[torch.Tensor]:
    """Per task: [B, 10 + nc, H, W] in HEAD_ORDER then hm (the merged layout the
    fast plan and the decode kernel use)."""
    return [torch.cat([p[n] for n in HEAD_ORDER] + [p["hm"]], dim=1) for p in preds]


def decode_reference(task_out: List[torch.Tensor], cfg: CenterPointConfig, class_offsets: List[int],
                     class_thresh=None):
    """fp32 det3d decode of merged task outputs → per image list of
    (boxes [N, 9] det3d order, scores [N], labels [N]) after score / centre-range
    filter, top nms_pre_max, rotated NMS, keep nms_post_max.  CPU reference.
    ``class_thresh``: optional per-global-class score thresholds (K13)."""
    import numpy as np

    from ..ops.nms import sort_and_nms_cpu

    r = cfg.voxel.point_cloud_range
    vx, vy = cfg.voxel.voxel_size[0], cfg.voxel.voxel_size[1]
    osf = cfg.out_size_factor
    pcr = cfg.post_center_range
    B = task_out[0].shape[0]
    out = []
    for b in range(B):
        boxes_all, scores_all, labels_all = [], [], []
        for t, o in enumerate(task_out):
            o = o[b].float()
            C, H, W = o.shape
            ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                                    indexing="ij")
            reg, hei, dim, rot, vel, hm = o[0:2], o[2:3], o[3:6], o[6:8], o[8:10], o[10:]
            score, lab = torch.sigmoid(hm).max(0)
            x = (xs + reg[0]) * osf * vx + r[0]
            y = (ys + reg[1]) * osf * vy + r[1]
            yaw = torch.atan2(rot[0], rot[1])
            d = torch.exp(dim)
            box = torch.stack([x, y, hei[0], d[0], d[1], d[2], vel[0], vel[1], yaw], -1).reshape(-1, 9)
            s = score.reshape(-1)
            lb = lab.reshape(-1)
            thr = torch.full_like(s, cfg.score_thresh)
            if class_thresh is not None:
                tab = torch.tensor([max(cfg.score_thresh, v) for v in class_thresh], dtype=torch.float32)
                thr = tab[(lb + class_offsets[t]).clamp(max=len(tab) - 1)]
            keep = (s > thr)
            keep &= (box[:, 0] >= pcr[0]) & (box[:, 1] >= pcr[1]) & (box[:, 2] >= pcr[2])
            keep &= (box[:, 0] <= pcr[3]) & (box[:, 1] <= pcr[4]) & (box[:, 2] <= pcr[5])
            idx = torch.nonzero(keep).flatten().numpy()
            if len(idx) == 0:
                continue
            bx = box[idx].numpy()
            nms_box = bx[:, [0, 1, 2, 3, 4, 5, 8]]
            kept = sort_and_nms_cpu(nms_box, s[idx].numpy(), np.zeros(len(idx), np.int32), idx, 1, cfg.nms_iou,
                                    cfg.nms_pre_max, cfg.nms_post_max, True)
            boxes_all.append(bx[kept])
            scores_all.append(s[idx].numpy()[kept])
            labels_all.append(lb[idx].numpy()[kept] + class_offsets[t])
        if boxes_all:
            out.append((np.concatenate(boxes_all), np.concatenate(scores_all), np.concatenate(labels_all)))
        else:
            out.append((np.zeros((0, 9), np.float32), np.zeros((0,), np.float32), np.zeros((0,), np.int64)))
    return out
