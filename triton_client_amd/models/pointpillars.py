"""PointPillars (OpenPCDet ``PointPillar`` topology) — the LiDAR detector the
reference serves as ``pointpillar_kitti`` through a Triton Python backend
(reference ``examples/pointpillar_kitti/1/model.py:91-186``, config
``data/pointpillar.yaml:50-142``).

Stages and where they run here:

* PillarVFE (10-d point features → Linear 10→64 → BN → ReLU → max over the
  pillar's 32 slots) — fused HIP kernel ``pillar_vfe`` (K8, MFMA 32x32x16 bf16)
  in ``csrc/kernels/pillars.hip``; :class:`PillarVFE` below is the fp32
  PyTorch definition (and CPU path).
* PointPillarScatter — fused into the VFE kernel's epilogue (it writes each
  pillar's feature straight into the NHWC BEV canvas).
* BaseBEVBackbone + AnchorHeadSingle convs — :class:`BEVBackbone` / :class:`AnchorHead`.
* Anchor decode + score filter + rotated-IoU NMS — ``ops.anchors`` / ``ops.nms3d``
  (K11 / K10).

Semantics kept from OpenPCDet that matter for parity: padded voxel slots are
zero *before* the linear layer, so they contribute relu(bn(0)) to the max;
the BEV canvas is zero where there is no pillar.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config.lidar import PointPillarsConfig, VoxelConfig
from .common import ConvBNAct, kaiming_init


def pillar_point_features(voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor,
                          vcfg: VoxelConfig, absolute_xyz: bool = True) -> torch.Tensor:
    """[V, P, 4] voxels → [V, P, 10] decorated features, padded slots zeroed.

    coords: [V, 4] (batch, z, y, x).  Matches OpenPCDet PillarVFE.forward.
    """
    vx, vy, vz = vcfg.voxel_size
    r = vcfg.point_cloud_range
    xyz = voxels[:, :, :3]
    n = num_points.clamp(min=1).to(voxels.dtype).view(-1, 1, 1)
    mean = xyz.sum(dim=1, keepdim=True) / n
    f_cluster = xyz - mean
    c = coords.to(voxels.dtype)
    f_center = torch.stack((
        xyz[:, :, 0] - (c[:, 3:4] * vx + (vx / 2 + r[0])),
        xyz[:, :, 1] - (c[:, 2:3] * vy + (vy / 2 + r[1])),
        xyz[:, :, 2] - (c[:, 1:2] * vz + (vz / 2 + r[2])),
    ), dim=-1)
    feats = [voxels if absolute_xyz else voxels[:, :, 3:], f_cluster, f_center]
    f = torch.cat(feats, dim=-1)
    P = voxels.shape[1]
    mask = (torch.arange(P, device=voxels.device).view(1, -1) < num_points.view(-1, 1)).to(f.dtype)
    return f * mask.unsqueeze(-1)


class PillarVFE(nn.Module):
    """Linear(10→C, no bias) → BN1d → ReLU → max over points."""

    def __init__(self, in_features: int = 10, out_features: int = 64):
        super().__init__()
        self.linear = nn.Linear(in_features, out_features, bias=False)
        self.norm = nn.BatchNorm1d(out_features, eps=1e-3, momentum=0.01)
        self.fused_weight = None  # [C, in] with BN folded
        self.fused_bias = None  # [C]

    @torch.no_grad()
    def fuse_bn(self) -> None:
        if self.fused_weight is not None:  # idempotent: a shared model is fused (fp32) once
            return
        scale = self.norm.weight / torch.sqrt(self.norm.running_var + self.norm.eps)
        self.fused_weight = (self.linear.weight * scale.view(-1, 1)).contiguous()
        self.fused_bias = (self.norm.bias - self.norm.running_mean * scale).contiguous()

    def forward(self, feats: torch.Tensor) -> torch.Tensor:  # [V, P, in] → [V, C]
        if self.fused_weight is not None:
            x = feats @ self.fused_weight.t().to(feats) + self.fused_bias.to(feats)
        else:
            x = self.linear(feats)
            x = self.norm(x.permute(0, 2, 1)).permute(0, 2, 1)
        return F.relu(x).max(dim=1).values


def scatter_to_bev(pillar_feats: torch.Tensor, coords: torch.Tensor, batch_size: int,
                   ny: int, nx: int, channels_last: bool = True) -> torch.Tensor:
    """PointPillarScatter: canvas[b, y, x, :] = feat[v]. Returns NHWC-contiguous
    tensor viewed as NCHW (channels_last memory format) or plain NCHW."""
    C = pillar_feats.shape[1]
    canvas = pillar_feats.new_zeros(batch_size * ny * nx, C)
    idx = coords[:, 0].long() * (ny * nx) + coords[:, 2].long() * nx + coords[:, 3].long()
    canvas[idx] = pillar_feats
    canvas = canvas.view(batch_size, ny, nx, C).permute(0, 3, 1, 2)
    return canvas if channels_last else canvas.contiguous()


class BEVBackbone(nn.Module):
    """BaseBEVBackbone: 3 down blocks + 3 up (transpose-conv) blocks, concat."""

    def __init__(self, c_in: int, layer_nums, layer_strides, num_filters, up_strides, up_filters):
        super().__init__()
        self.blocks = nn.ModuleList()
        self.deblocks = nn.ModuleList()
        c_prev = c_in
        for i, n in enumerate(layer_nums):
            layers = [ConvBNAct(c_prev, num_filters[i], 3, layer_strides[i], 1, act="relu")]
            layers += [ConvBNAct(num_filters[i], num_filters[i], 3, 1, 1, act="relu") for _ in range(n)]
            self.blocks.append(nn.Sequential(*layers))
            s = up_strides[i]
            self.deblocks.append(UpBlock(num_filters[i], up_filters[i], s))
            c_prev = num_filters[i]
        self.out_channels = sum(up_filters)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ups = []
        for blk, up in zip(self.blocks, self.deblocks):
            x = blk(x)
            ups.append(up(x))
        return torch.cat(ups, dim=1)


class UpBlock(nn.Module):
    """Upsample by ``s`` with a k=s, stride=s transpose conv (s ≥ 1), or
    downsample with a k=1/s, stride=1/s conv (s < 1; det3d RPN), + BN + ReLU.

    A k=s,stride=s transpose conv is a per-pixel GEMM [Cin]→[s*s*Cout]
    followed by a pixel shuffle; that is how the MFMA path executes it."""

    def __init__(self, c1: int, c2: int, s: float):
        super().__init__()
        self.s = s
        if s >= 1:
            s = int(round(s))
            self.conv = nn.ConvTranspose2d(c1, c2, s, stride=s, bias=False)
        else:
            k = int(round(1 / s))
            self.conv = nn.Conv2d(c1, c2, k, stride=k, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=1e-3, momentum=0.01)
        self.fused = False

    @torch.no_grad()
    def fuse_bn(self) -> None:
        if self.fused:
            return
        scale = self.bn.weight / torch.sqrt(self.bn.running_var + self.bn.eps)
        bias = self.bn.bias - self.bn.running_mean * scale
        w = self.conv.weight
        if isinstance(self.conv, nn.ConvTranspose2d):  # [Cin, Cout, k, k]
            new = nn.ConvTranspose2d(self.conv.in_channels, self.conv.out_channels, self.conv.kernel_size,
                                     stride=self.conv.stride, bias=True)
            new.weight.copy_(w * scale.view(1, -1, 1, 1))
        else:
            new = nn.Conv2d(self.conv.in_channels, self.conv.out_channels, self.conv.kernel_size,
                            stride=self.conv.stride, bias=True)
            new.weight.copy_(w * scale.view(-1, 1, 1, 1))
        new.bias.copy_(bias)
        self.conv = new.to(device=w.device, dtype=w.dtype)
        self.bn = None
        self.fused = True

    def forward(self, x):
        y = self.conv(x)
        if self.bn is not None:
            y = self.bn(y)
        return F.relu(y)


class AnchorHead(nn.Module):
    """AnchorHeadSingle: 1x1 convs for class, box residual and direction."""

    def __init__(self, c_in: int, num_anchors: int, num_classes: int, box_code: int = 7, dir_bins: int = 2):
        super().__init__()
        self.conv_cls = nn.Conv2d(c_in, num_anchors * num_classes, 1)
        self.conv_box = nn.Conv2d(c_in, num_anchors * box_code, 1)
        self.conv_dir = nn.Conv2d(c_in, num_anchors * dir_bins, 1)
        nn.init.constant_(self.conv_cls.bias, -math.log((1 - 0.01) / 0.01))
        nn.init.normal_(self.conv_box.weight, mean=0, std=0.001)
        nn.init.zeros_(self.conv_box.bias)

    def forward(self, x):
        return self.conv_cls(x), self.conv_box(x), self.conv_dir(x)


class PointPillars(nn.Module):
    def __init__(self, cfg: PointPillarsConfig | None = None):
        super().__init__()
        cfg = cfg or PointPillarsConfig()
        self.cfg = cfg
        self.vfe = PillarVFE(10, cfg.vfe_filters)
        self.backbone = BEVBackbone(cfg.bev_features, cfg.layer_nums, cfg.layer_strides, cfg.num_filters,
                                    cfg.upsample_strides, cfg.num_upsample_filters)
        self.head = AnchorHead(self.backbone.out_channels, cfg.num_anchors_per_loc, cfg.num_classes,
                               7, cfg.num_dir_bins)
        kaiming_init(self.vfe)
        kaiming_init(self.backbone)
        # restore head init after kaiming
        nn.init.constant_(self.head.conv_cls.bias, -math.log((1 - 0.01) / 0.01))

    def bev_forward(self, canvas: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """canvas [B, 64, ny, nx] → (cls [B, A*C, H, W], box [B, A*7, H, W], dir [B, A*2, H, W])."""
        return self.head(self.backbone(canvas))

    def forward(self, voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor, batch_size: int):
        feats = pillar_point_features(voxels, num_points, coords, self.cfg.voxel)
        pf = self.vfe(feats)
        nx, ny, _ = self.cfg.voxel.grid_size
        canvas = scatter_to_bev(pf, coords, batch_size, ny, nx, channels_last=True)
        return self.bev_forward(canvas)


def build_pointpillars(cfg: PointPillarsConfig | None = None, seed: int = 0) -> PointPillars:
    torch.manual_seed(seed)
    return PointPillars(cfg)
