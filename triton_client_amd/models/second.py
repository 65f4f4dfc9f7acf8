"""SECOND-IoU (OpenPCDet ``SECONDNetIoU``) — the LiDAR detector the reference
serves as ``second_iou`` through a Triton Python backend on the GPU
(reference ``examples/second_iou/1/model.py:91-182``, config
``examples/second_iou/1/second_iou.yaml``, ``examples/second_iou/config.pbtxt``).

This module is the fp32 PyTorch definition (CPU path, numerics reference of
the HIP kernels, calibration); the MI355X execution is
``pipelines/second.py`` on ``ops/spconv.py`` (``csrc/kernels/spconv.hip``).

Stages:

* MeanVFE — mean of each voxel's points (x, y, z, intensity).
* VoxelBackBone8x — sparse 3D CNN.  Sparse tensors are (features [N, C],
  coords [N, 4] = (b, z, y, x), spatial shape).  :class:`SparseConv3d`
  implements both spconv layer kinds with the same output-stationary
  neighbour-table formulation the GPU uses: ``out[o] = relu(sum_t
  W_t^T in[nbr(o, t)] + b)`` where ``nbr(o, t)`` is the input site at
  ``o * stride - padding + t``; SubMConv3d keeps the input sites, SparseConv3d
  outputs every site whose receptive field holds an input site.
* HeightCompression — dense [B, C, D, H, W] → [B, C*D, H, W] (channel c*D+d).
* BaseBEVBackbone + AnchorHeadSingle — :mod:`.pointpillars` modules.
* SECONDHead — proposals (top-1024 by max class logit, rotated NMS 0.7, ≤100),
  7x7 RoI grid pooling on the 512-channel BEV map (``affine_grid`` +
  bilinear ``grid_sample`` exactly as OpenPCDet ``second_head.py`` calls them,
  i.e. PyTorch's default ``align_corners=False``), shared FC [256, 256], IoU
  FC [256, 256] → 1 logit per RoI.  Final boxes are the RoIs rescored by
  sigmoid(IoU) (SECONDNetIoU post-processing with no SCORE_TYPE).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config.lidar import SecondIoUConfig, SparseConvSpec
from .common import kaiming_init
from .pointpillars import AnchorHead, BEVBackbone


# ----------------------------------------------------------------------------- sparse tensors
def _linear_key(coords: torch.Tensor, shape: Sequence[int]) -> torch.Tensor:
    """(b, z, y, x) int → int64 key over [B, Z, Y, X]."""
    Z, Y, X = shape
    c = coords.long()
    return ((c[:, 0] * Z + c[:, 1]) * Y + c[:, 2]) * X + c[:, 3]


def _lookup(keys_sorted: torch.Tensor, perm: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """Row index of each query key (-1 if absent)."""
    if keys_sorted.numel() == 0:
        return torch.full_like(q, -1)
    pos = torch.searchsorted(keys_sorted, q).clamp(max=keys_sorted.numel() - 1)
    hit = keys_sorted[pos] == q
    return torch.where(hit, perm[pos], torch.full_like(q, -1))


def kernel_offsets(spec: SparseConvSpec) -> torch.Tensor:
    """[T, 3] (kz, ky, kx), tap index t = (kz*KY + ky)*KX + kx."""
    KZ, KY, KX = spec.kernel
    g = torch.stack(torch.meshgrid(torch.arange(KZ), torch.arange(KY), torch.arange(KX), indexing="ij"), -1)
    return g.reshape(-1, 3)


def sparse_out_coords(coords: torch.Tensor, shape_in: Sequence[int], spec: SparseConvSpec):
    """Output sites of a strided SparseConv3d: every o with an input site at
    o*s - p + k for some tap k.  Returns (coords [M, 4] sorted by key, shape)."""
    shp = tuple((shape_in[d] + 2 * spec.padding[d] - spec.kernel[d]) // spec.stride[d] + 1 for d in range(3))
    if coords.shape[0] == 0:
        return coords.new_zeros((0, 4)), shp
    offs = kernel_offsets(spec).to(coords.device)
    s = torch.tensor(spec.stride, device=coords.device)
    p = torch.tensor(spec.padding, device=coords.device)
    num = coords[:, None, 1:].long() + p - offs[None]  # [N, T, 3] = o * s
    ok = (num >= 0).all(-1) & (num % s == 0).all(-1)
    o = torch.div(num, s, rounding_mode="floor")
    ok &= (o < torch.tensor(shp, device=coords.device)).all(-1)
    b = coords[:, None, 0:1].long().expand(-1, o.shape[1], 1)
    cand = torch.cat([b, o], -1)[ok]
    key = torch.unique(_linear_key(cand, shp))
    Z, Y, X = shp
    out = torch.stack([key // (Z * Y * X), (key // (Y * X)) % Z, (key // X) % Y, key % X], 1)
    return out.to(torch.int32), shp


def neighbour_table(coords_out: torch.Tensor, coords_in: torch.Tensor, shape_in: Sequence[int],
                    spec: SparseConvSpec) -> torch.Tensor:
    """nbr [M, T]: input row at coords_out*stride - padding + tap (-1 if none)."""
    keys_in = _linear_key(coords_in, shape_in)
    ks, perm = torch.sort(keys_in)
    offs = kernel_offsets(spec).to(coords_out.device)
    s = torch.tensor(spec.stride, device=coords_out.device)
    p = torch.tensor(spec.padding, device=coords_out.device)
    pos = coords_out[:, None, 1:].long() * s - p + offs[None]  # [M, T, 3]
    inb = (pos >= 0).all(-1) & (pos < torch.tensor(shape_in, device=coords_out.device)).all(-1)
    b = coords_out[:, None, 0:1].long().expand(-1, pos.shape[1], 1)
    q = _linear_key(torch.cat([b, pos.clamp(min=0)], -1).reshape(-1, 4), shape_in).view(pos.shape[:2])
    nbr = _lookup(ks, perm, q.reshape(-1)).view(q.shape)
    return torch.where(inb, nbr, torch.full_like(nbr, -1))


class SparseConv3d(nn.Module):
    """spconv SubMConv3d / SparseConv3d (bias-free) + BatchNorm1d + ReLU.

    ``weight`` is [Cout, KZ, KY, KX, Cin] (spconv 2.x layout).  After
    :meth:`fuse_bn` the layer is ``relu(gather(x) @ W' + b')``: exactly what
    ``sp_gemm_kernel`` computes."""

    def __init__(self, spec: SparseConvSpec):
        super().__init__()
        self.spec = spec
        KZ, KY, KX = spec.kernel
        self.weight = nn.Parameter(torch.empty(spec.cout, KZ, KY, KX, spec.cin))
        nn.init.kaiming_normal_(self.weight.view(spec.cout, -1), mode="fan_in", nonlinearity="relu")
        self.bn = nn.BatchNorm1d(spec.cout, eps=1e-3, momentum=0.01)
        self.bias = None  # set by fuse_bn

    @torch.no_grad()
    def fuse_bn(self) -> None:
        if self.bn is None:
            return
        scale = self.bn.weight / torch.sqrt(self.bn.running_var + self.bn.eps)
        self.weight.mul_(scale.view(-1, 1, 1, 1, 1))
        self.bias = nn.Parameter((self.bn.bias - self.bn.running_mean * scale).detach().clone())
        self.bn = None

    def gemm_weight(self) -> torch.Tensor:
        """[Cout, T*Cin] with k = tap*Cin + ci (tap-major)."""
        return self.weight.reshape(self.spec.cout, -1)

    def forward(self, feats: torch.Tensor, coords: torch.Tensor, shape: Sequence[int]):
        s = self.spec
        if s.subm:
            co, shp = coords, tuple(shape)
        else:
            co, shp = sparse_out_coords(coords, shape, s)
        nbr = neighbour_table(co, coords, shape, s)
        x = torch.cat([feats, feats.new_zeros(1, feats.shape[1])], 0)
        g = x[nbr.clamp(min=-1) % x.shape[0]]  # -1 → the zero row
        y = g.reshape(co.shape[0], -1) @ self.gemm_weight().t().to(feats.dtype)
        if self.bn is not None:
            y = self.bn(y)
        elif self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return F.relu(y), co, shp


def mean_vfe(voxels: torch.Tensor, num_points: torch.Tensor) -> torch.Tensor:
    """OpenPCDet MeanVFE: sum over all P slots (padding is zero) / max(n, 1)."""
    n = num_points.clamp(min=1).to(voxels.dtype).view(-1, 1)
    return voxels.sum(dim=1) / n


def height_compression(feats: torch.Tensor, coords: torch.Tensor, shape: Sequence[int], batch: int) -> torch.Tensor:
    """spconv ``dense()`` + view: [B, C*D, H, W] with channel c*D + d."""
    D, H, W = shape
    C = feats.shape[1]
    dense = feats.new_zeros(batch, D, H, W, C)
    c = coords.long()
    dense[c[:, 0], c[:, 1], c[:, 2], c[:, 3]] = feats
    return dense.permute(0, 4, 1, 2, 3).reshape(batch, C * D, H, W)


class VoxelBackBone8x(nn.Module):
    def __init__(self, specs: Sequence[SparseConvSpec]):
        super().__init__()
        self.layers = nn.ModuleList(SparseConv3d(s) for s in specs)

    def forward(self, feats, coords, shape):
        for layer in self.layers:
            feats, coords, shape = layer(feats, coords, shape)
        return feats, coords, shape


# ----------------------------------------------------------------------------- RoI head
def roi_grid_pool_reference(features: torch.Tensor, rois: torch.Tensor, cfg: SecondIoUConfig) -> torch.Tensor:
    """SECONDHead.roi_grid_pool: features [B, C, H, W], rois [B, R, 7] →
    [B*R, C, G, G] (OpenPCDet ``roi_heads/second_head.py``)."""
    B, C, H, W = features.shape
    R = rois.shape[1]
    G = cfg.roi_grid
    r0 = cfg.voxel.point_cloud_range
    vx, vy = cfg.voxel.voxel_size[0], cfg.voxel.voxel_size[1]
    ds = cfg.feature_map_stride
    out = []
    for b in range(B):
        ro = rois[b].float()
        x1 = (ro[:, 0] - ro[:, 3] / 2 - r0[0]) / (vx * ds)
        x2 = (ro[:, 0] + ro[:, 3] / 2 - r0[0]) / (vx * ds)
        y1 = (ro[:, 1] - ro[:, 4] / 2 - r0[1]) / (vy * ds)
        y2 = (ro[:, 1] + ro[:, 4] / 2 - r0[1]) / (vy * ds)
        cosa, sina = torch.cos(ro[:, 6]), torch.sin(ro[:, 6])
        theta = torch.stack(((x2 - x1) / (W - 1) * cosa, (x2 - x1) / (W - 1) * (-sina), (x1 + x2 - W + 1) / (W - 1),
                             (y2 - y1) / (H - 1) * sina, (y2 - y1) / (H - 1) * cosa, (y1 + y2 - H + 1) / (H - 1)),
                            dim=1).view(-1, 2, 3).float()
        grid = F.affine_grid(theta, [R, C, G, G], align_corners=False)
        fb = features[b].float().unsqueeze(0).expand(R, C, H, W)
        out.append(F.grid_sample(fb, grid, mode="bilinear", padding_mode="zeros", align_corners=False))
    return torch.cat(out, 0)


class SECONDHead(nn.Module):
    """Shared FC (Conv1d k=1, BN, ReLU [, dropout]) + IoU branch → 1 logit."""

    def __init__(self, cfg: SecondIoUConfig, c_in: int):
        super().__init__()
        self.cfg = cfg
        G = cfg.roi_grid
        pre = G * G * c_in
        sh: List[nn.Module] = []
        for k, c in enumerate(cfg.roi_shared_fc):
            sh += [nn.Conv1d(pre, c, 1, bias=False), nn.BatchNorm1d(c), nn.ReLU()]
            pre = c
            if k != len(cfg.roi_shared_fc) - 1:
                sh.append(nn.Dropout(0.3))
        self.shared_fc = nn.Sequential(*sh)
        io: List[nn.Module] = []
        for k, c in enumerate(cfg.roi_iou_fc):
            io += [nn.Conv1d(pre, c, 1, bias=False), nn.BatchNorm1d(c), nn.ReLU()]
            pre = c
            if k == 0:
                io.append(nn.Dropout(0.3))
        io.append(nn.Conv1d(pre, 1, 1, bias=True))
        self.iou_layers = nn.Sequential(*io)
        for m in self.modules():
            if isinstance(m, nn.Conv1d):
                nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")

    def forward(self, pooled: torch.Tensor) -> torch.Tensor:
        """pooled [N, C, G, G] → IoU logits [N]."""
        x = self.shared_fc(pooled.reshape(pooled.shape[0], -1, 1))
        return self.iou_layers(x).view(-1)

    @torch.no_grad()
    def folded_linears(self) -> List[Tuple[torch.Tensor, torch.Tensor, bool]]:
        """[(W [out, in], b [out], relu)] with eval-mode BN folded in."""
        out = []
        mods = [m for m in list(self.shared_fc) + list(self.iou_layers) if not isinstance(m, (nn.Dropout, nn.ReLU))]
        i = 0
        while i < len(mods):
            conv = mods[i]
            w = conv.weight.detach().float().squeeze(-1)
            b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(w.shape[0], device=w.device)
            if i + 1 < len(mods) and isinstance(mods[i + 1], nn.BatchNorm1d):
                bn = mods[i + 1]
                sc = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
                w = w * sc.view(-1, 1)
                b = (b - bn.running_mean.float()) * sc + bn.bias.float()
                out.append((w, b, True))
                i += 2
            else:
                out.append((w, b, False))
                i += 1
        return out


# ----------------------------------------------------------------------------- the detector
class SECONDNetIoU(nn.Module):
    def __init__(self, cfg: Optional[SecondIoUConfig] = None):
        super().__init__()
        cfg = cfg or SecondIoUConfig()
        self.cfg = cfg
        self.backbone3d = VoxelBackBone8x(cfg.sparse)
        self.backbone = BEVBackbone(cfg.bev_features, cfg.layer_nums, cfg.layer_strides, cfg.num_filters,
                                    cfg.upsample_strides, cfg.num_upsample_filters)
        self.head = AnchorHead(self.backbone.out_channels, cfg.num_anchors_per_loc, cfg.num_classes, 7,
                               cfg.num_dir_bins)
        self.roi_head = SECONDHead(cfg, self.backbone.out_channels)
        kaiming_init(self.backbone)
        nn.init.constant_(self.head.conv_cls.bias, -math.log((1 - 0.01) / 0.01))

    def fuse_bn(self) -> None:
        for m in self.backbone3d.layers:
            m.fuse_bn()

    def sparse_forward(self, voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor,
                       batch_size: int) -> torch.Tensor:
        """voxels [V, P, 4], num_points [V], coords [V, 4] (b, z, y, x) →
        HeightCompression BEV map [B, 256, ny/8, nx/8]."""
        f = mean_vfe(voxels.float(), num_points)
        f, c, shp = self.backbone3d(f, coords.to(torch.int32), self.cfg.sparse_shape)
        return height_compression(f, c, shp, batch_size)

    def bev_forward(self, bev: torch.Tensor):
        """→ (spatial_features_2d [B, 512, H, W], cls, box, dir)."""
        sf = self.backbone(bev)
        cls, box, dir_ = self.head(sf)
        return sf, cls, box, dir_

    def roi_iou(self, spatial_features: torch.Tensor, rois: torch.Tensor) -> torch.Tensor:
        """rois [B, R, 7] → IoU logits [B, R]."""
        pooled = roi_grid_pool_reference(spatial_features, rois, self.cfg)
        return self.roi_head(pooled).view(rois.shape[0], rois.shape[1])


def build_second_iou(cfg: Optional[SecondIoUConfig] = None, seed: int = 0) -> SECONDNetIoU:
    torch.manual_seed(seed)
    return SECONDNetIoU(cfg)


def proposal_config(cfg: SecondIoUConfig) -> SecondIoUConfig:
    """The anchor-decode / NMS parameters of SECONDHead's proposal layer
    (NMS_CONFIG.TEST: class-agnostic, pre 1024, post 100, IoU 0.7, no score
    threshold)."""
    import dataclasses
    return dataclasses.replace(cfg, score_thresh=0.0, nms_thresh=cfg.proposal_nms_thresh,
                               nms_pre_max=cfg.proposal_pre_max, nms_post_max=cfg.proposal_post_max)


def bev_channel_permutation(cfg: SecondIoUConfig) -> torch.Tensor:
    """perm[k] = HeightCompression channel held at NHWC channel k of the GPU's
    BEV map, which stores z-level-major (k = z*C + c) so the last sparse
    layer's epilogue writes 16-B channel vectors; the 2D backbone's first conv
    is permuted to match."""
    D = cfg.level_shapes()[-1][0]
    C = cfg.sparse[-1].cout
    return torch.tensor([c * D + z for z in range(D) for c in range(C)])


def postprocess_reference(rois: torch.Tensor, roi_labels: torch.Tensor, roi_count: torch.Tensor, iou_logits: torch.Tensor,
                          cfg: SecondIoUConfig):
    """SECONDNetIoU.post_processing (no SCORE_TYPE → score = sigmoid(IoU)),
    class-agnostic rotated NMS.  Returns per-frame (boxes, scores, labels)."""
    import numpy as np

    from ..ops.nms import sort_and_nms_cpu
    out = []
    for b in range(rois.shape[0]):
        n = int(roi_count[b])
        s = torch.sigmoid(iou_logits[b, :n].float()).numpy()
        idx = np.nonzero(s >= cfg.score_thresh)[0]
        bx = rois[b, :n].float().numpy()
        lab = roi_labels[b, :n].numpy()
        keep = sort_and_nms_cpu(bx[idx], s[idx], lab[idx], idx, 1, cfg.nms_thresh, cfg.nms_pre_max, cfg.nms_post_max,
                                True)
        k = idx[keep]
        out.append((bx[k], s[k], lab[k]))
    return out
