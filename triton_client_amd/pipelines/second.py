"""3D SECOND-IoU pipeline on one GPU: raw PointCloud2 payloads → 3D boxes.

    PointCloud2 bytes ─K6 unpack→ points ─K7 voxelise (0.05x0.05x0.1 m, 5 pts,
    40000 voxels: the reference client's own voxels, data/kitti_dataset.yaml)→
    slot lists ─MeanVFE→ sparse level 0 ─VoxelBackBone8x (12 gather-GEMM MFMA
    layers, spconv.hip)→ NHWC BEV map [B, 200, 176, 256] ─BaseBEVBackbone +
    AnchorHeadSingle (fused MFMA convs)→ cls/box/dir ─K11 decode + top-1024 +
    rotated NMS 0.7→ 100 RoIs ─RoI grid pool (7x7 x 512) + FC stack→ IoU
    ─sigmoid rescoring + rotated NMS 0.01→ boxes [B, 500, 7], scores, labels

The reference runs this on the server as OpenPCDet SECONDNetIoU behind a
Triton Python backend (``examples/second_iou/1/model.py:115-182``, KIND_GPU),
fed by the client's CPU voxeliser (``clients/preprocess/preprocess_3d.py``).
Here the whole step is one capturable sequence of HIP kernels + hipBLASLt
GEMMs on static buffers.
"""
from __future__ import annotations

import copy
import types
from typing import Optional

import torch

from ..config.lidar import SecondIoUConfig
from ..models.common import fuse_model, lsuv_rescale
from ..models.second import SECONDNetIoU, bev_channel_permutation, build_second_iou, proposal_config
from ..ops._ws import Workspace
from ..ops.conv import NHWC
from ..ops.lidar import AnchorPostprocess, PointLayout, Voxelizer, pc2_unpack
from ..ops.spconv import RoIHead, SparseBackbone


class SecondPipeline:
    def __init__(self, model: Optional[SECONDNetIoU] = None, batch: int = 16, max_points: int = 131072,
                 layout: Optional[PointLayout] = None, z_offset: float = 1.5, normalize_intensity: bool = True,
                 device="cuda", cfg: Optional[SecondIoUConfig] = None, seed: int = 0, from_voxels: bool = False,
                 precision: str = "fp32"):
        """from_voxels: the served-model variant (level 0 comes from received
        voxels via :meth:`run_voxels`; no point-cloud buffers).  precision
        "fp32" (default; the reference serves SECOND-IoU in fp32): fp32 sparse
        rows, BEV maps and RoI features with split-product MFMA GEMMs / convs;
        "bf16": the secondary mode."""
        self.device = torch.device(device)
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision {precision!r}")
        self.precision = precision
        if self.device.type != "cuda":
            raise ValueError("SecondPipeline runs on the GPU; use models.second on the CPU")
        self.B, self.max_points = batch, max_points
        self.layout = layout or PointLayout.xyzi_f32()
        self.z_offset, self.normalize = z_offset, normalize_intensity
        if model is None:
            model = build_second_iou(cfg, seed)
        model = fuse_model(model.eval())
        self.cfg = model.cfg
        self.model = model.to(self.device)
        self.from_voxels = from_voxels
        if not from_voxels:
            self.frame_bytes = max_points * self.layout.point_step
            self.data = torch.zeros(batch * self.frame_bytes, dtype=torch.uint8, device=self.device)
            self.frame_off = torch.arange(batch, dtype=torch.int64, device=self.device) * self.frame_bytes
            self.frame_n = torch.zeros(batch, dtype=torch.int32, device=self.device)
            self.vox = Voxelizer(self.cfg.voxel, batch, max_points, device=self.device, materialize=False)
        self.ws = Workspace(self.device)
        self.sparse = None
        self.fast = None
        self.prop = AnchorPostprocess(proposal_config(self.cfg), batch, device=self.device)
        self.roi = None

    # ------------------------------------------------------------------ plans
    def build(self):
        """(Re)build the GPU plans from the current weights."""
        cfg = self.cfg
        self.sparse = SparseBackbone(cfg, self.model.backbone3d.layers, self.B, self.device,
                                     max_rows0=self.B * cfg.voxel.max_voxels, precision=self.precision)
        # the GPU BEV map is z-level-major (channel z*128 + c): permute the first
        # 2D conv's input channels to match (models.second.bev_channel_permutation)
        bb = copy.deepcopy(self.model.backbone)
        first = bb.blocks[0][0].conv
        perm = bev_channel_permutation(cfg).to(first.weight.device)
        with torch.no_grad():
            first.weight.copy_(first.weight[:, perm])
        shim = types.SimpleNamespace(cfg=cfg, backbone=bb, head=self.model.head)
        _, Hb, Wb = cfg.bev_shape
        self.fast = FastBEVPlan(shim, self.B, self.device, (Hb, Wb), self.precision)
        self.roi = RoIHead(cfg, self.model.roi_head, self.B, self.fast.cat_channels, self.device, self.precision)
        return self

    # ------------------------------------------------------------------ calibration
    @torch.no_grad()
    def _reference_sparse_input(self):
        """Voxels of the current sweeps for the fp32 reference model."""
        import numpy as np

        from ..ops.lidar import voxelize_np
        pts, cnt = pc2_unpack(self.ws, self.data, self.frame_off, self.frame_n, self.layout, self.max_points,
                              self.normalize, self.z_offset)
        pts, cnt = pts.cpu().numpy(), cnt.cpu().numpy()
        vs, ns, cs = [], [], []
        for b in range(self.B):
            v, zyx, num, _ = voxelize_np(pts[b, :int(cnt[b]), :4], self.cfg.voxel, 4)
            vs.append(v)
            ns.append(num)
            cs.append(np.concatenate([np.full((len(zyx), 1), b, np.int32), zyx], 1))
        dev = self.device
        return (torch.from_numpy(np.concatenate(vs)).to(dev), torch.from_numpy(np.concatenate(ns)).to(dev),
                torch.from_numpy(np.concatenate(cs)).to(dev))

    @torch.no_grad()
    def calibrate_detection_density(self, target_per_frame: float = 60.0, lsuv: bool = True) -> float:
        """Random-init SECOND-IoU: LSUV-rescale the sparse and 2D convolutions
        on the current sweeps (what BN statistics do for a trained model), then
        shift the IoU head's output bias so ~target RoIs per frame pass the 0.1
        score threshold before the final NMS.  Returns the shift."""
        m = self.model
        vox, nump, coords = self._reference_sparse_input()
        if lsuv:
            # sparse layers: unit output std, layer by layer, on the real sites
            from ..models.second import mean_vfe
            f, c, shp = mean_vfe(vox.float(), nump), coords.int(), self.cfg.sparse_shape
            for layer in m.backbone3d.layers:
                y, c2, shp2 = layer(f, c, shp)
                std = y.float().std().item()
                if std > 1e-8:
                    layer.weight.mul_(1.0 / std)
                    if layer.bias is not None:
                        layer.bias.mul_(1.0 / std)
                f, c, shp = layer(f, c, shp)
            bev = m.sparse_forward(vox, nump, coords, self.B)
            h = m.head
            lsuv_rescale(m, lambda: m.bev_forward(bev), head_modules=[h.conv_cls, h.conv_dir])
            h.conv_box.weight.mul_(0.2)  # plausible box residuals (exp(dl) near 1)
            h.conv_box.bias.mul_(0.2)
        bev = m.sparse_forward(vox, nump, coords, self.B)
        sf, cls, box, dir_ = m.bev_forward(bev)
        props = AnchorPostprocess(proposal_config(self.cfg), self.B, device=self.device)(cls.contiguous(),
                                                                                         box.contiguous(),
                                                                                         dir_.contiguous())
        logits = m.roi_iou(sf.float(), props.box)
        valid = torch.arange(props.box.shape[1], device=self.device)[None] < props.count[:, None].long()
        lg = logits[valid]
        if lsuv and lg.numel() > 1:
            last = m.roi_head.iou_layers[-1]
            s = 1.5 / max(lg.std().item(), 1e-6)
            last.weight.mul_(s)
            last.bias.mul_(s)
            lg = lg * s
        t = self.cfg.score_thresh

        def count(d):
            return (torch.sigmoid(lg + d) >= t).float().sum().item() / self.B

        lo, hi = -30.0, 30.0
        for _ in range(50):
            mid = 0.5 * (lo + hi)
            if count(mid) > target_per_frame:
                hi = mid
            else:
                lo = mid
        d = 0.5 * (lo + hi)
        m.roi_head.iou_layers[-1].bias += d
        self.calibration_shift = d
        self.sparse = self.fast = self.roi = None  # rebuild from the calibrated weights
        return d

    # ------------------------------------------------------------------ step
    def _second_stage(self):
        bev = self.sparse.bev
        cls, box, dir_ = self.fast.forward(NHWC(bev))
        props = self.prop(cls, box, dir_)
        return self.roi(self.fast.cat.t, props)

    @torch.no_grad()
    def step(self):
        if self.sparse is None:
            self.build()
        pts, cnt = pc2_unpack(self.ws, self.data, self.frame_off, self.frame_n, self.layout, self.max_points,
                              self.normalize, self.z_offset)
        self.sparse.reset()
        self.vox.assign(pts, cnt)
        self.sparse.encode_from_slots(pts, self.vox)
        self.vox.finish(pts, cnt, gather=False)
        self.sparse.forward()
        return self._second_stage()

    @torch.no_grad()
    def run_voxels(self, voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor, n: torch.Tensor):
        """Served path: voxels [cap, P, F] fp32, num_points [cap], coords
        [cap, 4] (b, z, y, x) int32, n [1] device voxel count (batch 1)."""
        if self.sparse is None:
            self.build()
        self.sparse.reset()
        self.sparse.encode_from_voxels(voxels, num_points, coords, n)
        self.sparse.forward()
        return self._second_stage()


class FastBEVPlan:
    """BaseBEVBackbone + merged anchor head on the fused convs, keeping the
    512-channel concat (SECONDHead pools its RoI grids from it)."""

    def __init__(self, shim, batch: int, device, bev_hw, precision: str = "fp32"):
        from ..models.fast import FastBEV
        # fp32: plain fp32 activations (the sparse BEV map is fp32 rows; SECONDHead pools the concat)
        self.plan = FastBEV(shim, batch, device, fused_neck=False, bev_hw=bev_hw, precision=precision, pair=False)
        self.cat = self.plan.cat
        self.cat_channels = self.cat.t.shape[-1]

    def forward(self, bev: NHWC):
        return self.plan.forward(bev)
