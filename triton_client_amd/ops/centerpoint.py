"""CenterPoint ops: 2-layer PFN + scatter (K8b/K9) and CenterHead decode + NMS (K12/K13/K10).

GPU paths call ``csrc/kernels/centerpoint.hip`` and ``csrc/kernels/nms.hip``;
CPU paths are the fp32 PyTorch / NumPy definitions in
:mod:`triton_client_amd.models.centerpoint`.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native
from ..config.lidar import CenterPointConfig, VoxelConfig
from ._ws import Workspace, dtype_code
from .lidar import Voxelizer
from .nms import Candidates, NmsResult, sort_and_nms

# nuScenes per-class thresholds (reference detector_3d_postprocess.py:103-112), keyed by
# the 0-based label of data/nuScenes.names
NUSC_CLASS_THRESH = {0: 0.4, 1: 0.4, 2: 0.4, 3: 0.3, 4: 0.4, 5: 0.4, 6: 0.15, 7: 0.15, 8: 0.1, 9: 0.1}
DET3D_ORDER = [0, 1, 2, 3, 4, 5, 7, 8, 6]  # internal [x,y,z,w,l,h,yaw,vx,vy] → det3d [...,vx,vy,yaw]


def _carr(ctype, vals):
    return (ctype * len(vals))(*vals)


class PFNEncoder:
    """Fused 2-layer PillarFeatureNet (BN folded) + scatter into an NHWC canvas:
    bf16, or fp32 with both layers as split products (``precision="fp32"``)."""

    def __init__(self, cfg: VoxelConfig, pfn, batch: int, device="cuda", precision: str = "bf16"):
        l1, l2 = pfn.layers
        assert l1.fused_weight is not None, "fuse_bn() the PillarFeatureNet first"
        self.cfg, self.B = cfg, batch
        self.device = torch.device(device)
        self.C = l2.units
        assert l1.units == 32 and l2.units == 64 and l1.linear.in_features == 10, "det3d [64, 64] PFN"
        f = lambda t: t.detach().float().contiguous().to(self.device)  # noqa: E731
        self.W1, self.b1, self.W2, self.b2 = f(l1.fused_weight), f(l1.fused_bias), f(l2.fused_weight), f(l2.fused_bias)
        nx, ny, _ = cfg.grid_size
        self.nx, self.ny = nx, ny
        self.ws = Workspace(self.device)
        self.f32 = precision == "fp32"
        self.canvas = self.ws.get("canvas", (batch, ny, nx, self.C), torch.float32 if self.f32 else torch.bfloat16,
                                  init=0)
        self._range = _carr(ctypes.c_float, cfg.point_cloud_range)
        self._vsize = _carr(ctypes.c_float, cfg.voxel_size)

    def clear_coords(self, coords: torch.Tensor, voxel_count: torch.Tensor, stream=None) -> None:
        _native.call("tca_pillar_canvas_clear", _native.ptr(coords), _native.ptr(voxel_count), coords.shape[0],
                     coords.shape[1], self.nx, self.ny, self.C, _native.ptr(self.canvas), dtype_code(self.canvas),
                     _native.stream_ptr(stream))

    def clear(self, vox: Voxelizer, stream=None) -> None:
        self.clear_coords(vox.coords, vox.voxel_count, stream)

    def encode_from_slots(self, points: torch.Tensor, vox: Voxelizer, feat_out=None, stream=None) -> torch.Tensor:
        _native.call("tca_pfn2_slots", _native.ptr(points), points.shape[-1], vox.max_points, _native.ptr(vox.slots),
                     _native.ptr(vox.vcount), _native.ptr(vox.coords), _native.ptr(vox.voxel_count), self.B,
                     self.cfg.max_voxels, self.cfg.max_points_per_voxel, _native.ptr(self.W1), _native.ptr(self.b1),
                     _native.ptr(self.W2), _native.ptr(self.b2), self._range, self._vsize, self.nx, self.ny,
                     _native.ptr(self.canvas), _native.ptr(feat_out), int(self.f32), _native.stream_ptr(stream))
        return self.canvas

    def encode_from_voxels(self, voxels, num_points, coords, voxel_count, feat_out=None, stream=None):
        """voxels [B, V, P, F>=4] fp32, num_points [B, V], coords [B, V, 4], voxel_count [B]."""
        _native.call("tca_pfn2_voxels", _native.ptr(voxels), voxels.shape[-1], _native.ptr(num_points),
                     _native.ptr(coords), _native.ptr(voxel_count), voxels.shape[0], voxels.shape[1], voxels.shape[2],
                     _native.ptr(self.W1), _native.ptr(self.b1), _native.ptr(self.W2), _native.ptr(self.b2),
                     self._range, self._vsize, self.nx, self.ny, _native.ptr(self.canvas), _native.ptr(feat_out),
                     int(self.f32), _native.stream_ptr(stream))
        return self.canvas


@dataclass
class CenterPointResult:
    """Per (frame, task) segment NMS output; ``per_image`` assembles frames."""
    nms: NmsResult   # box [B*T, max_out, 9] internal order, score, cls (global label), count [B*T]
    batch: int
    ntask: int

    def per_image(self) -> List[dict]:
        segs = self.nms.per_image()
        out = []
        for b in range(self.batch):
            parts = segs[b * self.ntask:(b + 1) * self.ntask]
            box = np.concatenate([p["box"] for p in parts]) if parts else np.zeros((0, 9), np.float32)
            out.append({"pred_boxes": box[:, DET3D_ORDER].astype(np.float32),
                        "pred_scores": np.concatenate([p["score"] for p in parts]).astype(np.float32),
                        "pred_labels": np.concatenate([p["cls"] for p in parts]).astype(np.int64)})
        return out

    @property
    def count(self) -> torch.Tensor:
        return self.nms.count.view(self.batch, self.ntask).sum(1)


class CenterPointPostprocess:
    """Merged NHWC head output [B, H, W, ldc] (task t's channels at ``task_offsets[t]``:
    reg 2, height 1, dim 3, rot 2, vel 2, hm nc) → per-task rotated NMS."""

    def __init__(self, cfg: CenterPointConfig, batch: int, task_offsets: Sequence[int], device="cuda",
                 class_thresh: Optional[dict] = None):
        self.cfg, self.B = cfg, batch
        self.device = torch.device(device)
        self.T = len(cfg.tasks)
        self.task_offsets = list(task_offsets)
        ncs = [len(t.class_names) for t in cfg.tasks]
        self.class_offsets = list(np.cumsum([0] + ncs)[:-1].astype(int))
        info = []
        for off, nc, c0 in zip(self.task_offsets, ncs, self.class_offsets):
            info += [off, nc, c0]
        self._info = _carr(ctypes.c_int, info)
        self.ncls = sum(ncs)
        th = [cfg.score_thresh] * self.ncls
        for c, v in (class_thresh or {}).items():
            if c < self.ncls:
                th[c] = float(v)
        self.class_thresh = th
        self._thresh = _carr(ctypes.c_float, th)
        self._range = _carr(ctypes.c_float, cfg.voxel.point_cloud_range)
        self._vsize = _carr(ctypes.c_float, cfg.voxel.voxel_size)
        self._pcr = _carr(ctypes.c_float, cfg.post_center_range)
        self.H, self.W = cfg.feature_map_size
        self.cap = min(self.H * self.W, 1 << 16)
        if self.device.type == "cuda":
            self.ws = Workspace(self.device)

    def __call__(self, head, stream=None) -> CenterPointResult:
        """head: NHWC tensor [B, H, W, ldc] (bf16/fp32/fp16) or an NHWC slice wrapper."""
        from .conv import NHWC
        t = head.t if isinstance(head, NHWC) else head
        base_off = head.off if isinstance(head, NHWC) else 0
        if t.device.type != "cuda":
            return self.cpu(t[..., base_off:].float())
        B, H, W, ldc = t.shape
        S = B * self.T
        cand = Candidates.alloc(self.ws, "cp_", S, self.cap, 9)
        ptr = _native.ptr(t) + base_off * t.element_size()
        _native.call("tca_centerhead_decode", ptr, dtype_code(t), ldc, B, H, W, self.T, self._info, self._thresh,
                     self.ncls, float(self.cfg.score_thresh), self._range, self._vsize, self.cfg.out_size_factor,
                     self._pcr, _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls),
                     _native.ptr(cand.key), _native.ptr(cand.count), self.cap, _native.stream_ptr(stream))
        res = sort_and_nms(self.ws, cand, 1, self.cfg.nms_iou, self.cfg.nms_pre_max, self.cfg.nms_post_max, True,
                           None, prefix="cp_nms_", stream=stream)
        return CenterPointResult(res, B, self.T)

    def cpu(self, head: torch.Tensor) -> CenterPointResult:
        """CPU reference (models.centerpoint.decode_reference) packed like the GPU result."""
        from ..models.centerpoint import decode_reference

        B = head.shape[0]
        outs = []
        for t, (off, tk) in enumerate(zip(self.task_offsets, self.cfg.tasks)):
            nc = len(tk.class_names)
            outs.append(head[..., off:off + 10 + nc].permute(0, 3, 1, 2))
        mo = self.cfg.nms_post_max
        S = B * self.T
        box = np.zeros((S, mo, 9), np.float32)
        score = np.zeros((S, mo), np.float32)
        cls = np.zeros((S, mo), np.int32)
        cnt = np.zeros((S,), np.int32)
        for t in range(self.T):
            per = decode_reference([outs[t]], self.cfg, [self.class_offsets[t]], self.class_thresh)
            for b, (bx, sc, lb) in enumerate(per):
                k = min(len(sc), mo)
                s = b * self.T + t
                box[s, :k] = bx[:k][:, [0, 1, 2, 3, 4, 5, 8, 6, 7]]  # det3d → internal order
                score[s, :k] = sc[:k]
                cls[s, :k] = lb[:k]
                cnt[s] = k
        return CenterPointResult(NmsResult(torch.from_numpy(box), torch.from_numpy(score), torch.from_numpy(cls),
                                           torch.from_numpy(cnt)), B, self.T)
