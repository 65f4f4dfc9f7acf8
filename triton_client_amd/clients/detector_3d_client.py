"""3D LiDAR client (reference ``clients/detector_3d_client.py``,
``clients/preprocess/preprocess_3d.py`` (OpenPCDet/spconv voxeliser),
``clients/preprocess/voxelize.py`` (det3d voxeliser),
``clients/postprocess/detector_3d_postprocess.py``).

Voxelisation runs in the spconv-exact HIP voxeliser (K7) when the points are
on the GPU, or its vectorised NumPy twin otherwise.  The voxel geometry comes
from the *served model's* ``ModelConfig.parameters`` when present (fixes
SURVEY Appendix A9: the reference voxelised with SECOND parameters — 5
points/voxel — for every 3D model), else from ``data/kitti_dataset.yaml``
like the reference.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import numpy as np
import torch
import yaml

from ..config.lidar import KITTI_SECOND_VOXELS, NUSC_PILLARS, VoxelConfig
from ..ops.lidar import Voxelizer, voxelize_np
from .base_client import Client
from .postprocess.base_postprocess import Postprocess
from .yolov5_client import DATA


def voxel_config_from_yaml(path: str) -> VoxelConfig:
    with open(path) as f:
        y = yaml.safe_load(f)
    rng = y["POINT_CLOUD_RANGE"]
    for p in y.get("DATA_PROCESSOR", []):
        if p.get("NAME") == "transform_points_to_voxels":
            mv = p["MAX_NUMBER_OF_VOXELS"]
            mv = mv.get("test", mv) if isinstance(mv, dict) else mv
            nf = len(y.get("POINT_FEATURE_ENCODING", {}).get("used_feature_list", ["x", "y", "z", "intensity"]))
            return VoxelConfig(tuple(rng), tuple(p["VOXEL_SIZE"]), int(p["MAX_POINTS_PER_VOXEL"]), int(mv), nf)
    raise ValueError(f"{path}: no transform_points_to_voxels entry")


def voxel_config_from_model(model_config) -> Optional[VoxelConfig]:
    p = getattr(model_config, "parameters", None)
    if p is None or "voxel_size" not in p:
        return None
    g = lambda k: json.loads(p[k].string_value)  # noqa: E731
    nf = int(g("num_point_features")) if "num_point_features" in p else 4
    return VoxelConfig(tuple(g("point_cloud_range")), tuple(g("voxel_size")), int(g("max_points_per_voxel")),
                       int(g("max_voxels")), nf)


class PointpillarPreprocess:
    """filter_pc(points [N, 4]) → {points, voxels [V, P, 4], voxel_coords [V, 4]
    (batch, z, y, x), voxel_num_points [V]} (reference preprocess_3d.py:30-52)."""

    def __init__(self, cfg: Optional[VoxelConfig] = None, device: str = "cpu", max_points: int = 262144):
        if cfg is None:
            path = os.path.join(DATA, "kitti_dataset.yaml")
            cfg = voxel_config_from_yaml(path) if os.path.exists(path) else KITTI_SECOND_VOXELS
        self.cfg = cfg
        self.device = torch.device(device)
        self.max_points = max_points
        self._vox = None

    def preprocess(self):
        pass

    def _mask_range(self, pc: np.ndarray) -> np.ndarray:
        r = self.cfg.point_cloud_range
        m = ((pc[:, 0] >= r[0]) & (pc[:, 0] <= r[3]) & (pc[:, 1] >= r[1]) & (pc[:, 1] <= r[4]))
        return pc[m]

    def filter_pc(self, pointcloud_array: np.ndarray) -> Dict[str, np.ndarray]:
        pc = np.ascontiguousarray(pointcloud_array, np.float32)
        nf = self.cfg.num_point_features
        if pc.shape[1] < nf:  # e.g. zero time-lag column for nuScenes (voxelize.py:38-39)
            pc = np.concatenate([pc, np.zeros((len(pc), nf - pc.shape[1]), np.float32)], 1)
        pc = self._mask_range(pc[:, :nf])  # OpenPCDet mask_points_and_boxes_outside_range
        if self.device.type == "cuda" and len(pc) <= self.max_points:
            if self._vox is None:
                self._vox = Voxelizer(self.cfg, 1, self.max_points, device=self.device, nfeat=nf)
            pts = torch.zeros((1, self.max_points, nf), dtype=torch.float32, device=self.device)
            pts[0, :len(pc)] = torch.from_numpy(pc).to(self.device)
            cnt = torch.tensor([len(pc)], dtype=torch.int32, device=self.device)
            v, c, n, vc = self._vox(pts, cnt)
            k = int(vc[0])
            voxels = v[0, :k].cpu().numpy()
            coords = c[0, :k].cpu().numpy().astype(np.int32)
            coords[:, 0] = 0
            num = n[0, :k].cpu().numpy().astype(np.int32)
        else:
            voxels, zyx, num, _ = voxelize_np(pc, self.cfg, nf)
            coords = np.pad(zyx, ((0, 0), (1, 0)), constant_values=0).astype(np.int32)
        return {"points": pc, "voxels": voxels, "voxel_coords": coords, "voxel_num_points": num}


    # ------------------------------------------------------------------ GPU, from the message bytes
    _TORCH = {"FP32": torch.float32, "INT32": torch.int32, "INT64": torch.int64, "FP16": torch.float16}

    def filter_cloud_gpu(self, cloud, normalize_intensity: bool = True, z_offset: float = 0.0,
                         dtypes: Optional[Dict[str, str]] = None,
                         out: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, torch.Tensor]:
        """PointCloud2 → {voxels, voxel_coords, voxel_num_points} as PINNED host
        tensors the wire encoder reads directly.  The payload bytes are uploaded
        once (pinned → device); unpack (K6: skip NaN, i /= max, z += offset —
        reference ros_inference3d.py:125-128), the spconv-order voxeliser (K7)
        and the dtype casts run on the GPU; only the V valid rows come back, by
        one DMA per tensor into reusable pinned staging — or, for a name in
        ``out`` (page-locked host arrays of max_voxels rows, e.g. a slot of a
        registered shared-memory region), straight into that array; the
        returned tensor is then a view of its first V rows."""
        from ..ops._ws import Workspace
        from ..ops.lidar import pc2_unpack
        from ..ros.compat import cloud_layout

        lay = cloud_layout(cloud)
        n = cloud.width * cloud.height
        nb = n * cloud.point_step
        cap = getattr(self, "_gcap", 0)
        if n > self.max_points:
            raise ValueError(f"{n} points > max_points {self.max_points}")
        if cap < nb:  # (re)build the device staging for this payload size
            self._gcap = cap = max(nb, 1 << 20)
            self._ws = Workspace(self.device)
            self._pin_raw = torch.empty((cap,), dtype=torch.uint8).pin_memory()
            self._dev_raw = torch.empty((cap,), dtype=torch.uint8, device=self.device)
            self._off = torch.zeros((1,), dtype=torch.int64, device=self.device)
            self._n = torch.zeros((1,), dtype=torch.int32, device=self.device)
            V, P, F = self.cfg.max_voxels, self.cfg.max_points_per_voxel, self.cfg.num_point_features
            self._pin_out = {"voxels": torch.empty((V, P, F), dtype=torch.float32).pin_memory(),
                             "voxel_coords": torch.empty((V, 4), dtype=torch.int64).pin_memory(),
                             "voxel_num_points": torch.empty((V,), dtype=torch.int64).pin_memory()}
            if self._vox is None:
                self._vox = Voxelizer(self.cfg, 1, self.max_points, device=self.device,
                                      nfeat=self.cfg.num_point_features)
        self._pin_raw[:nb].numpy()[...] = np.frombuffer(cloud.data, np.uint8, nb)
        self._dev_raw[:nb].copy_(self._pin_raw[:nb], non_blocking=True)
        self._n.fill_(n)
        pts, cnt = pc2_unpack(self._ws, self._dev_raw, self._off, self._n, lay, self.max_points, normalize_intensity,
                              z_offset, out_stride=self.cfg.num_point_features)
        v, c, num, vc = self._vox(pts, cnt)
        k = int(vc[0])  # the one small sync: how many rows to bring back
        dts = dtypes or {}
        dst, out = out or {}, {}
        for name, t in (("voxels", v[0, :k]), ("voxel_coords", c[0, :k]), ("voxel_num_points", num[0, :k])):
            tdt = self._TORCH.get(dts.get(name, ""), t.dtype if name == "voxels" else torch.int32)
            if name == "voxel_coords":
                t = t.clone()
                t[:, 0] = 0
            if name in dst:  # a host (page-locked) array, or a device tensor (device shared memory)
                pin = dst[name] if isinstance(dst[name], torch.Tensor) else torch.from_numpy(dst[name])
                if pin.dtype != tdt or pin.shape[0] < k or tuple(pin.shape[1:]) != tuple(t.shape[1:]):
                    raise ValueError(f"{name}: destination {tuple(pin.shape)} {pin.dtype} cannot take "
                                     f"{k} rows of {tuple(t.shape[1:])} {tdt}")
            else:
                pin = self._pin_out[name]
                if pin.dtype != tdt:
                    pin = self._pin_out[name] = torch.empty(pin.shape, dtype=tdt).pin_memory()
            pin[:k].copy_(t.to(tdt), non_blocking=True)
            out[name] = pin[:k]
        torch.cuda.current_stream(self.device).synchronize()
        return out


class det3DPreprocess(PointpillarPreprocess):
    """det3d / CenterPoint voxeliser: 5 features (zero time-lag), 0.2 m pillars,
    20 points, 20000 voxels (reference clients/preprocess/voxelize.py:11-49)."""

    def __init__(self, cfg: Optional[VoxelConfig] = None, device: str = "cpu", max_points: int = 262144):
        super().__init__(cfg or NUSC_PILLARS, device, max_points)


NUSC_SCORE_THRESH = {0: 0.4, 1: 0.4, 2: 0.4, 3: 0.3, 4: 0.4, 5: 0.4, 6: 0.15, 7: 0.15, 8: 0.1, 9: 0.1}


class PointPillarPostprocess(Postprocess):
    def load_class_names(self, namesfile: Optional[str] = None) -> List[str]:
        return Postprocess.load_class_names(namesfile or os.path.join(DATA, "nuScenes.names"))

    def extract_boxes(self, prediction) -> Dict[str, np.ndarray]:
        names = self.output_names(prediction)
        out = {n: self.output_array(prediction, i) for i, n in enumerate(names)}
        boxes = out.get("pred_boxes", self.output_array(prediction, 0))
        scores = out.get("pred_scores", self.output_array(prediction, 1))
        labels = out.get("pred_labels", self.output_array(prediction, 2))
        return {"pred_boxes": boxes.reshape(-1, boxes.shape[-1] if boxes.ndim > 1 else 7),
                "pred_scores": scores.reshape(-1), "pred_labels": labels.reshape(-1)}

    @staticmethod
    def get_annotations_indices(types, thresh, label_preds, scores) -> List[int]:
        return [int(i) for i in np.nonzero((label_preds == types) & (scores >= thresh))[0]]

    def remove_low_score_nu(self, predictions: Dict[str, np.ndarray], thresh: Optional[Dict[int, float]] = None):
        """Per-class nuScenes score thresholds (reference :98-133, with the
        dictionary keys fixed to pred_labels / pred_scores — Appendix A12)."""
        thresh = thresh or NUSC_SCORE_THRESH
        labels, scores = predictions["pred_labels"], predictions["pred_scores"]
        keep = np.zeros(len(labels), bool)
        for c, t in thresh.items():
            keep |= (labels == c) & (scores >= t)
        return {k: v[keep] for k, v in predictions.items() if k != "metadata"}


class Pointpillars_client(Client):
    def __init__(self, device: str = "cpu", voxel_cfg: Optional[VoxelConfig] = None, centerpoint: bool = False):
        super().__init__()
        self.device, self.voxel_cfg, self.centerpoint = device, voxel_cfg, centerpoint

    def get_preprocess(self):
        if self.centerpoint:
            return det3DPreprocess(self.voxel_cfg, self.device)
        return PointpillarPreprocess(self.voxel_cfg, self.device)

    def get_postprocess(self):
        return PointPillarPostprocess()

    def parse_model(self, model_metadata, model_config):
        if len(model_metadata.inputs) != 3:  # voxels, coords, num_points
            raise Exception(f"expecting 3 input, got {len(model_metadata.inputs)}")
        if len(model_metadata.outputs) != 3:
            raise Exception(f"expecting 3 output, got {len(model_metadata.outputs)}")
        cfg = voxel_config_from_model(model_config)
        if cfg is not None:
            self.voxel_cfg = cfg
        inp = [{"name": t.name, "shape": list(t.shape), "dtype": t.datatype} for t in model_metadata.inputs]
        out = [{"name": t.name, "shape": list(t.shape), "dtype": t.datatype} for t in model_metadata.outputs]
        return inp, out
