"""Detection engines: what turns sensor frames into detections for the drivers.

The reference has exactly one execution model — preprocess on the client
CPU, one blocking gRPC ``ModelInfer`` per frame, postprocess on the client
CPU (``communicator/ros_inference.py:117-175``,
``communicator/ros_inference3d.py:120-213``).  Here the drivers are
engine-agnostic and two engines implement the same ``detect(batch)``:

* **Local** (:class:`LocalDetector2D`, :class:`LocalDetector3D`) — the
  MI355X-native path: raw frame bytes go to the GPU, the captured
  camera / LiDAR hipGraph (K1 → fused-MFMA YOLOv5 → K3 → K4, or K6 → K7 →
  K8/K9 → fused BEV → K11 → K10) runs, and only the compacted detections come
  back.  Frames are micro-batched ``batch`` at a time (one graph replay per
  micro-batch); a pipeline is built per source geometry / point layout.
* **Remote** (:class:`RemoteDetector2D`, :class:`RemoteDetector3D`) — the
  reference's KServe-v2 client contract against any Triton / KServe server
  (including :mod:`triton_client_amd.server`): the model's tensor contract
  is read from ``ModelMetadata`` + ``ModelConfig``; requests go through the
  zero-copy C++ wire codec (``infer_raw``) or, with ``wire="proto"``, the
  reference's mutate-and-send ``ModelInferRequest``; ``mode="async"`` keeps
  several RPCs in flight (``-a``), ``mode="stream"`` uses ``ModelStreamInfer``
  (``--streaming``).

2D results: ``[n, 6]`` float32 ``x1, y1, x2, y2, conf, cls`` in *original
frame* pixels (the reference's H/W-swapped ``_scale_boxes`` is fixed,
SURVEY Appendix A2).  3D results: dict ``pred_boxes [n, 7]`` (x, y, z, dx,
dy, dz, yaw in the sensor frame — the +z offset applied before voxelising is
removed, reference ``ros_inference3d.py:172``), ``pred_scores [n]``,
``pred_labels [n]`` (1-based).
"""
from __future__ import annotations

import threading
from abc import ABC, abstractmethod
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops.image import frame_xform, preprocess
from ..ros import msgs
from ..utils.trace import trace_range
from ..utils.model_store import load_state_dict


def _device(device) -> torch.device:
    if device in (None, "auto"):
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(device)


FUSED_MARK = "_tca_fused_calibrated"


def load_weights(model, uri: str):
    """Load a checkpoint into ``model``: a plain state_dict of the module, or one written
    by :func:`export_weights` (BN folded, head prior calibrated), which is loaded into the
    model after folding its BN the same way."""
    from ..models.common import fuse_model

    sd = load_state_dict(uri)
    if FUSED_MARK in sd:
        sd = {k: v for k, v in sd.items() if k != FUSED_MARK}
        model = fuse_model(model.eval())
    model.load_state_dict(sd)
    return model


def export_weights(model, path: str) -> None:
    """The engine's model as a fused, calibrated checkpoint (fp32, CPU): loading it with
    ``--weights`` reproduces this engine's weights exactly (no re-calibration)."""
    sd = {k: v.detach().float().cpu().contiguous() for k, v in model.state_dict().items()}
    sd[FUSED_MARK] = torch.ones(1)
    torch.save(sd, path)


def _empty2d() -> np.ndarray:
    return np.zeros((0, 6), np.float32)


def _empty3d(box_dim: int = 7) -> dict:
    return {"pred_boxes": np.zeros((0, box_dim), np.float32), "pred_scores": np.zeros((0,), np.float32),
            "pred_labels": np.zeros((0,), np.int64)}


class Detector2D(ABC):
    names: List[str] = []

    @abstractmethod
    def detect(self, frames: Sequence[np.ndarray]) -> List[np.ndarray]:
        """frames: HxWx3 uint8 RGB arrays → per-frame [n, 6] detections."""


class Detector3D(ABC):
    names: List[str] = []

    @abstractmethod
    def detect(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        """PointCloud2 messages → per-cloud {pred_boxes, pred_scores, pred_labels}."""


def pack_task_segments(res, k: int, max_out: int):
    """CenterPointResult (NMS segments [B * T, mo, 9] internal box order, counts [B * T])
    -> the first ``k`` frames as fixed-size device rows: box [k, max_out, 9] in det3d
    order, score [k, max_out], label [k, max_out] int64, count [k] int32.  Segment t of
    frame b lands at rows sum(count[b, :t]) ..; rows past max_out are dropped.  Pure
    device ops (an exclusive prefix sum and one scatter): no host sync, graph-safe."""
    from ..ops.centerpoint import DET3D_ORDER

    T, nms = res.ntask, res.nms
    mo, D = nms.box.shape[1], nms.box.shape[2]
    dev = nms.box.device
    seg_box = nms.box[:k * T].view(k, T, mo, D)[..., list(DET3D_ORDER)].float().reshape(k, T * mo, D)
    seg_sc = nms.score[:k * T].reshape(k, T * mo).float()
    seg_lb = nms.cls[:k * T].reshape(k, T * mo).long()
    c = nms.count[:k * T].view(k, T).long().clamp(max=mo)
    ar = torch.arange(mo, device=dev)
    dest = (torch.cumsum(c, 1) - c)[..., None] + ar  # [k, T, mo]
    dest = torch.where((ar < c[..., None]) & (dest < max_out), dest, max_out).reshape(k, T * mo)  # max_out: trash row
    box = torch.zeros((k, max_out + 1, D), dtype=torch.float32, device=dev)
    score = torch.zeros((k, max_out + 1), dtype=torch.float32, device=dev)
    lab = torch.zeros((k, max_out + 1), dtype=torch.int64, device=dev)
    box.scatter_(1, dest[..., None].expand(-1, -1, D), seg_box)
    score.scatter_(1, dest, seg_sc)
    lab.scatter_(1, dest, seg_lb)
    return box[:, :max_out], score[:, :max_out], lab[:, :max_out], c.sum(1).clamp(max=max_out).to(torch.int32)


# =============================================================================== local
CAMERA_FAMILIES = ("yolov5", "yolov4", "retinanet", "fcos")


class LocalDetector2D(Detector2D):
    """A camera detector on this GPU, one captured graph per source geometry:

    * ``family="yolov5"`` — :class:`~triton_client_amd.pipelines.CameraPipeline`
      (the reference's ``Yolov5client`` models: YOLOv5nCOCO, YOLOv5nCROP / weed_detector);
    * ``"yolov4"`` — :class:`~triton_client_amd.pipelines.yolov4.Yolov4Pipeline`
      (``examples/YOLOv4/config.pbtxt``: 512 x 512, decode + per-class NMS);
    * ``"retinanet"`` / ``"fcos"`` — :class:`~triton_client_amd.pipelines.detectron.DetectronPipeline`
      (the reference's ``FCOS_client`` models, ``test_model`` =
      ``examples/RetinaNet_detectron/config.pbtxt``), fp32 like the served libtorch model.

    ``img`` is the model input (int: square); ``variant`` applies to YOLOv5 only."""

    def __init__(self, variant: str = "n", nc: int = 80, img=640, batch: int = 1, letterbox: bool = True,
                 conf_thres: float = 0.3, iou_thres: float = 0.45, max_det: int = 300, device="auto",
                 graph: bool = True, weights: Optional[str] = None, calibrate_target: Optional[float] = "auto",
                 seed: int = 0, names: Optional[Sequence[str]] = None, precision: str = "fp32",
                 family: str = "yolov5"):
        if family not in CAMERA_FAMILIES:
            raise ValueError(f"family {family!r}: one of {CAMERA_FAMILIES}")
        self.family = family
        self.device = _device(device)
        if family != "yolov5" and self.device.type != "cuda":
            raise ValueError(f"the local {family} engine runs on the GPU (device {self.device}); "
                             "on a GPU-less host serve the model and use --engine remote")
        self.precision = precision
        self.B, self.img = batch, (img, img) if isinstance(img, int) else tuple(img)
        self.mode = "letterbox" if letterbox else "stretch"
        self.conf_thres, self.iou_thres, self.max_det = conf_thres, iou_thres, max_det
        self.graph = graph and self.device.type == "cuda"
        if family == "yolov5":
            from ..models.yolov5 import build_yolov5
            self.model = build_yolov5(variant, nc, self.img, seed)
        elif family == "yolov4":
            from ..models.yolov4 import build_yolov4
            self.model = build_yolov4(nc, self.img, seed)
        else:
            from ..config.detectron import DetectronConfig
            from ..models.detectron import build_detectron
            self.det_cfg = DetectronConfig(arch=family, input_hw=self.img, num_classes=nc)
            self.model = build_detectron(self.det_cfg, seed)
            self.max_det = min(max_det, self.det_cfg.max_detections)
        if weights:
            self.model = load_weights(self.model, weights)
            calibrate_target = None
        if calibrate_target == "auto":
            calibrate_target = 300.0 if family in ("retinanet", "fcos") else 100.0
        self.calibrate_target = calibrate_target
        self.names = list(names) if names is not None else [str(i) for i in range(nc)]
        self._pipes: Dict[Tuple[int, int], tuple] = {}
        self._lock = threading.Lock()

    def _new_pipeline(self, hw: Tuple[int, int]):
        kw = dict(batch=self.B, src_hw=hw, mode=self.mode, device=self.device, precision=self.precision)
        if self.family == "yolov5":
            from ..pipelines import CameraPipeline
            return CameraPipeline(self.model, img_hw=self.img, conf_thres=self.conf_thres, iou_thres=self.iou_thres,
                                  max_det=self.max_det, **kw)
        if self.family == "yolov4":
            from ..pipelines.yolov4 import Yolov4Pipeline
            return Yolov4Pipeline(self.model, img=self.img[0], nc=self.model.cfg.nc, conf_thres=self.conf_thres,
                                  nms_thres=self.iou_thres, max_out=self.max_det, **kw)
        from ..pipelines.detectron import DetectronPipeline
        return DetectronPipeline(self.model, **kw)

    def _calibrated_pipeline(self, hw: Tuple[int, int], sample: Optional[np.ndarray]):
        """A new pipeline for frames of ``hw``; the first one built sets the
        random-init head prior from ``sample`` (HxWx3 uint8) once."""
        p = self._new_pipeline(hw)
        if self.calibrate_target is not None:  # random-init weights: set the head prior once
            if sample is None:
                from ..utils.synthetic import camera_frame
                sample = camera_frame(hw[0], hw[1], 0)
            p.frames.copy_(torch.from_numpy(np.array(sample, np.uint8)).to(p.frames.device).expand_as(p.frames))
            p.calibrate_detection_density(self.calibrate_target)
            self.calibrate_target = None
        self.model = p.model
        return p

    def live(self):
        """The streaming executor over this engine's model (``inference/live.py``):
        the live drivers' device path (GPU JPEG ingest, double-buffered graphs,
        GPU annotation, zero-copy publish); None on a GPU-less host."""
        if self.device.type != "cuda":
            return None
        if getattr(self, "_live", None) is None:
            from .live import LiveCamera
            with self._lock:
                if getattr(self, "_live", None) is None:
                    self._live = LiveCamera(self)
        return self._live

    def _pipe(self, hw: Tuple[int, int], sample: np.ndarray):
        if hw in self._pipes:
            return self._pipes[hw]
        from ..pipelines import GraphRunner

        p = self._calibrated_pipeline(hw, sample)
        pinned = torch.empty((self.B, *hw, 3), dtype=torch.uint8, pin_memory=self.device.type == "cuda")
        entry = (p, GraphRunner(p.step, enabled=self.graph), pinned)
        self._pipes[hw] = entry
        return entry

    @torch.no_grad()
    def calibrate_synthetic(self, seed: int = 0) -> None:
        """Set the random-init head prior from a synthetic frame (same on every
        rank, so data-parallel replicas agree before the parameter broadcast)."""
        if self.calibrate_target is not None:
            from ..utils.synthetic import camera_frame

            self._pipe(self.img, camera_frame(self.img[0], self.img[1], seed))

    @torch.no_grad()
    def detect(self, frames: Sequence[np.ndarray]) -> List[np.ndarray]:
        return self._run(frames, annotate=False)[0]

    @torch.no_grad()
    def detect_device(self, frames: torch.Tensor, max_det: Optional[int] = None):
        """Device-resident detection for the data-parallel path: ``frames``
        [n, H, W, 3] uint8 already in this GPU's memory (a DP shard) is copied
        device-to-device into the pipeline's frame buffer; returns
        ``(dets [n, max_det, 6] fp32, count [n] int32)`` on the device (x1, y1,
        x2, y2, conf, cls in frame pixels).  No host transfer of frames or
        results."""
        if self.device.type != "cuda" or not frames.is_cuda:
            raise ValueError("detect_device needs a GPU engine and GPU frames")
        n, H, W = frames.shape[:3]
        md = max_det or self.max_det
        if self.calibrate_target is not None:
            self.calibrate_synthetic()
        dets = torch.zeros((n, md, 6), dtype=torch.float32, device=frames.device)
        cnt = torch.zeros((n,), dtype=torch.int32, device=frames.device)
        with self._lock:
            p, run, _ = self._pipe((int(H), int(W)), None)
            for s in range(0, n, self.B):
                k = min(self.B, n - s)
                p.frames[:k].copy_(frames[s:s + k, ..., :3])
                res = run()
                m = min(md, res.box.shape[1])
                dets[s:s + k, :m, :4] = res.box[:k, :m]
                dets[s:s + k, :m, 4] = res.score[:k, :m]
                dets[s:s + k, :m, 5] = res.cls[:k, :m].float()
                cnt[s:s + k] = res.count[:k].clamp(max=md)
        return dets, cnt

    @torch.no_grad()
    def detect_annotated(self, frames: Sequence[np.ndarray], thickness: int = 2):
        """→ (annotated frames, detections).  The rectangles are drawn on the
        GPU into the pipeline's resident frame buffer (K15, ``ops.image.draw_boxes_``)
        and come back in the one D2H copy the publisher needs; only the label
        text is left to the host."""
        return self._run(frames, annotate=True, thickness=thickness)

    def _run(self, frames, annotate: bool, thickness: int = 2):
        from ..ops.image import draw_boxes_

        out: List[Optional[np.ndarray]] = [None] * len(frames)
        imgs: List[Optional[np.ndarray]] = [None] * len(frames)
        groups: Dict[Tuple[int, int], List[int]] = {}
        for i, f in enumerate(frames):
            groups.setdefault(tuple(f.shape[:2]), []).append(i)
        with self._lock:
            for hw, idx in groups.items():
                p, run, pinned = self._pipe(hw, frames[idx[0]][..., :3])
                for s in range(0, len(idx), self.B):
                    chunk = idx[s:s + self.B]
                    for j, i in enumerate(chunk):
                        pinned[j].numpy()[...] = frames[i][..., :3]
                    p.frames.copy_(pinned, non_blocking=True)
                    with trace_range("camera_graph"):
                        res = run()
                        if annotate:
                            draw_boxes_(p.frames, res.box, res.cls, res.count, thickness)
                            host = p.frames[:len(chunk)].cpu().numpy()
                        per = res.per_image()
                    for j, i in enumerate(chunk):
                        d = per[j]
                        out[i] = np.concatenate([d["box"], d["score"][:, None],
                                                 d["cls"][:, None].astype(np.float32)], 1).astype(np.float32)
                        if annotate:
                            imgs[i] = host[j]
        return out, imgs


class LocalDetector3D(Detector3D):
    """A LiDAR detector on this GPU (PointCloud2 payload bytes in, boxes out):

    * ``family="pointpillars"`` — :class:`~triton_client_amd.pipelines.LidarPipeline`
      (KITTI PointPillars, the served ``pointpillar_kitti``);
    * ``"second_iou"`` — :class:`~triton_client_amd.pipelines.SecondPipeline`
      (the reference's default 3D model, ``main3d.py -m second_iou``);
    * ``"centerpoint"`` — :class:`~triton_client_amd.pipelines.centerpoint.CenterPointPipeline`
      (nuScenes, 9-d boxes with yaw at index 8, 0-based labels).

    On a GPU-less host the same semantics run on the CPU (vectorised
    voxeliser + the fp32 reference modules)."""

    FAMILIES = {"pointpillars": 2000.0, "second_iou": 60.0, "centerpoint": 1000.0}  # default calibration targets
    Z_OFFSET = {"pointpillars": 1.5, "second_iou": 1.5, "centerpoint": 0.0}

    def __init__(self, cfg=None, batch: int = 1, device="auto", graph: bool = True, weights: Optional[str] = None,
                 calibrate_target="auto", z_offset: Optional[float] = None, normalize_intensity: bool = True,
                 seed: int = 0, max_points: int = 131072, family: str = "pointpillars"):
        if family not in self.FAMILIES:
            raise ValueError(f"family {family!r}: one of {sorted(self.FAMILIES)}")
        self.family = family
        self.device = _device(device)
        if family == "pointpillars":
            from ..config.lidar import PointPillarsConfig
            from ..models.pointpillars import build_pointpillars

            self.cfg = cfg or PointPillarsConfig()
            self.model = build_pointpillars(self.cfg, seed)
        elif family == "second_iou":
            from ..config.lidar import SecondIoUConfig
            from ..models.second import build_second_iou

            self.cfg = cfg or SecondIoUConfig()
            self.model = build_second_iou(self.cfg, seed)
        else:
            from ..config.lidar import CenterPointConfig
            from ..models.centerpoint import build_centerpoint

            self.cfg = cfg or CenterPointConfig()
            self.model = build_centerpoint(self.cfg, seed)
        self.box_dim = 9 if family == "centerpoint" else 7
        self.B, self.normalize = batch, normalize_intensity
        self.z_offset = self.Z_OFFSET[family] if z_offset is None else z_offset
        self.graph = graph and self.device.type == "cuda"
        if weights:
            self.model = load_weights(self.model, weights)
            calibrate_target = None
        self.calibrate_target = self.FAMILIES[family] if calibrate_target == "auto" else calibrate_target
        self.max_points = max_points
        self.names = list(self.cfg.class_names)
        self._pipes: Dict[tuple, tuple] = {}
        self._lock = threading.Lock()
        self._cpu = None

    # ----------------------------------------------------------------- GPU path
    def _pipeline_cls(self):
        if self.family == "second_iou":
            from ..pipelines import SecondPipeline
            return SecondPipeline
        if self.family == "centerpoint":
            from ..pipelines.centerpoint import CenterPointPipeline
            return CenterPointPipeline
        from ..pipelines import LidarPipeline
        return LidarPipeline

    def _calibrated_pipeline(self, layout, max_points: int, sample: Optional[msgs.PointCloud2]):
        """A new pipeline for clouds of ``layout`` (<= max_points points); the
        first one built sets the random-init head prior from ``sample`` once."""
        p = self._pipeline_cls()(self.model, batch=self.B, max_points=max_points, layout=layout,
                                 z_offset=self.z_offset, normalize_intensity=self.normalize, device=self.device)
        if self.calibrate_target is not None:
            if sample is None:
                sample = self._sample_cloud(0)
            raw = torch.frombuffer(bytearray(sample.data), dtype=torch.uint8)
            raw = raw[:min(raw.numel(), p.frame_bytes)]
            for b in range(self.B):
                p.data[b * p.frame_bytes: b * p.frame_bytes + raw.numel()].copy_(raw)
            p.frame_n.fill_(min(sample.width * sample.height, p.max_points))
            p.calibrate_detection_density(self.calibrate_target)
            self.calibrate_target = None
        self.model = p.model
        return p

    def live(self):
        """The streaming executor over this engine's model (``inference/live.py``):
        the live driver's device path (pinned payload ring, double-buffered
        graphs, one D2H of the results per batch)."""
        if self.device.type != "cuda":
            return None
        if getattr(self, "_live", None) is None:
            from .live import LiveLidar
            with self._lock:
                if getattr(self, "_live", None) is None:
                    self._live = LiveLidar(self)
        return self._live

    def _pipe(self, layout, npts: int, sample: msgs.PointCloud2):
        from ..pipelines import GraphRunner

        maxp = self.max_points
        while maxp < npts:
            maxp *= 2
        key = (layout.point_step, layout.offsets, layout.dtypes)
        ent = self._pipes.get(key)
        if ent is not None and ent[0].max_points >= npts:
            return ent
        p = self._calibrated_pipeline(layout, maxp, sample)
        pinned = torch.empty((self.B * p.frame_bytes,), dtype=torch.uint8, pin_memory=True)
        ent = (p, GraphRunner(p.step, enabled=self.graph), pinned, torch.zeros(self.B, dtype=torch.int32))
        self._pipes[key] = ent
        return ent

    def _sample_cloud(self, seed: int):
        from ..ros.compat import create_cloud_xyzi
        from ..utils.synthetic import LidarSpec, lidar_sweep

        spec = (LidarSpec(rings=32, azimuth_steps=1800, sensor_height=1.8) if self.family == "centerpoint"
                else LidarSpec(sensor_height=3.23))
        pts = lidar_sweep(spec, seed)
        return create_cloud_xyzi(np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4))

    @torch.no_grad()
    def calibrate_synthetic(self, seed: int = 0) -> None:
        """Set the random-init head prior from a synthetic sweep (rank-independent)."""
        if self.calibrate_target is None:
            return
        from ..ros.compat import cloud_layout

        cloud = self._sample_cloud(seed)
        if self.device.type == "cuda":
            self._pipe(cloud_layout(cloud), cloud.width, cloud)
        else:
            self._detect_cpu(cloud)

    def _frames_out(self, res) -> List[dict]:
        """Pipeline result → per-frame dicts in the sensor frame (z offset removed)."""
        if self.family == "centerpoint":
            per = res.per_image()
            for d in per:
                d["pred_boxes"] = d["pred_boxes"].copy()
                d["pred_boxes"][:, 2] -= self.z_offset
            return per
        out = []
        for d in res.per_image():
            box = d["box"].astype(np.float32).copy()
            box[:, 2] -= self.z_offset
            out.append({"pred_boxes": box, "pred_scores": d["score"].astype(np.float32),
                        "pred_labels": d["cls"].astype(np.int64)})
        return out

    @torch.no_grad()
    def detect(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        if self.device.type != "cuda":
            return [self._detect_cpu(c) for c in clouds]
        from ..ros.compat import cloud_layout

        out: List[Optional[dict]] = [None] * len(clouds)
        with self._lock:
            groups: Dict[tuple, List[int]] = {}
            lays = {}
            for i, c in enumerate(clouds):
                lay = cloud_layout(c)
                k = (lay.point_step, lay.offsets, lay.dtypes)
                lays[k] = lay
                groups.setdefault(k, []).append(i)
            for k, idx in groups.items():
                npts = max(clouds[i].width * clouds[i].height for i in idx)
                p, run, pinned, nh = self._pipe(lays[k], npts, clouds[idx[0]])
                for s in range(0, len(idx), self.B):
                    chunk = idx[s:s + self.B]
                    nh.zero_()
                    pn = pinned.numpy()
                    for j, i in enumerate(chunk):
                        c = clouds[i]
                        n = c.width * c.height
                        pn[j * p.frame_bytes: j * p.frame_bytes + n * c.point_step] = np.frombuffer(
                            c.data, np.uint8, n * c.point_step)
                        nh[j] = n
                    p.data.copy_(pinned, non_blocking=True)
                    p.frame_n.copy_(nh, non_blocking=True)
                    with trace_range("lidar_graph"):
                        per = self._frames_out(run())
                    for j, i in enumerate(chunk):
                        out[i] = per[j]
        return out

    @torch.no_grad()
    def detect_device(self, data: torch.Tensor, npts: torch.Tensor, fields, point_step: int,
                      max_out: int = 500):
        """Device-resident detection for the data-parallel path: ``data``
        [n, maxb] uint8 PointCloud2 payloads and ``npts`` [n] already in this
        GPU's memory; → ``(box [n, M, D], score [n, M], label [n, M] int64,
        count [n] int32)`` on the device, boxes in the sensor frame (z offset
        removed).  PointPillars / SECOND-IoU return their NmsResult rows; CenterPoint's
        per-(frame, task) NMS segments (6 tasks x <= 83, ``nms_post_max``) are packed on
        the device into each frame's first ``count`` rows, in task order, with the 9-d
        det3d box order (the layout of ``CenterPointResult.per_image``)."""
        from ..ops.lidar import PointLayout

        if self.device.type != "cuda" or not data.is_cuda:
            raise ValueError("detect_device needs a GPU engine and GPU payloads")
        by = {f.name: f for f in fields}
        names = ("x", "y", "z", "intensity")
        layout = PointLayout(int(point_step), tuple(by[k].offset for k in names), tuple(by[k].datatype for k in names))
        n, maxb = data.shape
        if self.calibrate_target is not None:
            self.calibrate_synthetic()
        D = self.box_dim
        dev = data.device
        box = torch.zeros((n, max_out, D), dtype=torch.float32, device=dev)
        score = torch.zeros((n, max_out), dtype=torch.float32, device=dev)
        lab = torch.zeros((n, max_out), dtype=torch.int64, device=dev)
        cnt = torch.zeros((n,), dtype=torch.int32, device=dev)
        with self._lock:
            p, run, _, _ = self._pipe(layout, max(1, maxb // max(1, int(point_step))), None)
            if maxb > p.frame_bytes:
                raise ValueError(f"payload of {maxb} B exceeds the pipeline's {p.frame_bytes} B frame slot")
            slots = p.data.view(p.B, p.frame_bytes)
            for s in range(0, n, self.B):
                k = min(self.B, n - s)
                slots[:k, :maxb].copy_(data[s:s + k])
                p.frame_n[:k].copy_(npts[s:s + k].to(torch.int32))
                res = run()
                if self.family == "centerpoint":
                    b, sc, lb, c = pack_task_segments(res, k, max_out)
                    box[s:s + k] = b
                    box[s:s + k, :, 2] -= self.z_offset
                    score[s:s + k], lab[s:s + k], cnt[s:s + k] = sc, lb, c
                    continue
                m = min(max_out, res.box.shape[1])
                b = res.box[:k, :m, :D].float()
                box[s:s + k, :m] = b
                box[s:s + k, :m, 2] -= self.z_offset
                score[s:s + k, :m] = res.score[:k, :m]
                lab[s:s + k, :m] = res.cls[:k, :m].long()
                cnt[s:s + k] = res.count[:k].clamp(max=max_out)
        return box, score, lab, cnt

    # ----------------------------------------------------------------- CPU path
    def _detect_cpu(self, cloud: msgs.PointCloud2) -> dict:
        from ..models.common import fuse_model
        from ..models.pointpillars import pillar_point_features, scatter_to_bev
        from ..ops.lidar import AnchorPostprocess, voxelize_np
        from ..ros.compat import cloud_to_numpy

        if self.family != "pointpillars":
            return self._detect_cpu_voxels(cloud)
        if self._cpu is None:
            self.model = fuse_model(self.model.eval()).float()
            self._cpu = AnchorPostprocess(self.cfg, 1, device="cpu")
        pts = cloud_to_numpy(cloud, normalize_intensity=self.normalize, z_offset=self.z_offset)
        v, zyx, num, _ = voxelize_np(pts, self.cfg.voxel, 4)
        if len(v) == 0:
            return _empty3d()
        coords = torch.from_numpy(np.pad(zyx, ((0, 0), (1, 0))).astype(np.int32))
        feats = pillar_point_features(torch.from_numpy(v), torch.from_numpy(num.astype(np.int64)), coords,
                                      self.cfg.voxel)
        if self.calibrate_target is not None:
            self._calibrate_cpu(feats, coords)
        nx, ny, _ = self.cfg.voxel.grid_size
        canvas = scatter_to_bev(self.model.vfe(feats), coords, 1, ny, nx, channels_last=False)
        res = self._cpu.cpu(*self.model.bev_forward(canvas))
        k = int(res.count[0])
        box = np.asarray(res.box[0, :k], np.float32).copy()
        box[:, 2] -= self.z_offset
        return {"pred_boxes": box, "pred_scores": np.asarray(res.score[0, :k], np.float32),
                "pred_labels": np.asarray(res.cls[0, :k]).astype(np.int64)}

    def _detect_cpu_voxels(self, cloud: msgs.PointCloud2) -> dict:
        """SECOND-IoU / CenterPoint on the CPU: the client-side voxeliser, then
        the served model's CPU path (same code as the KServe ``second_iou`` /
        ``centerpoint_pp`` models).  Random-init heads are not calibrated here."""
        from ..models.common import fuse_model
        from ..ops.lidar import voxelize_np
        from ..ros.compat import cloud_to_numpy

        if self._cpu is None:
            from ..server.models import CenterPointModel, SecondIoUModel

            m = (SecondIoUModel if self.family == "second_iou" else CenterPointModel)(cfg=self.cfg, device="cpu")
            self.model = m.model = fuse_model(self.model.eval()).float()
            m.ready = True
            self._cpu = m
            self.calibrate_target = None
        pts = cloud_to_numpy(cloud, normalize_intensity=self.normalize, z_offset=self.z_offset)
        v, zyx, num, _ = voxelize_np(pts, self.cfg.voxel, 4)
        if len(v) == 0:
            return _empty3d(self.box_dim)
        coords = np.pad(zyx, ((0, 0), (1, 0))).astype(np.int32)
        out = self._cpu.execute({"voxels": v, "voxel_coords": coords, "voxel_num_points": num.astype(np.int32)}, None)
        out = dict(out)
        out["pred_boxes"] = np.asarray(out["pred_boxes"], np.float32).copy()
        out["pred_boxes"][:, 2] -= self.z_offset
        return out

    def _calibrate_cpu(self, feats, coords):
        """CPU twin of LidarPipeline.calibrate_detection_density (bias shift only)."""
        from ..models.pointpillars import scatter_to_bev

        nx, ny, _ = self.cfg.voxel.grid_size
        cls, _, _ = self.model.bev_forward(scatter_to_bev(self.model.vfe(feats), coords, 1, ny, nx,
                                                          channels_last=False))
        m = cls.float().permute(0, 2, 3, 1).reshape(-1, self.cfg.num_classes).max(-1).values
        t, target = self.cfg.score_thresh, self.calibrate_target
        lo, hi = -30.0, 30.0
        for _ in range(40):
            mid = 0.5 * (lo + hi)
            if (torch.sigmoid(m + mid) >= t).float().sum().item() > target:
                hi = mid
            else:
                lo = mid
        self.model.head.conv_cls.bias += 0.5 * (lo + hi)
        self.calibrate_target = None


# =============================================================================== remote
class _stage:
    """Optional per-stage wall time: ``timer`` is a dict name -> [seconds]."""

    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        if self.timer is not None:
            import time as _t
            self.t0 = _t.perf_counter()

    def __exit__(self, *exc):
        if self.timer is not None:
            import time as _t
            self.timer.setdefault(self.name, []).append(_t.perf_counter() - self.t0)


_NP_OF = {"FP32": np.float32, "FP16": np.float16, "UINT8": np.uint8, "INT8": np.int8, "FP64": np.float64,
          "INT32": np.int32, "INT64": np.int64}


def _set_outputs(channel, names: Sequence[str]):
    from ..proto import service_pb2 as pb

    channel.request.ClearField("outputs")
    for n in names:
        channel.request.outputs.add(name=n)
    channel.output = pb.ModelInferRequest.InferRequestedOutputTensor(name=names[0]) if names else None


def _new_region(wire: str, nbytes: int, device):
    """The client's shared-memory region for a wire: system (page-locked /dev/shm
    mapping) or device (a GPU allocation shared by HIP IPC handle)."""
    from ..channel.shm import DeviceShmRegion, ShmRegion
    if wire == "devshm":
        if torch.device(device).type != "cuda":
            raise ValueError("wire='devshm' needs a GPU client (device='cuda')")
        return DeviceShmRegion(nbytes, device)
    return ShmRegion(nbytes)


def _device_output_to_host(a: torch.Tensor, conf_thres: float) -> np.ndarray:
    """A model output in device shared memory → the host array the postprocess reads.
    A decoded YOLO prediction [1, N, 5 + nc] comes back as only its rows with
    objectness > conf_thres (the postprocess's first filter, so its results are
    unchanged: the surviving rows keep their order); anything else whole."""
    if a.dim() == 3 and a.shape[0] == 1 and a.shape[2] > 5 and a.dtype == torch.float32:
        rows = a[0][a[0, :, 4] > conf_thres]
        return rows.cpu().numpy()[None]
    return a.cpu().numpy()


class _RemoteBase:
    def release_transport(self) -> None:
        """Unregister and free the shared-memory regions this client registered with the server
        (its own and its device path's): the drivers call it when they stop."""
        live = getattr(self, "_live", None)
        if live is not None and hasattr(live, "close"):
            live.close()
        close = getattr(self, "close_shm", None)
        if close is not None:
            close()

    def __init__(self, channel, client, mode: str = "sync", wire: str = "raw", window: int = 8):
        if mode not in ("sync", "async", "stream"):
            raise ValueError(f"mode {mode!r}")
        # shm: KServe system shared memory (same-host server); devshm: device shared memory
        # (a GPU allocation shared by HIP IPC handle: tensors stay on the GPU end to end)
        if wire not in ("raw", "proto", "shm", "devshm"):
            raise ValueError(f"wire {wire!r}")
        self.channel, self.client, self.mode, self.wire, self.window = channel, client, mode, wire, window
        # the client's staging (pinned buffers, shared-memory slots) is reused from call to call:
        # concurrent driver workers take turns on it; their RPCs still overlap
        self._stage_lock = threading.Lock()
        self._shm_lock = threading.Lock()
        md = channel.get_metadata()
        cfg = md["config_response"]
        self.model_metadata = md["metadata_response"]
        self.model_config = cfg.config if hasattr(cfg, "config") else cfg

    def _encode(self, inputs, outputs: Sequence[str], rid: str = "") -> bytes:
        """Raw wire: the request bytes, each tensor (numpy or pinned CPU torch
        staging) copied once by the C++ encoder."""
        from ..channel.wire import encode_request

        return encode_request(self.channel.model_name, [(n, a) for n, _, a in inputs], outputs,
                              self.channel.model_version, rid, [d for _, d, _ in inputs])

    def _send(self, raws: List[bytes]) -> list:
        """Pre-encoded requests → ParsedResponses (sync, or a window of futures)."""
        from ..channel.wire import parse_response

        ch = self.channel
        if self.mode != "async":
            return [ch.send_raw(r) for r in raws]
        res, fl = [None] * len(raws), []
        for i, r in enumerate(raws):
            fl.append((i, ch.send_raw_async(r)))
            if len(fl) >= self.window:
                j, f = fl.pop(0)
                res[j] = parse_response(f.result())
        for j, f in fl:
            res[j] = parse_response(f.result())
        return res

    def _request(self, inputs: Sequence[Tuple[str, str, np.ndarray]], outputs: Sequence[str], rid: str = ""):
        from ..proto import service_pb2 as pb

        req = pb.ModelInferRequest(model_name=self.channel.model_name, model_version=self.channel.model_version,
                                   id=rid)
        for name, dt, a in inputs:
            req.inputs.add(name=name, datatype=dt, shape=list(a.shape))
            req.raw_input_contents.append(np.ascontiguousarray(a).tobytes())
        for n in outputs:
            req.outputs.add(name=n)
        return req

    def _run(self, batches: List[Sequence[Tuple[str, str, np.ndarray]]], outputs: Sequence[str]) -> list:
        """One inference per item → responses (ParsedResponse or ModelInferResponse)."""
        ch = self.channel
        if self.mode == "sync":
            res = []
            for inp in batches:
                if self.wire == "raw":
                    res.append(ch.infer_raw([(n, a) for n, _, a in inp], outputs, [d for _, d, _ in inp]))
                else:  # the reference's reusable request, cleared and refilled (ros_inference.py:143-147)
                    r = ch.request
                    r.ClearField("inputs")
                    r.ClearField("raw_input_contents")
                    for name, dt, a in inp:
                        r.inputs.add(name=name, datatype=dt, shape=list(a.shape))
                        r.raw_input_contents.append(np.ascontiguousarray(a).tobytes())
                    r.ClearField("outputs")
                    for n in outputs:
                        r.outputs.add(name=n)
                    res.append(ch.do_inference())
            return res
        reqs = [self._request(inp, outputs, str(i)) for i, inp in enumerate(batches)]
        if self.mode == "async":  # bounded window of in-flight futures
            res, fl = [None] * len(reqs), []
            for i, rq in enumerate(reqs):
                fl.append((i, ch._grpc_stub.ModelInfer.future(rq, timeout=ch.timeout_s)))
                if len(fl) >= self.window:
                    j, f = fl.pop(0)
                    res[j] = f.result()
            for j, f in fl:
                res[j] = f.result()
            return res
        res = [None] * len(reqs)
        for k, r in enumerate(ch.stream_inference(reqs)):
            if r.error_message:
                raise RuntimeError(f"stream inference failed: {r.error_message}")
            i = int(r.infer_response.id) if r.infer_response.id else k
            res[i] = r.infer_response
        return res


class RemoteDetector2D(_RemoteBase, Detector2D):
    """2D detection through a KServe server (reference ``RosInference`` body)."""

    def __init__(self, channel, client, letterbox: bool = False, conf_thres: float = 0.3, iou_thres: float = 0.45,
                 mode: str = "sync", wire: str = "raw", scaling: Optional[str] = None, device="cpu",
                 names_file: Optional[str] = None):
        super().__init__(channel, client, mode, wire)
        (self.input_name, self.output_names, c, self.h, self.w, self.format,
         self.dtype) = client.parse_model(self.model_metadata, self.model_config)
        from ..proto import model_config_pb2 as mc

        self.nhwc = self.format == mc.ModelInput.FORMAT_NHWC
        # the tensor shape sent is the model's declared one (reference ros_inference.py:64-68:
        # [c, h, w] / [h, w, c]; Triton's `reshape` adds the batch dim), or [1, ...] when the
        # model declares an explicit batch dimension
        self.batch_dim = len(self.model_metadata.inputs[0].shape) == 4
        # the reference requests all 4 outputs of a Detectron model, else the first one
        # (ros_inference.py:70-87); YOLOv4's two outputs (confs, boxes) are both needed
        self.requested = list(self.output_names)
        ch = channel
        if ch.input is not None:
            ch.input.name, ch.input.datatype = self.input_name, self.dtype
            ch.input.ClearField("shape")
            shape = [self.h, self.w, c] if self.nhwc else [c, self.h, self.w]
            ch.input.shape.extend(([1] if self.batch_dim else []) + shape)
            _set_outputs(ch, self.requested)
        self.pre, self.post = client.get_preprocess(), client.get_postprocess()
        self.scaling = scaling or getattr(self.pre, "scaling", "COCO")
        self.mode2d = "letterbox" if letterbox else "stretch"
        self.conf_thres, self.iou_thres = conf_thres, iou_thres
        self.device = _device(device)
        self.names = self.post.load_class_names(names_file) if names_file else self.post.load_class_names()

    _TORCH_OF = {"FP32": torch.float32, "FP16": torch.float16, "UINT8": torch.uint8}

    def live(self):
        """The drivers' device path on a GPU client (``inference/remote_live.py``):
        GPU JPEG decode, K1 preprocess, one KServe request per frame, K3/K4 on the
        response, GPU annotation, zero-copy publish.  None on a CPU client (config 1).
        The shared-memory wires run it too: ``shm`` with the model input / outputs in a
        page-locked /dev/shm region, ``devshm`` with both in a device allocation the server maps
        by HIP IPC handle, so no tensor crosses host memory."""
        if self.device.type != "cuda":
            return None
        if getattr(self, "_live", None) is None:
            from .remote_live import RemoteLiveCamera
            self._live = RemoteLiveCamera(self)
        return self._live

    def _gpu_staging(self, hw):
        """Per source geometry: pinned frame upload buffer, device input, and
        the pinned staging the model input lands in (one D2H DMA)."""
        st = getattr(self, "_st", None)
        if st is None or st[0] != hw:
            H0, W0 = hw
            tdt = self._TORCH_OF.get(self.dtype, torch.float32)
            shape = (self.h, self.w, 3) if self.nhwc else (3, self.h, self.w)
            st = (hw, torch.empty((1, H0, W0, 3), dtype=torch.uint8).pin_memory(),
                  torch.empty((1, H0, W0, 3), dtype=torch.uint8, device=self.device),
                  torch.empty(((1,) if self.batch_dim else ()) + shape, dtype=tdt).pin_memory(), tdt)
            self._st = st
        return st

    def _prep(self, frame: np.ndarray):
        """→ (model input, xform).  GPU: frame → pinned → device → K1 preprocess
        → pinned staging (returned as a CPU torch tensor the wire encoder reads
        directly: no NumPy round trip, no intermediate host copy)."""
        if self.device.type == "cuda":
            _, pin_in, dev_in, pin_out, tdt = self._gpu_staging(tuple(frame.shape[:2]))
            pin_in[0].numpy()[...] = frame[..., :3]
            dev_in.copy_(pin_in, non_blocking=True)
            x, xf = preprocess(dev_in, (self.h, self.w), self.mode2d, self.scaling, torch.float32,
                               "NHWC" if self.nhwc else "NCHW")
            if self.nhwc:
                x = x.permute(0, 2, 3, 1)
            if not self.batch_dim:
                x = x[0]
            pin_out.copy_(x.to(tdt), non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            return pin_out, xf
        t = torch.from_numpy(np.array(frame[..., :3], np.uint8))
        x, xf = preprocess(t, (self.h, self.w), self.mode2d, self.scaling, torch.float32,
                           "NHWC" if self.nhwc else "NCHW")
        if self.nhwc:
            x = x.permute(0, 2, 3, 1)
        if not self.batch_dim:
            x = x[0]
        a = x.numpy()
        a = np.ascontiguousarray(a.astype(_NP_OF.get(self.dtype, np.float32), copy=False))
        return a, xf

    # ------------------------------------------------------------ shared memory
    def _shm_layout(self):
        """One request's slot: (slot bytes, input shape, input dtype, [(output, offset, bytes)])."""
        from ..proto import KSERVE_TO_NP

        def nbytes(shape, dt):
            return int(np.prod(shape)) * np.dtype(dt).itemsize

        def align(n):
            return (n + 4095) // 4096 * 4096

        in_shape = ((1,) if self.batch_dim else ()) + ((self.h, self.w, 3) if self.nhwc else (3, self.h, self.w))
        in_dt = _NP_OF.get(self.dtype, np.float32)
        layout, off = [], align(nbytes(in_shape, in_dt))
        md = {o.name: o for o in self.model_metadata.outputs}
        for n in self.requested:
            shape = [int(d) for d in md[n].shape]
            if any(d < 0 for d in shape):
                raise ValueError(f"shared memory transport needs a static shape for output '{n}', got {shape}")
            b = nbytes(shape, KSERVE_TO_NP[md[n].datatype])
            layout.append((n, off, b))
            off += align(b)
        return off, in_shape, in_dt, layout

    def _shm_setup(self):
        """Client shm region of `window` slots (input tensor + requested outputs
        each), registered with the server once."""
        if getattr(self, "_shm", None) is not None:
            return self._shm
        off, in_shape, in_dt, layout = self._shm_layout()
        region = _new_region(self.wire, off * self.window, self.device)
        region.register(self.channel)
        self._shm = (region, off, in_shape, in_dt, layout)
        return self._shm

    def close_shm(self) -> None:
        st = getattr(self, "_shm", None)
        if st is not None:
            try:
                st[0].unregister(self.channel)
            finally:
                st[0].close()
                self._shm = None

    def _prep_into(self, frame: np.ndarray, dst):
        """Preprocess straight into a shm slot (GPU: one D2H into the pinned mapping)."""
        if self.device.type == "cuda":
            _, pin_in, dev_in, _, tdt = self._gpu_staging(tuple(frame.shape[:2]))
            pin_in[0].numpy()[...] = frame[..., :3]
            dev_in.copy_(pin_in, non_blocking=True)
            x, xf = preprocess(dev_in, (self.h, self.w), self.mode2d, self.scaling, torch.float32,
                               "NHWC" if self.nhwc else "NCHW")
            if self.nhwc:
                x = x.permute(0, 2, 3, 1)
            if not self.batch_dim:
                x = x[0]
            (dst if isinstance(dst, torch.Tensor) else torch.from_numpy(dst)).copy_(x.to(tdt), non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()  # complete before the server reads it
            return xf
        a, xf = self._prep(frame)
        np.copyto(dst, a.reshape(dst.shape), casting="same_kind")
        return xf

    def _detect_shm(self, frames: Sequence[np.ndarray]) -> List[np.ndarray]:
        from ..channel.shm import shm_params
        from ..channel.wire import ParsedResponse
        from ..proto import KSERVE_TO_NP, service_pb2 as pb

        region, slot, in_shape, in_dt, layout = self._shm_setup()
        ch, timer = self.channel, getattr(self, "timer", None)
        res: List[Optional[np.ndarray]] = [None] * len(frames)
        free, inflight = list(range(self.window)), []

        def finish():
            i, k, xf, fut = inflight.pop(0)
            with _stage(timer, "rpc"):
                resp = pb.ModelInferResponse.FromString(fut.result())
            pr = ParsedResponse()
            pr.model_name = resp.model_name
            offs = {n: o for n, o, _ in layout}
            for t in resp.outputs:
                a = region.view(k * slot + offs[t.name], KSERVE_TO_NP[t.datatype], tuple(t.shape))
                if isinstance(a, torch.Tensor):  # device shared memory: only what the host needs comes back
                    a = _device_output_to_host(a, self.conf_thres)
                pr.outputs[t.name] = a
                pr.datatypes[t.name] = t.datatype
                pr.order.append(t.name)
            d = self._extract(pr)  # consumed before slot k is reused
            if len(d):
                d[:, :4] = xf.unmap_boxes(d[:, :4])
            res[i] = d
            free.append(k)

        for i, f in enumerate(frames):
            if not free:
                finish()
            k = free.pop(0)
            with _stage(timer, "preprocess"):
                xf = self._prep_into(f, region.view(k * slot, in_dt, in_shape))
            with _stage(timer, "encode"):
                req = pb.ModelInferRequest(model_name=ch.model_name, model_version=ch.model_version, id=str(i))
                t = req.inputs.add(name=self.input_name, datatype=self.dtype, shape=list(in_shape))
                shm_params(t, region.key, k * slot, int(np.prod(in_shape)) * np.dtype(in_dt).itemsize)
                for n, o, b in layout:
                    shm_params(req.outputs.add(name=n), region.key, k * slot + o, b)
                raw = req.SerializeToString()
            inflight.append((i, k, xf, ch._grpc_stub.ModelInferRaw.future(raw, timeout=ch.timeout_s)))
        while inflight:
            finish()
        return res

    def _extract(self, resp) -> np.ndarray:
        kw = {"conf_thres": self.conf_thres}
        if "iou_thres" in self.post.extract_boxes.__code__.co_varnames:
            kw["iou_thres"] = self.iou_thres
        d = self.post.extract_boxes(resp, **kw)
        d = d[0] if isinstance(d, list) else d
        return np.asarray(d, np.float32).reshape(-1, 6) if len(d) else _empty2d()

    def detect(self, frames: Sequence[np.ndarray]) -> List[np.ndarray]:
        from ..utils.trace import trace_range
        timer = getattr(self, "timer", None)
        if self.wire in ("shm", "devshm"):
            with self._shm_lock:
                return self._detect_shm(frames)
        if self.wire == "raw" and self.mode != "stream":
            # prepare + encode frame by frame: the staging buffer is reused, each
            # request's bytes are complete before the next frame is prepared
            xfs, raws = [], []
            for i, f in enumerate(frames):
                with self._stage_lock:
                    with trace_range("preprocess"), _stage(timer, "preprocess"):
                        a, xf = self._prep(f)
                    with _stage(timer, "encode"):
                        raws.append(self._encode([(self.input_name, self.dtype, a)], self.requested, str(i)))
                xfs.append(xf)
            with trace_range("rpc"), _stage(timer, "rpc"):
                resps = self._send(raws)
            preps = [(None, xf) for xf in xfs]
        else:
            preps = []
            for f in frames:
                with self._stage_lock, trace_range("preprocess"):
                    a, xf = self._prep(f)
                    preps.append((a.numpy().copy() if isinstance(a, torch.Tensor) else a, xf))
            with trace_range("rpc"):
                resps = self._run([[(self.input_name, self.dtype, a)] for a, _ in preps], self.requested)
        out = []
        for (a, xf), r in zip(preps, resps):
            d = self._extract(r)
            if len(d):
                d[:, :4] = xf.unmap_boxes(d[:, :4])
            out.append(d)
        return out


def _voxel_key(name: str, position: int) -> str:
    """Model input name → filter_pc() output (by name, else by position)."""
    n = name.lower()
    if "coord" in n:
        return "voxel_coords"
    if "num" in n:
        return "voxel_num_points"
    if "voxel" in n:
        return "voxels"
    return ("voxels", "voxel_coords", "voxel_num_points")[position]


class RemoteDetector3D(_RemoteBase, Detector3D):
    """3D detection through a KServe server (reference ``RosInference3D`` body):
    PointCloud2 → points (i/=max, z+=offset) → voxels (model's own voxel
    geometry, Appendix A9) → ModelInfer(voxels, voxel_coords, voxel_num_points)."""

    def __init__(self, channel, client, z_offset: float = 1.5, normalize_intensity: bool = True,
                 mode: str = "sync", wire: str = "raw", device="cpu"):
        super().__init__(channel, client, mode, wire)
        self.inputs, self.outputs = client.parse_model(self.model_metadata, self.model_config)
        self.pre, self.post = client.get_preprocess(), client.get_postprocess()
        if getattr(client, "voxel_cfg", None) is not None:
            from ..clients.detector_3d_client import PointpillarPreprocess

            self.pre = type(self.pre)(client.voxel_cfg, device) if isinstance(self.pre, PointpillarPreprocess) \
                else self.pre
        else:
            from ..clients.detector_3d_client import PointpillarPreprocess

            if isinstance(self.pre, PointpillarPreprocess) and str(device) != "cpu":
                self.pre = type(self.pre)(self.pre.cfg, device)
        self.names = self.post.load_class_names()
        self.z_offset, self.normalize = z_offset, normalize_intensity
        self.out_names = [o["name"] for o in self.outputs]
        ch = channel
        if ch.input is not None:
            _set_outputs(ch, self.out_names)

    def _detect_gpu_raw(self, clouds) -> List[dict]:
        """GPU unpack + voxelise into pinned staging, one C++-encoded request per
        cloud (no NumPy round trip of points or voxels)."""
        timer = getattr(self, "timer", None)
        keys = [_voxel_key(spec["name"], k) for k, spec in enumerate(self.inputs)]
        dts = {key: spec["dtype"] for key, spec in zip(keys, self.inputs)}
        raws, keep = [], []
        for i, c in enumerate(clouds):
            with self._stage_lock:  # the voxeliser's pinned staging is read by the encoder
                with _stage(timer, "preprocess"):
                    d = self.pre.filter_cloud_gpu(c, self.normalize, self.z_offset, dts)
                if d["voxels"].shape[0] == 0:
                    continue
                with _stage(timer, "encode"):
                    raws.append(self._encode([(spec["name"], spec["dtype"], d[key])
                                              for key, spec in zip(keys, self.inputs)], self.out_names, str(i)))
            keep.append(i)
        with _stage(timer, "rpc"):
            resps = self._send(raws)
        return keep, resps

    def _detect_gpu_shm(self, clouds) -> Tuple[List[int], list]:
        """Voxelise on the GPU, copy the voxel tensors from pinned staging into a
        slot of the client's shared-memory region and send only the region
        references (KServe system shared memory); detections return as raw
        outputs (variable-size)."""
        from ..channel.shm import ShmRegion, shm_params
        from ..channel.wire import parse_response
        from ..proto import service_pb2 as pb

        timer = getattr(self, "timer", None)
        ch = self.channel
        keys = [_voxel_key(spec["name"], k) for k, spec in enumerate(self.inputs)]
        dts = {key: spec["dtype"] for key, spec in zip(keys, self.inputs)}
        keep, resps, inflight = [], [], []
        free = list(range(self.window))

        def finish():
            j, k, fut = inflight.pop(0)
            with _stage(timer, "rpc"):
                resps.append((j, parse_response(fut.result())))
            free.append(k)

        if getattr(self, "_shm", None) is None:  # slot layout from the model's voxel budget and input dtypes
            cfg = self.pre.cfg
            vm = int(cfg.max_voxels)
            shapes = {"voxels": (vm, int(cfg.max_points_per_voxel), int(cfg.num_point_features)),
                      "voxel_coords": (vm, 4), "voxel_num_points": (vm,)}
            lay, off = [], 0
            for key in keys:
                dt = np.dtype(_NP_OF.get(dts.get(key, ""), np.float32 if key == "voxels" else np.int32))
                b = int(np.prod(shapes[key], dtype=np.int64)) * dt.itemsize
                lay.append((key, off, b, dt, shapes[key]))
                off += (b + 4095) // 4096 * 4096
            # system: page-locked, the voxeliser's D2H lands in it; device: written on the GPU
            region = _new_region(self.wire, off * self.window, getattr(self.pre, "device", "cpu"))
            region.register(ch)
            self._shm = (region, off, lay)
        region, slot, lay = self._shm

        for i, c in enumerate(clouds):
            if not free:
                finish()
            k = free.pop(0)
            with _stage(timer, "preprocess"):
                dst = {key: region.view(k * slot + o, dt, shp) for key, o, _, dt, shp in lay}
                d = self.pre.filter_cloud_gpu(c, self.normalize, self.z_offset, dts, out=dst)
            if d["voxels"].shape[0] == 0:
                free.append(k)
                continue
            with _stage(timer, "encode"):
                req = pb.ModelInferRequest(model_name=ch.model_name, model_version=ch.model_version, id=str(i))
                for (key, o, b, _, _), spec in zip(lay, self.inputs):
                    a = d[key]
                    t = req.inputs.add(name=spec["name"], datatype=spec["dtype"], shape=list(a.shape))
                    shm_params(t, region.key, k * slot + o, a.numel() * a.element_size())
                for n in self.out_names:
                    req.outputs.add(name=n)
                raw = req.SerializeToString()
            inflight.append((i, k, ch._grpc_stub.ModelInferRaw.future(raw, timeout=ch.timeout_s)))
            keep.append(i)
        while inflight:
            finish()
        order = {j: r for j, r in resps}
        return keep, [order[j] for j in keep]

    def close_shm(self) -> None:
        st = getattr(self, "_shm", None)
        if st is not None:
            try:
                st[0].unregister(self.channel)
            finally:
                st[0].close()
                self._shm = None

    def detect(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        from ..ros.compat import cloud_to_numpy

        gpu_pre = (getattr(self.pre, "device", None) is not None and self.pre.device.type == "cuda"
                   and hasattr(self.pre, "filter_cloud_gpu"))
        if self.wire == "devshm" and not gpu_pre:
            raise ValueError("wire='devshm' needs the GPU preprocess (device='cuda')")
        if self.wire in ("shm", "devshm") and gpu_pre:
            with self._shm_lock:
                keep, resps = self._detect_gpu_shm(clouds)
            return self._outputs(clouds, keep, resps)
        if self.wire == "raw" and self.mode != "stream" and gpu_pre:
            keep, resps = self._detect_gpu_raw(clouds)
            return self._outputs(clouds, keep, resps)
        batches, empty = [], []
        for c in clouds:
            pts = cloud_to_numpy(c, normalize_intensity=self.normalize, z_offset=self.z_offset)
            with self._stage_lock:
                d = self.pre.filter_pc(pts)
            empty.append(len(d["voxels"]) == 0)
            batches.append([(spec["name"], spec["dtype"],
                             np.ascontiguousarray(d[_voxel_key(spec["name"], k)].astype(_NP_OF[spec["dtype"]])))
                            for k, spec in enumerate(self.inputs)])
        keep = [i for i, e in enumerate(empty) if not e]
        resps = self._run([batches[i] for i in keep], self.out_names)
        return self._outputs(clouds, keep, resps)

    def _outputs(self, clouds, keep, resps) -> List[dict]:
        out = [_empty3d() for _ in clouds]
        for i, r in zip(keep, resps):
            d = self.post.extract_boxes(r)
            box = np.asarray(d["pred_boxes"], np.float32).copy()
            if len(box):
                box[:, 2] -= self.z_offset
            out[i] = {"pred_boxes": box, "pred_scores": np.asarray(d["pred_scores"], np.float32),
                      "pred_labels": np.asarray(d["pred_labels"]).astype(np.int64)}
        return out
