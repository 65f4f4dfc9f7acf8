"""Live 3D inference driver (reference ``communicator/ros_inference3d.py:44-213``).

PointCloud2 in → boxes out as a jsk ``BoundingBoxArray`` (default) or a
``vision_msgs/Detection3DArray``, header stamp/frame_id copied from the
cloud.  Reference behaviours kept as configurable defaults:
z offset +1.5 before voxelising (removed from the output boxes), intensity
normalised by its max, only label 2 (Pedestrian) with score > 0.5 published,
jsk dimensions swapped (x = dy, y = dx).  Fixed: the Detection3DArray yaw is
taken from the box's own dimension (index 6 for 7-d boxes, 8 for 9-d; A8).
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import numpy as np

from ..ros import compat, msgs
from ..utils.metrics import StageTimer
from .base_inference import BaseInference
from .engines import Detector3D, RemoteDetector3D


def select_boxes(pred: dict, labels: Optional[Sequence[int]] = (2,), score_thresh: float = 0.5) -> np.ndarray:
    """Indices kept for publishing (reference :156 keeps label==2 & score>0.5)."""
    s, l_ = pred["pred_scores"], pred["pred_labels"]
    keep = s > score_thresh
    if labels is not None:
        keep &= np.isin(l_, np.asarray(labels))
    return np.nonzero(keep)[0]


def jsk_columns(pred: dict, idx) -> dict:
    """The published fields of the selected boxes as columns (float64 like the
    message): position [n, 3], orientation [n, 4] (yaw about +z, reference
    ``yaw2quaternion`` :117-118), dimensions [n, 3] with the reference's x/y
    swap (:169-171), value [n] fp32, label [n] uint32."""
    idx = np.asarray(idx, np.int64)
    b = np.asarray(pred["pred_boxes"])[idx].astype(np.float64)
    yaw = b[:, 8 if b.shape[-1] >= 9 else 6] if len(b) else np.zeros((0,))
    quat = np.zeros((len(b), 4))
    quat[:, 2], quat[:, 3] = np.sin(yaw / 2), np.cos(yaw / 2)
    return {"position": b[:, :3], "orientation": quat, "dimensions": b[:, [4, 3, 5]] if len(b) else np.zeros((0, 3)),
            "value": np.asarray(pred["pred_scores"])[idx].astype(np.float32),
            "label": np.asarray(pred["pred_labels"])[idx].astype(np.uint32)}


def boxes_to_jsk(pred: dict, idx, header: msgs.Header) -> msgs.BoundingBoxArray:
    """jsk BoundingBoxArray of the selected boxes, built from columns: the
    BoundingBox objects are made only if a subscriber reads ``boxes``
    (:class:`~triton_client_amd.ros.msgs.ArrayList`); serialisation packs the
    columns directly (``ros.rosmsg``)."""
    cols = jsk_columns(pred, idx)

    def build():
        P, Q, D = cols["position"].tolist(), cols["orientation"].tolist(), cols["dimensions"].tolist()
        V, L = cols["value"].tolist(), cols["label"].tolist()
        return [msgs.BoundingBox(header=header, pose=msgs.Pose(msgs.Point(*p), msgs.Quaternion(*q)),
                                 dimensions=msgs.Vector3(*d), value=v, label=lb)
                for p, q, d, v, lb in zip(P, Q, D, V, L)]
    return msgs.BoundingBoxArray(header=header, boxes=msgs.ArrayList(len(cols["value"]), build, cols))


def boxes_to_detection3d(pred: dict, idx, header: msgs.Header) -> msgs.Detection3DArray:
    arr = msgs.Detection3DArray(header=header)
    b = pred["pred_boxes"]
    yaw_i = 8 if b.shape[-1] >= 9 else 6
    for i in idx:
        x = b[i]
        arr.detections.append(msgs.Detection3D(
            header=header,
            results=[msgs.ObjectHypothesisWithPose(id=int(pred["pred_labels"][i]), score=float(pred["pred_scores"][i]))],
            bbox=msgs.BoundingBox3D(
                center=msgs.Pose(msgs.Point(float(x[0]), float(x[1]), float(x[2])),
                                 compat.yaw2quaternion(float(x[yaw_i]))),
                size=msgs.Vector3(float(x[3]), float(x[4]), float(x[5])))))
    return arr


class RosInference3D(BaseInference):
    def __init__(self, channel=None, client=None, engine: Optional[Detector3D] = None, params: Optional[dict] = None,
                 bus=None, jsk: bool = True, labels: Optional[Sequence[int]] = (2,), score_thresh: float = 0.5,
                 z_offset: float = 1.5, queue_size: Optional[int] = 50, metrics=None, mode: str = "sync",
                 wire: str = "raw", batch: int = 1, workers: int = 1):
        super().__init__(channel, client)
        self._params = params or {}
        self.engine = engine or RemoteDetector3D(channel, client, z_offset=z_offset, mode=mode, wire=wire)
        self.bus, self.jsk, self.labels, self.score_thresh = bus, jsk, labels, score_thresh
        self.queue_size, self.metrics = queue_size, metrics
        self.frames = 0
        self.sub = self.pub = None
        # batch > 1: the reference's queue of 50 becomes a latest-wins window
        # drained as micro-batches (one engine call per batch), re-published in
        # header.seq order (see .batching)
        self.batch, self.workers = max(1, batch), max(1, workers)
        self.runner = None

    def start_inference(self, spin: bool = True, timeout: Optional[float] = None):
        p = self.params
        t = msgs.BoundingBoxArray if self.jsk else msgs.Detection3DArray
        self.pub = compat.Publisher(p["pub_topic"], t, queue_size=1, bus=self.bus)
        cb, qs = self._pc_callback, self.queue_size
        if self.batch > 1 or self.workers > 1:
            from .batching import MicroBatchRunner
            self.runner = MicroBatchRunner(lambda cs: [m for m, _ in self.process(cs)], self.pub.publish,
                                           batch=self.batch, workers=self.workers,
                                           capacity=max(self.queue_size or 0, 2 * self.batch * self.workers))
            cb, qs = self.runner.push, None
        self.sub = compat.Subscriber(p["sub_topic"], msgs.PointCloud2, cb, queue_size=qs, bus=self.bus,
                                     ingest=getattr(self.engine, "ingest_buffer", None))
        if spin:
            compat.spin(self.bus, timeout)

    def stop(self, drain: bool = True):
        if self.sub is not None:
            self.sub.unregister()
            self.sub = None
        if self.runner is not None:
            self.runner.close(drain=drain)
            self.runner = None

    def to_msg(self, pred: dict, header: msgs.Header):
        idx = select_boxes(pred, self.labels, self.score_thresh)
        hdr = msgs.Header(seq=header.seq, stamp=header.stamp, frame_id=header.frame_id)
        return boxes_to_jsk(pred, idx, hdr) if self.jsk else boxes_to_detection3d(pred, idx, hdr)

    def _live(self):
        """The engine's streaming device path (LocalDetector3D on a GPU), else None."""
        if not hasattr(self, "_live_exec"):
            fn = getattr(self.engine, "live", None)
            self._live_exec = fn() if callable(fn) else None
        return self._live_exec

    def process(self, clouds: Sequence[msgs.PointCloud2]) -> List[tuple]:
        t0 = time.perf_counter()
        timer = StageTimer(self.metrics)
        live = self._live()
        with timer("detect3d"):
            preds = live.process(clouds) if live is not None else self.engine.detect(clouds)
        with timer("boxes_publish"):
            out = [(self.to_msg(p, c.header), p) for c, p in zip(clouds, preds)]
        self.frames += len(clouds)
        if self.metrics is not None:
            self.metrics.stage("frame3d", (time.perf_counter() - t0) / max(len(clouds), 1))
            self.metrics.frame(len(clouds))
        return out

    def _pc_callback(self, msg):
        for m, _ in self.process([msg]):
            self.pub.publish(m)
