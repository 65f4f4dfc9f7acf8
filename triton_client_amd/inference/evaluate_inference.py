"""Accuracy evaluation with Prometheus export (reference ``communicator/evaluate_inference.py:26-446``).

Subscribes to the image topic and the ground-truth ``Detection2DArray``
topic, runs the detector on every image, and computes COCO-style metrics
(:mod:`..utils.evaluation`) that are exported as Prometheus ``Summary``
metrics ``precision``, ``recall``, ``ap``, ``fone`` and ``ap_class`` on
port 7658 — the same names and port as the reference.

Fixed relative to the reference:

* predictions and ground truth are joined on ``header.seq``.  The ground
  truth's seq is that of its ``source_img`` header.  The reference instead
  zipped two lists filled by independent threads;
* completion is detected, not waited for.  The evaluator finishes when a seq
  repeats (the bag looped, as in the reference), when :meth:`finish` is
  called, or at the end of :meth:`evaluate_bag`.  There is no fixed
  ``sleep(20)``;
* AP is computed over the statistics of all matched frames.  The reference
  computed it per message.

The ground-truth boxes are centre/size in original image pixels and are
converted to corner form (xyxy), as in the reference (:350-398).
Predictions are scaled back to the original frame by the engine.
"""
from __future__ import annotations

import threading
from typing import Optional

import numpy as np

from ..ros import compat, msgs
from ..ros.bag import Bag
from ..utils.evaluation import DetectionEvaluator, EvalSummary
from .base_inference import BaseInference
from .engines import Detector2D, RemoteDetector2D
from .ros_inference import decode_image_msg


def gt_from_msg(msg: msgs.Detection2DArray) -> tuple:
    """→ (seq, [n, 6] x1,y1,x2,y2,score,cls)."""
    g = np.zeros((len(msg.detections), 6), np.float64)
    for i, d in enumerate(msg.detections):
        r = d.results[0] if d.results else msgs.ObjectHypothesisWithPose()
        g[i] = [d.bbox.center.x - d.bbox.size_x / 2, d.bbox.center.y - d.bbox.size_y / 2,
                d.bbox.center.x + d.bbox.size_x / 2, d.bbox.center.y + d.bbox.size_y / 2, r.score, r.id]
    seq = msg.detections[0].source_img.header.seq if msg.detections else msg.header.seq
    return seq, g


class EvaluateInference(BaseInference):
    def __init__(self, channel=None, client=None, engine: Optional[Detector2D] = None, params: Optional[dict] = None,
                 bus=None, metrics_port: Optional[int] = 7658, conf_thres: float = 0.001, letterbox: bool = False,
                 class_names=None):
        super().__init__(channel, client)
        self._params = params or {}
        self.engine = engine or RemoteDetector2D(channel, client, letterbox=letterbox, conf_thres=conf_thres)
        self.class_names = class_names or list(getattr(self.engine, "names", []) or [])
        self.bus = bus
        self.evaluator = DetectionEvaluator()
        self.metrics = None
        if metrics_port is not None:
            from ..utils.metrics import EvalMetrics

            self.metrics = EvalMetrics(metrics_port)
        self.img_processed = self.gt_processed = False
        self.done = threading.Event()
        self._lock = threading.Lock()
        self.summary: Optional[EvalSummary] = None
        self.img_sub = self.gt_sub = None

    # ------------------------------------------------------------------ live
    def start_inference(self, spin: bool = True, timeout: Optional[float] = None):
        p = self.params
        self.img_sub = compat.Subscriber(p["sub_topic"], msgs.Image, self.image_callback, queue_size=None,
                                         bus=self.bus)
        self.gt_sub = compat.Subscriber(p["gt_topic"], msgs.Detection2DArray, self.gt_callback, queue_size=None,
                                        bus=self.bus)
        if spin:
            self.done.wait(timeout)
            return self.finish()

    def image_callback(self, msg):
        seq = msg.header.seq
        with self._lock:
            if seq in self.evaluator.preds:  # bag looped: images are complete
                self.img_processed = True
                self._maybe_done()
                return
        d = self.engine.detect([decode_image_msg(msg)])[0]
        with self._lock:
            self.evaluator.add_prediction(seq, d)

    def gt_callback(self, msg):
        seq, g = gt_from_msg(msg)
        with self._lock:
            if seq in self.evaluator.gts:
                self.gt_processed = True
                self._maybe_done()
                return
            self.evaluator.add_ground_truth(seq, g)

    def _maybe_done(self):
        if self.img_processed and self.gt_processed:
            self.done.set()

    # ------------------------------------------------------------------ offline
    def evaluate_bag(self, bagfile: str, batch: int = 8) -> EvalSummary:
        """Evaluate the sensor + ground-truth topics of a bag.  Images are run
        ``batch`` at a time."""
        p = self.params
        pending = []
        with Bag(bagfile) as bag:
            for topic, m, _ in bag.read_messages(topics=[p["sub_topic"], p["gt_topic"]]):
                if topic == p["gt_topic"]:
                    seq, g = gt_from_msg(m)
                    self.evaluator.add_ground_truth(seq, g)
                    continue
                pending.append(m)
                if len(pending) == batch:
                    self._run(pending)
                    pending = []
        if pending:
            self._run(pending)
        return self.finish()

    def _run(self, images):
        for m, d in zip(images, self.engine.detect([decode_image_msg(m) for m in images])):
            self.evaluator.add_prediction(m.header.seq, d)

    # ------------------------------------------------------------------ metrics
    def calculate_metrics(self) -> EvalSummary:
        with self._lock:
            s = self.evaluator.summary()
        if self.metrics is not None and getattr(self.metrics, "reg", None) is not None:
            for v in s.precision:
                self.metrics.p_summary.observe(float(v))
            for v in s.recall:
                self.metrics.r_summary.observe(float(v))
            for v in s.ap[:, 0] if len(s.ap) else []:
                self.metrics.ap_summary.observe(float(v))
            for v in s.f1:
                self.metrics.f1_summary.observe(float(v))
            for v in s.classes:
                self.metrics.ap_class_summary.observe(float(v))
        return s

    def finish(self) -> EvalSummary:
        for sub in (self.img_sub, self.gt_sub):
            if sub is not None:
                sub.unregister()
        self.img_sub = self.gt_sub = None
        self.summary = self.calculate_metrics()
        return self.summary
