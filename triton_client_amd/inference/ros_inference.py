"""Live 2D inference driver (reference ``communicator/ros_inference.py:25-175``).

Subscribes to the camera topic (``CompressedImage`` JPEG or raw ``Image``,
SURVEY Appendix A3), runs the engine (local MI355X pipeline or remote KServe
server), draws the boxes and publishes an annotated ``Image`` (rgb8) carrying
the *input* header (A4) — plus a ``vision_msgs/Detection2DArray`` on
``<pub_topic>/detections`` (the intent of ``utils/pred2ros_msg.py:21-52``).
An empty detection set still publishes the frame (fixes A5).

``batch > 1`` (or ``workers > 1``): the callback only enqueues; frames are
run as micro-batches (one engine call — one graph replay, or one DP scatter
over the node's GPUs — per batch) from a latest-wins window, and results are
re-published in ``header.seq`` order (:mod:`.batching`).
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import numpy as np

from ..ros import compat, msgs
from ..utils.draw import draw_detections
from ..utils.metrics import StageTimer
from .base_inference import BaseInference
from .engines import Detector2D, RemoteDetector2D


def decode_image_msg(msg) -> np.ndarray:
    """CompressedImage (jpeg/png) or Image → HxWx3 uint8 RGB (reference :119-133)."""
    if isinstance(msg, msgs.CompressedImage) or (hasattr(msg, "format") and not hasattr(msg, "encoding")):
        if "compressed" in msg.format or msg.format.lower() in ("jpeg", "jpg", "png"):
            return compat.jpeg_decode_rgb(msg.data)
    return compat.imgmsg_to_numpy(msg, "rgb8")


def detections_to_msg(dets: np.ndarray, header: msgs.Header, source: Optional[msgs.Image] = None) -> msgs.Detection2DArray:
    """Detection2DArray over dets [n, 6]; the Detection2D objects are built only
    if a subscriber reads ``detections`` (:class:`~triton_client_amd.ros.msgs.ArrayList`,
    columns ``{"dets": dets}``)."""
    dets = np.asarray(dets, np.float32).reshape(-1, 6)

    def build():
        src = msgs.Image(header=header) if source is None else source
        out = []
        for x1, y1, x2, y2, conf, c in dets.tolist():
            out.append(msgs.Detection2D(
                header=header, results=[msgs.ObjectHypothesisWithPose(id=int(c), score=conf)],
                bbox=msgs.BoundingBox2D(center=msgs.Pose2D((x1 + x2) / 2, (y1 + y2) / 2, 0.0), size_x=x2 - x1,
                                        size_y=y2 - y1),
                source_img=src))
        return out
    return msgs.Detection2DArray(header=header, detections=msgs.ArrayList(len(dets), build, {"dets": dets}))


class RosInference(BaseInference):
    def __init__(self, channel=None, client=None, engine: Optional[Detector2D] = None, params: Optional[dict] = None,
                 bus=None, letterbox: bool = False, conf_thres: float = 0.3, draw: bool = True,
                 publish_detections: bool = True, queue_size: Optional[int] = 1, metrics=None, mode: str = "sync",
                 wire: str = "raw", batch: int = 1, workers: int = 1):
        super().__init__(channel, client)
        self._params = params or {}
        self.engine = engine or RemoteDetector2D(channel, client, letterbox=letterbox, conf_thres=conf_thres,
                                                 mode=mode, wire=wire)
        self.class_names = list(getattr(self.engine, "names", []) or [])
        self.bus, self.draw, self.publish_detections = bus, draw, publish_detections
        self.queue_size, self.metrics = queue_size, metrics
        self.frames = 0
        self.sub = self.pub = self.det_pub = None
        self.batch, self.workers = max(1, batch), max(1, workers)
        self.runner = None

    # ------------------------------------------------------------------ run
    def start_inference(self, spin: bool = True, timeout: Optional[float] = None):
        p = self.params
        self.pub = compat.Publisher(p["pub_topic"], msgs.Image, queue_size=10, bus=self.bus)
        if self.publish_detections:
            self.det_pub = compat.Publisher(p["pub_topic"] + "/detections", msgs.Detection2DArray, queue_size=10,
                                            bus=self.bus)
        cb, qs = self._callback, self.queue_size
        if self.batch > 1 or self.workers > 1:
            from .batching import MicroBatchRunner
            self.runner = MicroBatchRunner(lambda ms: [(im, det) for im, det, _ in self.process(ms)], self._publish,
                                           batch=self.batch, workers=self.workers,
                                           capacity=max(self.queue_size or 0, 2 * self.batch * self.workers))
            cb, qs = self.runner.push, None  # the window is the (latest-wins) queue
        self.sub = compat.Subscriber(p["sub_topic"], msgs.CompressedImage, cb, queue_size=qs, bus=self.bus,
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

    def _publish(self, item) -> None:
        im, det = item
        self.pub.publish(im)
        if self.det_pub is not None:
            self.det_pub.publish(det)

    # ------------------------------------------------------------------ work
    def _live(self):
        """The engine's streaming device path (LocalDetector2D on a GPU), else None."""
        if not hasattr(self, "_live_exec"):
            fn = getattr(self.engine, "live", None)
            self._live_exec = fn() if callable(fn) else None
        return self._live_exec

    def process(self, images: Sequence) -> List[tuple]:
        """Messages → [(annotated Image msg, Detection2DArray, dets [n,6])]."""
        t0 = time.perf_counter()
        timer = StageTimer(self.metrics)
        live = self._live()
        if live is not None:  # device path: GPU decode, graph step, GPU annotation, zero-copy Image
            with timer("device"):
                res = live.process(images, draw=self.draw, names=self.class_names)
            with timer("messages"):
                out = [(im, detections_to_msg(d, m.header), d) for m, (im, d) in zip(images, res)]
            self.frames += len(images)
            if self.metrics is not None:
                self.metrics.stage("frame", (time.perf_counter() - t0) / max(len(images), 1))
                self.metrics.frame(len(images))
            return out
        with timer("decode"):
            rgb = [decode_image_msg(m) for m in images]
        gpu_draw = self.draw and hasattr(self.engine, "detect_annotated") and \
            getattr(getattr(self.engine, "device", None), "type", "cpu") == "cuda"
        with timer("detect"):
            if gpu_draw:  # rectangles drawn on the GPU (K15), labels below
                dets, drawn = self.engine.detect_annotated(rgb)
            else:
                dets, drawn = self.engine.detect(rgb), None
        out = []
        with timer("draw_publish"):
            for j, (m, img, d) in enumerate(zip(images, rgb, dets)):
                if drawn is not None:
                    img = draw_detections(drawn[j], d, self.class_names, rects=False)
                elif self.draw:
                    img = draw_detections(img.copy(), d, self.class_names)
                im = compat.numpy_to_imgmsg(img, "rgb8", header=m.header)
                out.append((im, detections_to_msg(d, m.header), d))
        self.frames += len(images)
        if self.metrics is not None:
            self.metrics.stage("frame", (time.perf_counter() - t0) / max(len(images), 1))
            self.metrics.frame(len(images))
        return out

    def _callback(self, msg):
        for im, det, _ in self.process([msg]):
            self.pub.publish(im)
            if self.det_pub is not None:
                self.det_pub.publish(det)
