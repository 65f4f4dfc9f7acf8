"""The live drivers' device path: sensor messages in, publishable results out.

The reference's product is its subscriber callback — one message, decode,
preprocess, one blocking ``ModelInfer``, NMS, draw, publish
(``communicator/ros_inference.py:117-175``; ``communicator/ros_inference3d.py:120-213``).
Here :class:`~triton_client_amd.inference.ros_inference.RosInference` /
:class:`~triton_client_amd.inference.ros_inference3d.RosInference3D` hand
micro-batches of messages to these executors, which keep the frames on the
device from ingest to the one D2H copy the publisher needs:

camera (:class:`LiveCamera`)
    ``CompressedImage`` JPEG: C++ Huffman decode (``csrc/runtime/jpeg_entropy.cpp``,
    host threads, no GIL) straight into a pinned slot -> H2D -> HIP IDCT +
    colour (``csrc/kernels/jpeg.hip``) into the pipeline's frame buffer.  Raw
    ``Image`` rgb8: the rows are gathered into the pinned slot by C++ threads
    (``csrc/runtime/host_copy.cpp``).  Then the captured YOLOv5 / YOLOv4 /
    Detectron step, and boxes + labels drawn on the resident frames
    (``csrc/kernels/draw.hip``); the annotated frames and the detections come
    back in one D2H into pinned memory that the published ``Image`` wraps
    without a copy.
LiDAR (:class:`LiveLidar`)
    ``PointCloud2`` payload bytes gathered into a pinned slot -> H2D -> the
    captured unpack / voxelise / network / NMS step -> one D2H of the result
    rows; the jsk ``BoundingBoxArray`` is built from those columns.

Both run on :class:`~triton_client_amd.pipelines.stream.StreamExecutor`: two
input sets, one captured graph per set, separate H2D / compute / D2H streams.
There is no engine-wide lock: several driver workers stage, submit and
collect batches concurrently; only the enqueue itself is serialised.
"""
from __future__ import annotations

import ctypes
import logging
import os
import threading
from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from ..ops.jpeg import GEOM_FIELDS, JpegGeometry, decode_pil, probe
from ..pipelines.stream import PinnedSlots, StreamExecutor
from ..ros import msgs

log = logging.getLogger("triton_client_amd.live")


def _threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def _buffers(bufs: Sequence) -> Tuple[ctypes.Array, list]:
    """void* array over bytes-like objects (no copy) + the views keeping them alive."""
    views = [np.frombuffer(b, np.uint8) for b in bufs]
    return (ctypes.c_void_p * len(views))(*[v.ctypes.data for v in views]), views


def gather_copy(dst_ptrs: Sequence[int], srcs: Sequence, sizes: Sequence[int], threads: int) -> None:
    """dst_ptrs[i] <- srcs[i][:sizes[i]] on C++ threads (GIL released)."""
    n = len(srcs)
    if n == 0:
        return
    sp, keep = _buffers(srcs)
    dp = (ctypes.c_void_p * n)(*dst_ptrs)
    nb = (ctypes.c_int64 * n)(*sizes)
    rc = _native.runtime().tca_host_gather_copy(n, dp, sp, nb, threads)
    del keep
    if rc:
        raise ValueError("tca_host_gather_copy: bad arguments")


# ============================================================================ camera
def _is_compressed(m) -> bool:
    return isinstance(m, msgs.CompressedImage) or (hasattr(m, "format") and not hasattr(m, "encoding"))


class _CameraEngine:
    """One frame geometry + input kind: a calibrated pipeline, its two captured
    graphs and a pool of pinned staging slots."""

    def __init__(self, live: "LiveCamera", kind: str, hw: Tuple[int, int], geo: Optional[JpegGeometry],
                 draw: bool, names: Tuple[str, ...], sample: np.ndarray):
        det = live.det
        self.live, self.kind, self.hw, self.geo, self.draw = live, kind, hw, geo, draw
        self.B, dev = det.B, det.device
        self.p = det._calibrated_pipeline(hw, sample)
        self.names_dev = None
        if draw and names:
            from ..utils.draw import names_table
            self.names_dev = torch.from_numpy(names_table(names)).to(dev)
        self.ex = StreamExecutor(self._step, [(self.p, "frames")], dev, graph=det.graph)
        H, W = hw
        if geo is not None:
            self.geom_rec = np.array([geo.width, geo.height, geo.nc, geo.hmax, geo.vmax, geo.mcux, geo.mcuy,
                                      *[v for hv in geo.sampling for v in hv], geo.nblocks, 0, 0], np.int32)
            self.coef_dev = [torch.empty((self.B, geo.nblocks, 64), dtype=torch.int16, device=dev)
                             for _ in range(self.ex.sets)]
            self.q_dev = [torch.empty((self.B, 192), dtype=torch.float32, device=dev) for _ in range(self.ex.sets)]
            self.planes = torch.empty((self.B, geo.plane_bytes), dtype=torch.uint8, device=dev)

        def make_slot():
            s = SimpleNamespace(frames=torch.empty((self.B, H, W, 3), dtype=torch.uint8).pin_memory())
            s.frames_np = s.frames.numpy()
            if geo is not None:
                s.coef = torch.empty((self.B, geo.nblocks, 64), dtype=torch.int16).pin_memory()
                s.q = torch.empty((self.B, 192), dtype=torch.float32).pin_memory()
                s.geoms = np.zeros((self.B, GEOM_FIELDS), np.int32)
                s.status = np.zeros((self.B,), np.int32)
            return s
        self.slots = PinnedSlots(live.slots, make_slot)

    def _step(self):
        """Capture-safe: the pipeline step, then boxes + labels onto the frames."""
        res = self.p.step()
        if self.draw:
            from ..ops.image import draw_annotations_
            draw_annotations_(self.p.frames, res.box, res.score, res.cls, res.count, self.names_dev,
                              thickness=self.live.thickness)
        return res

    # ------------------------------------------------------------------ host staging
    def _stage_jpeg(self, s, datas: List) -> List[int]:
        n, g = len(datas), self.geo
        ptrs, keep = _buffers(datas)
        lens = (ctypes.c_int64 * n)(*[len(v) for v in keep])
        failed = _native.runtime().tca_jpeg_decode_batch(
            ptrs, lens, n, s.coef.data_ptr(), g.nblocks, s.q.data_ptr(), s.geoms.ctypes.data, s.status.ctypes.data,
            self.live.threads)
        fb = []
        for i in range(n):
            if (failed and s.status[i]) or not np.array_equal(s.geoms[i], self.geom_rec):
                s.frames_np[i] = self.live.host_rgb(datas[i], self.hw)
                fb.append(i)
        return fb

    def _stage_frames(self, s, batch: Sequence) -> None:
        H, W = self.hw
        direct, srcs = [], []
        for i, m in enumerate(batch):
            if (not _is_compressed(m) and m.encoding == "rgb8" and m.step == 3 * W
                    and len(m.data) >= H * W * 3):
                direct.append(i)
                srcs.append(m.data)
            else:
                s.frames_np[i] = self.live.host_rgb(m, self.hw)
        frame = H * W * 3
        gather_copy([s.frames.data_ptr() + i * frame for i in direct], srcs, [frame] * len(direct),
                    self.live.threads)

    # ------------------------------------------------------------------ one batch
    def submit(self, batch: Sequence, out_frames: Optional[Sequence[torch.Tensor]] = None):
        """Stage ``batch`` (<= B messages of this engine's kind and geometry) and
        enqueue its device work; returns the pending batch for :meth:`finish`.
        ``out_frames``: page-locked [H, W, 3] host tensors (one per message) the
        annotated frames are copied into instead of a fresh pinned buffer."""
        n = len(batch)
        if not 0 < n <= self.B:
            raise ValueError(f"{n} frames for a batch of {self.B}")
        s = self.slots.acquire()
        ticket = None
        try:
            fb: List[int] = []
            if self.kind == "jpeg":
                fb = self._stage_jpeg(s, [m.data for m in batch])
            else:
                self._stage_frames(s, batch)
            if self.kind == "jpeg":
                def copies(k):
                    return [(self.coef_dev[k], s.coef[:n]), (self.q_dev[k], s.q[:n])]

                def pre(k):
                    g, st = self.geo, _native.stream_ptr(torch.cuda.current_stream())
                    out = self.ex.inputs[k][0]
                    _native.call("tca_jpeg_idct", self.coef_dev[k].data_ptr(), self.q_dev[k].data_ptr(),
                                 self.planes.data_ptr(), self.geom_rec.ctypes.data, g.nblocks, g.plane_bytes, n, st)
                    _native.call("tca_jpeg_color", self.planes.data_ptr(), out.data_ptr(), self.geom_rec.ctypes.data,
                                 g.plane_bytes, g.height * g.width * 3, n, st)
                    for i in fb:  # frames the entropy decoder handed to the host decoder
                        out[i].copy_(s.frames[i], non_blocking=True)
            else:
                def copies(k):
                    return [(self.ex.inputs[k][0], s.frames[:n])]
                pre = None
            if out_frames is not None:
                ticket = self.ex.submit(copies, pre, lambda k: [self.ex.inputs[k][0][i] for i in range(n)],
                                        extras_dst=list(out_frames))
            else:
                ticket = self.ex.submit(copies, pre, lambda k: [self.ex.inputs[k][0][:n]])
        finally:
            # the slot is read by the H2D (and the host-decoded frames by pre() on the compute
            # stream): free once the batch's last device work is done
            self.slots.release(s, ticket.done if ticket is not None else None)
        return SimpleNamespace(batch=batch, ticket=ticket, out_frames=out_frames)

    def finish(self, pend) -> List[tuple]:
        """-> [(Image, dets [n, 6])] of a submitted batch (waits for its D2H)."""
        ticket, batch = pend.ticket.wait(), pend.batch
        res = ticket.result()
        cnt = res.count.numpy()
        box, score, cls = res.box.numpy(), res.score.numpy(), res.cls.numpy()
        H, W = self.hw
        frames = [f.numpy() for f in ticket.extras] if pend.out_frames is not None else ticket.extras[0].numpy()
        out = []
        for j, m in enumerate(batch):
            c = int(min(cnt[j], box.shape[1]))
            d = np.empty((c, 6), np.float32)
            d[:, :4] = box[j, :c, :4]
            d[:, 4] = score[j, :c]
            d[:, 5] = cls[j, :c]
            im = msgs.Image(header=m.header, height=H, width=W, encoding="rgb8", is_bigendian=0, step=3 * W,
                            data=memoryview(frames[j].reshape(-1)))  # zero-copy view of the pinned D2H buffer
            out.append((im, d))
        return out

    def run(self, batch: Sequence) -> List[tuple]:
        return self.finish(self.submit(batch))

    def zero_stage(self) -> List[torch.Tensor]:
        """Result-shaped device zeros (an empty shard's part of a gather)."""
        if getattr(self, "_zero", None) is None:
            self._zero = [torch.zeros_like(t) for t in self.ex.stage[0]]
        return self._zero


class LiveCamera:
    """Camera messages -> (annotated ``Image``, detections [n, 6]) per message,
    for a :class:`~triton_client_amd.inference.engines.LocalDetector2D` on the GPU."""

    def __init__(self, det, slots: int = 4, threads: Optional[int] = None, thickness: int = 2):
        self.det, self.slots, self.thickness = det, slots, thickness
        self.threads = threads or _threads()
        self.engines: Dict[tuple, _CameraEngine] = {}
        self.lock = threading.Lock()

    @staticmethod
    def host_rgb(msg_or_data, hw: Optional[Tuple[int, int]] = None) -> np.ndarray:
        """Host decode for what the device path does not take (progressive JPEG,
        PNG, bgr8 / mono8 / padded rows): HxWx3 uint8 RGB."""
        from ..ros import compat
        if isinstance(msg_or_data, (bytes, bytearray, memoryview)):
            try:
                rgb = decode_pil(bytes(msg_or_data))
            except Exception as e:  # noqa: BLE001 - a corrupt frame must not end the stream
                log.warning("undecodable camera frame (%s): publishing it black", e)
                return np.zeros((*hw, 3), np.uint8)
        elif _is_compressed(msg_or_data):
            return LiveCamera.host_rgb(msg_or_data.data, hw)
        else:
            rgb = compat.imgmsg_to_numpy(msg_or_data, "rgb8")
        if hw is not None and rgb.shape[:2] != tuple(hw):
            raise ValueError(f"frame {rgb.shape[1]}x{rgb.shape[0]} in a {hw[1]}x{hw[0]} batch")
        return rgb

    def _key(self, m):
        if _is_compressed(m):
            try:
                geo = probe(m.data if isinstance(m.data, bytes) else bytes(m.data))
            except ValueError:
                geo = None
            if geo is not None and geo.gpu_ok:
                return ("jpeg", (geo.height, geo.width), geo)
            rgb = self.host_rgb(m)
            return ("frames", rgb.shape[:2], None)
        return ("frames", (int(m.height), int(m.width)), None)

    def _engine(self, key, draw: bool, names: Tuple[str, ...], sample_msg) -> _CameraEngine:
        k = (key, draw, names)
        eng = self.engines.get(k)
        if eng is None:
            with self.lock:
                eng = self.engines.get(k)
                if eng is None:
                    kind, hw, geo = key
                    sample = self.host_rgb(sample_msg, hw) if self.det.calibrate_target is not None else None
                    eng = self.engines[k] = _CameraEngine(self, kind, hw, geo, draw, names, sample)
        return eng

    def process(self, messages: Sequence, draw: bool = True, names: Optional[Sequence[str]] = None) -> List[tuple]:
        """-> [(Image, dets [n, 6] x1,y1,x2,y2,conf,cls in frame pixels)] in message order."""
        names = tuple(names or ())
        groups: Dict[tuple, List[int]] = {}
        for i, m in enumerate(messages):
            groups.setdefault(self._key(m), []).append(i)
        out: List[Optional[tuple]] = [None] * len(messages)
        B = self.det.B
        for key, idx in groups.items():
            eng = self._engine(key, draw, names, messages[idx[0]])
            for s in range(0, len(idx), B):
                chunk = idx[s:s + B]
                for i, r in zip(chunk, eng.run([messages[i] for i in chunk])):
                    out[i] = r
        return out


# ============================================================================ LiDAR
class _LidarEngine:
    def __init__(self, live: "LiveLidar", layout, max_points: int, sample):
        det = live.det
        self.live, self.layout = live, layout
        self.B, dev = det.B, det.device
        self.p = det._calibrated_pipeline(layout, max_points, sample)
        self.max_points, self.fb = self.p.max_points, self.p.frame_bytes
        self.ex = StreamExecutor(self.p.step, [(self.p, "data"), (self.p, "frame_n")], dev, graph=det.graph)

        def make_slot():
            s = SimpleNamespace(data=torch.empty((self.B * self.fb,), dtype=torch.uint8).pin_memory(),
                                n=torch.zeros((self.B,), dtype=torch.int32).pin_memory())
            s.n_np = s.n.numpy()
            return s
        self.slots = PinnedSlots(live.slots, make_slot)

    def submit(self, clouds: Sequence[msgs.PointCloud2]):
        n, fb, step = len(clouds), self.fb, self.layout.point_step
        if not 0 < n <= self.B:
            raise ValueError(f"{n} clouds for a batch of {self.B}")
        counts = [int(c.width * c.height) for c in clouds]
        sizes = [k * step for k in counts]
        for c, sz in zip(clouds, sizes):
            if len(c.data) < sz or sz > fb:
                raise ValueError(f"PointCloud2 of {c.width}x{c.height} points x {step} B has {len(c.data)} B of data "
                                 f"(slot {fb} B)")
        s = self.slots.acquire()
        ticket = None
        try:
            gather_copy([s.data.data_ptr() + j * fb for j in range(n)], [c.data for c in clouds], sizes,
                        self.live.threads)
            s.n_np[:] = 0
            s.n_np[:n] = counts

            def copies(k):
                d, nd = self.ex.inputs[k]
                return [(d[j * fb:j * fb + sz], s.data[j * fb:j * fb + sz]) for j, sz in enumerate(sizes) if sz] + \
                    [(nd, s.n)]
            ticket = self.ex.submit(copies)
        finally:
            self.slots.release(s, ticket.uploaded if ticket is not None else None)
        return SimpleNamespace(n=n, ticket=ticket)

    def finish(self, pend) -> List[dict]:
        return self.live.det._frames_out(pend.ticket.wait().result())[:pend.n]

    def run(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        return self.finish(self.submit(clouds))

    def zero_stage(self) -> List[torch.Tensor]:
        if getattr(self, "_zero", None) is None:
            self._zero = [torch.zeros_like(t) for t in self.ex.stage[0]]
        return self._zero


class LiveLidar:
    """PointCloud2 messages -> per-cloud {pred_boxes, pred_scores, pred_labels}
    (sensor frame) for a :class:`~triton_client_amd.inference.engines.LocalDetector3D`
    on the GPU."""

    def __init__(self, det, slots: int = 4, threads: Optional[int] = None):
        self.det, self.slots = det, slots
        self.threads = threads or _threads()
        self.engines: Dict[tuple, _LidarEngine] = {}
        self.lock = threading.Lock()

    def _engine(self, layout, npts: int, sample) -> _LidarEngine:
        key = (layout.point_step, layout.offsets, layout.dtypes)
        eng = self.engines.get(key)
        if eng is None or eng.max_points < npts:
            with self.lock:
                eng = self.engines.get(key)
                if eng is None or eng.max_points < npts:
                    maxp = self.det.max_points
                    while maxp < npts:
                        maxp *= 2
                    eng = self.engines[key] = _LidarEngine(self, layout, maxp, sample)
        return eng

    def process(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        from ..ros.compat import cloud_layout

        groups: Dict[tuple, List[int]] = {}
        lays = {}
        for i, c in enumerate(clouds):
            lay = cloud_layout(c)
            k = (lay.point_step, lay.offsets, lay.dtypes)
            lays[k] = lay
            groups.setdefault(k, []).append(i)
        out: List[Optional[dict]] = [None] * len(clouds)
        B = self.det.B
        for k, idx in groups.items():
            npts = max(clouds[i].width * clouds[i].height for i in idx)
            eng = self._engine(lays[k], npts, clouds[idx[0]])
            for s in range(0, len(idx), B):
                chunk = idx[s:s + B]
                for i, r in zip(chunk, eng.run([clouds[i] for i in chunk])):
                    out[i] = r
        return out
