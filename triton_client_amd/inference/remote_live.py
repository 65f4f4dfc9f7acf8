"""The remote engine's device path: the reference's client loop with every
per-frame numeric step on the GPU of the client.

The reference's camera callback (``communicator/ros_inference.py:117-175``)
decodes the ``CompressedImage`` with ``cv2.imdecode`` (:119-133), resizes and
normalises it on the CPU (:140-146, ``clients/preprocess/yolov5_preprocess.py:20-24``),
sends one blocking ``ModelInfer`` (:147), filters + NMSes the response on the CPU
(:148, ``clients/postprocess/yolov5_postprocess.py:28-125``), draws (:149-169) and
publishes (:173-175).  :class:`RemoteLiveCamera` keeps that contract — one
KServe request per frame, any KServe / Triton server — and moves the numeric
steps to the client's GPU:

* decode: C++ Huffman decode (``csrc/runtime/jpeg_entropy.cpp``, host threads,
  no GIL) into page-locked staging -> H2D -> HIP IDCT + colour
  (``csrc/kernels/jpeg.hip``) into a device frame batch; raw ``Image`` rows are
  gathered by C++ threads and uploaded;
* preprocess: K1 (``tca_image_preprocess``: stretch / letterbox, scaling, layout)
  -> the model input, one D2H into page-locked staging that the C++ wire encoder
  serialises from directly (``channel/wire.py``: no NumPy copy);
* postprocess: the response's output bytes -> page-locked batch -> one H2D ->
  K3 (``tca_yolo_filter_decoded``) + K4 sort / bitmask NMS with the box rescale
  to frame pixels fused in (YOLOv5, YOLOv4), or the server's final boxes
  (Detectron2) uploaded as they are;
* annotation: boxes and labels drawn on the resident frames
  (``tca_draw_annotations``), one D2H of the annotated frames into page-locked
  memory the published ``Image`` wraps without a copy.

Several driver workers may call :meth:`RemoteLiveCamera.process` at once: ingest,
preprocess and the RPCs of one batch overlap another's; only the postprocess +
annotation (which share the postprocess workspaces) is serialised.
"""
from __future__ import annotations

import ctypes
import logging
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from ..ops.image import draw_annotations_, preprocess
from ..ops.jpeg import GEOM_FIELDS, JpegGeometry
from ..ros import msgs
from ..utils.trace import trace_range
from .live import LiveCamera, _buffers, _is_compressed, _threads, gather_copy

log = logging.getLogger("triton_client_amd.remote_live")


class _Ingest:
    """One input kind + frame geometry: messages -> uint8 RGB frames [n, H, W, 3] on the GPU."""

    def __init__(self, kind: str, hw: Tuple[int, int], geo: Optional[JpegGeometry], device, threads: int):
        self.kind, self.hw, self.geo, self.device, self.threads = kind, hw, geo, device, threads
        if geo is not None:
            self.geom_rec = np.array([geo.width, geo.height, geo.nc, geo.hmax, geo.vmax, geo.mcux, geo.mcuy,
                                      *[v for hv in geo.sampling for v in hv], geo.nblocks, 0, 0], np.int32)

    def __call__(self, batch: Sequence) -> torch.Tensor:
        n, (H, W) = len(batch), self.hw
        dev = self.device
        frames = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
        if self.kind == "jpeg":
            g = self.geo
            coef = torch.empty((n, g.nblocks, 64), dtype=torch.int16, pin_memory=True)
            q = torch.empty((n, 192), dtype=torch.float32, pin_memory=True)
            geoms = np.zeros((n, GEOM_FIELDS), np.int32)
            status = np.zeros((n,), np.int32)
            datas = [m.data for m in batch]
            ptrs, keep = _buffers(datas)
            lens = (ctypes.c_int64 * n)(*[len(v) for v in keep])
            failed = _native.runtime().tca_jpeg_decode_batch(ptrs, lens, n, coef.data_ptr(), g.nblocks, q.data_ptr(),
                                                            geoms.ctypes.data, status.ctypes.data, self.threads)
            coef_d, q_d = coef.to(dev, non_blocking=True), q.to(dev, non_blocking=True)
            planes = torch.empty((n, g.plane_bytes), dtype=torch.uint8, device=dev)
            st = _native.stream_ptr(torch.cuda.current_stream(dev))
            _native.call("tca_jpeg_idct", coef_d.data_ptr(), q_d.data_ptr(), planes.data_ptr(), self.geom_rec.ctypes.data,
                         g.nblocks, g.plane_bytes, n, st)
            _native.call("tca_jpeg_color", planes.data_ptr(), frames.data_ptr(), self.geom_rec.ctypes.data,
                         g.plane_bytes, H * W * 3, n, st)
            for i in range(n):  # frames the entropy decoder hands to the host decoder
                if (failed and status[i]) or not np.array_equal(geoms[i], self.geom_rec):
                    rgb = torch.from_numpy(LiveCamera.host_rgb(datas[i], self.hw)).pin_memory()
                    frames[i].copy_(rgb, non_blocking=True)
            return frames
        host = torch.empty((n, H, W, 3), dtype=torch.uint8, pin_memory=True)
        hn = host.numpy()
        direct, srcs = [], []
        for i, m in enumerate(batch):
            if (not _is_compressed(m) and m.encoding == "rgb8" and m.step == 3 * W and len(m.data) >= H * W * 3):
                direct.append(i)
                srcs.append(m.data)
            else:
                hn[i] = LiveCamera.host_rgb(m, self.hw)
        gather_copy([host.data_ptr() + i * H * W * 3 for i in direct], srcs, [H * W * 3] * len(direct), self.threads)
        frames.copy_(host, non_blocking=True)
        return frames


class RemoteLiveCamera:
    """Camera messages -> (annotated ``Image``, detections [n, 6] in frame pixels)
    through a :class:`~triton_client_amd.inference.engines.RemoteDetector2D` whose
    client runs on a GPU (``--device``; ``auto`` picks the GPU when present)."""

    def __init__(self, det, threads: Optional[int] = None, thickness: int = 2):
        self.det, self.thickness = det, thickness
        self.device = det.device
        self.threads = threads or _threads()
        self._ingest: Dict[tuple, _Ingest] = {}
        self._names: Dict[tuple, Optional[torch.Tensor]] = {}
        self.lock = threading.Lock()       # postprocess workspaces + annotation
        self._mk = threading.Lock()        # ingest table
        self.stats = {"frames": 0, "batches": 0}

    # ------------------------------------------------------------------ pieces
    def _key(self, m):
        return LiveCamera._key(self, m)

    host_rgb = staticmethod(LiveCamera.host_rgb)

    def _ingest_for(self, key) -> _Ingest:
        ing = self._ingest.get(key)
        if ing is None:
            with self._mk:
                ing = self._ingest.get(key)
                if ing is None:
                    kind, hw, geo = key
                    ing = self._ingest[key] = _Ingest(kind, hw, geo, self.device, self.threads)
        return ing

    def _names_dev(self, names: Tuple[str, ...]) -> Optional[torch.Tensor]:
        if not names:
            return None
        t = self._names.get(names)
        if t is None:
            from ..utils.draw import names_table
            t = self._names[names] = torch.from_numpy(names_table(names)).to(self.device)
        return t

    def _model_input(self, frames: torch.Tensor):
        """Frames on the GPU -> (page-locked model inputs [n, ...model shape], xform)."""
        d = self.det
        x, xf = preprocess(frames, (d.h, d.w), d.mode2d, d.scaling, torch.float32, "NHWC" if d.nhwc else "NCHW")
        if d.nhwc:
            x = x.permute(0, 2, 3, 1)
        tdt = d._TORCH_OF.get(d.dtype, torch.float32)
        pin = torch.empty(x.shape, dtype=tdt, pin_memory=True)
        pin.copy_(x.to(tdt), non_blocking=True)
        return pin, xf

    def _rpc(self, inputs: torch.Tensor) -> list:
        """One KServe request per frame (the reference's contract), through the
        detector's wire and RPC mode; the raw wire encodes from the pinned rows."""
        d = self.det
        per = [inputs[i:i + 1] if d.batch_dim else inputs[i] for i in range(inputs.shape[0])]
        if d.wire == "raw" and d.mode != "stream":
            raws = [d._encode([(d.input_name, d.dtype, a)], d.requested, str(i)) for i, a in enumerate(per)]
            return d._send(raws)
        return d._run([[(d.input_name, d.dtype, a.numpy())] for a in per], d.requested)

    def _post(self, responses: list, xform):
        d = self.det
        post = d.post
        kw = {"conf_thres": d.conf_thres, "iou_thres": d.iou_thres, "xform": xform}
        if hasattr(post, "extract_boxes_device"):
            if "device" in post.extract_boxes_device.__code__.co_varnames:
                kw["device"] = self.device
            return post.extract_boxes_device(responses, **kw)
        from ..clients.postprocess.device import pack_host_detections

        per = []
        for r in responses:
            det = d._extract(r)
            if len(det):
                det[:, :4] = xform.unmap_boxes(det[:, :4])
            per.append(det)
        return pack_host_detections(per, self.device)

    # ------------------------------------------------------------------ one batch
    def run(self, key, batch: Sequence, draw: bool, names: Tuple[str, ...]) -> List[tuple]:
        n, (H, W) = len(batch), key[1]
        with trace_range("remote_ingest"):
            frames = self._ingest_for(key)(batch)
        with trace_range("remote_preprocess"):
            inputs, xf = self._model_input(frames)
            torch.cuda.current_stream(self.device).synchronize()  # the inputs are in host memory
        with trace_range("remote_rpc"):
            responses = self._rpc(inputs)
        with getattr(self.det.post, "lock", self.lock), trace_range("remote_postprocess"):
            res = self._post(responses, xf)
            if draw:
                draw_annotations_(frames, res.box, res.score, res.cls, res.count, self._names_dev(names),
                                  thickness=self.thickness)
            out = torch.empty((n, H, W, 3), dtype=torch.uint8, pin_memory=True)
            out.copy_(frames, non_blocking=True)
            host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in (res.box, res.score, res.cls,
                                                                                    res.count)]
            for h, t in zip(host, (res.box, res.score, res.cls, res.count)):
                h.copy_(t, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
        box, score, cls, cnt = [h.numpy() for h in host]
        fr = out.numpy()
        result = []
        for j, m in enumerate(batch):
            c = int(min(cnt[j], box.shape[1]))
            det = np.empty((c, 6), np.float32)
            det[:, :4] = box[j, :c, :4]
            det[:, 4] = score[j, :c]
            det[:, 5] = cls[j, :c]
            im = msgs.Image(header=m.header, height=H, width=W, encoding="rgb8", is_bigendian=0, step=3 * W,
                            data=memoryview(fr[j].reshape(-1)))  # zero-copy view of the pinned D2H buffer
            result.append((im, det))
        self.stats["frames"] += n
        self.stats["batches"] += 1
        return result

    def process(self, messages: Sequence, draw: bool = True, names: Optional[Sequence[str]] = None,
                max_batch: int = 32) -> List[tuple]:
        """-> [(Image, dets [n, 6] x1, y1, x2, y2, conf, cls in frame pixels)] in message order."""
        names = tuple(names or ())
        groups: Dict[tuple, List[int]] = {}
        for i, m in enumerate(messages):
            groups.setdefault(self._key(m), []).append(i)
        out: List[Optional[tuple]] = [None] * len(messages)
        for key, idx in groups.items():
            for s in range(0, len(idx), max_batch):
                chunk = idx[s:s + max_batch]
                for i, r in zip(chunk, self.run(key, [messages[i] for i in chunk], draw, names)):
                    out[i] = r
        return out
