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

Shared-memory wires (``--wire shm`` / ``devshm``, reference
``communicator/channel/grpc_channel.py:26-30,73-78`` for the RPC it replaces): K1 writes
each frame's model input straight into its slot of the client's registered region and the
request carries only region references; the server writes the outputs back into the same
slot.  With ``devshm`` the region is a device allocation the server maps by HIP IPC handle:
the input never leaves the GPU, and K3/K4 read the decoded YOLOv5 output where the server
wrote it -- no tensor crosses host memory.

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
        self._tl = threading.local()       # shared-memory wires: each worker thread's own region
        self._regions: list = []

    # ------------------------------------------------------------------ shared-memory wires
    def _region(self, n: int):
        """This thread's registered region of >= n request slots (input + requested outputs each)."""
        from .engines import _new_region
        st = getattr(self._tl, "shm", None)
        if st is None or st[-1] < n:
            d = self.det
            if st is not None:
                try:
                    st[0].unregister(d.channel)
                finally:
                    st[0].close()
                    self._regions.remove(st[0])
            slot, in_shape, in_dt, layout = d._shm_layout()
            nslots = max(n, 8)
            region = _new_region(d.wire, slot * nslots, self.device)
            region.register(d.channel)
            self._regions.append(region)
            st = self._tl.shm = (region, slot, in_shape, in_dt, layout, nslots)
        return st

    def close(self) -> None:
        """Unregister and free every worker's shared-memory region."""
        for r in self._regions:
            try:
                r.unregister(self.det.channel)
            except Exception:  # noqa: BLE001 - the server may be gone already
                pass
            r.close()
        self._regions = []
        self._tl = threading.local()

    @staticmethod
    def _slots(region, slot: int, off: int, dtype, shape, n: int) -> torch.Tensor:
        """[n, *shape] view of the same tensor in n consecutive slots of a device region."""
        tdt = torch.from_numpy(np.empty(0, np.dtype(dtype))).dtype
        isz = np.dtype(dtype).itemsize
        base = region.alloc.tensor.view(tdt)
        inner = [int(np.prod(shape[i + 1:], dtype=np.int64)) for i in range(len(shape))]
        return base.as_strided((n,) + tuple(shape), (slot // isz,) + tuple(inner), off // isz)

    def _rpc_shm(self, x: torch.Tensor, n: int):
        """Model inputs [n, ...] on the GPU -> their slots; one request per frame carrying
        only region references; -> (region, slot, layout) once every response is in."""
        from ..channel.shm import shm_params
        from ..proto import service_pb2 as pb

        d = self.det
        region, slot, in_shape, in_dt, layout, _ = self._region(n)
        tdt = d._TORCH_OF.get(d.dtype, torch.float32)
        with trace_range("remote_shm_input"):
            xs = x.to(tdt).reshape((n,) + tuple(in_shape))
            if d.wire == "devshm":
                self._slots(region, slot, 0, in_dt, in_shape, n).copy_(xs)  # device to device, one kernel
            else:
                for k in range(n):  # D2H into the page-locked mapping
                    torch.from_numpy(region.view(k * slot, in_dt, in_shape)).copy_(xs[k], non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()  # complete before the server reads it
        ch = d.channel
        nin = int(np.prod(in_shape)) * np.dtype(in_dt).itemsize
        futs = []
        for k in range(n):
            req = pb.ModelInferRequest(model_name=ch.model_name, model_version=ch.model_version, id=str(k))
            t = req.inputs.add(name=d.input_name, datatype=d.dtype, shape=list(in_shape))
            shm_params(t, region.key, k * slot, nin)
            for name, o, b in layout:
                shm_params(req.outputs.add(name=name), region.key, k * slot + o, b)
            futs.append(ch._grpc_stub.ModelInferRaw.future(req.SerializeToString(), timeout=ch.timeout_s))
        resps = [pb.ModelInferResponse.FromString(f.result()) for f in futs]
        return region, slot, layout, resps

    def _post_shm(self, region, slot: int, layout, resps, n: int, xf):
        """Detections from the outputs the server wrote into the slots."""
        from ..channel.wire import ParsedResponse
        from ..proto import KSERVE_TO_NP
        from .engines import _device_output_to_host

        d = self.det
        post = d.post
        offs = {name: o for name, o, _ in layout}
        t0 = resps[0].outputs[0] if resps and len(resps[0].outputs) else None
        if (d.wire == "devshm" and t0 is not None and len(resps[0].outputs) == 1 and t0.datatype == "FP32"
                and len(t0.shape) == 3 and int(t0.shape[0]) == 1 and hasattr(post, "_post")
                and all(tuple(r.outputs[0].shape) == tuple(t0.shape) for r in resps)):
            # YOLOv5: K3 + K4 read the decoded output in the device region (one D2D gather of the slots)
            N, no = int(t0.shape[1]), int(t0.shape[2])
            pred = self._slots(region, slot, offs[t0.name], np.float32, (N, no), n).contiguous()
            pp = post._post(no - 5, d.conf_thres, d.iou_thres, None, False, False, 300, self.device)
            return pp.filter_decoded(pred, xf)
        prs = []
        for k, r in enumerate(resps):
            pr = ParsedResponse()
            pr.model_name = r.model_name
            for t in r.outputs:
                a = region.view(k * slot + offs[t.name], KSERVE_TO_NP[t.datatype], tuple(t.shape))
                if isinstance(a, torch.Tensor):
                    a = _device_output_to_host(a, d.conf_thres)
                pr.outputs[t.name] = a
                pr.datatypes[t.name] = t.datatype
                pr.order.append(t.name)
            prs.append(pr)
        return self._post(prs, xf)

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
        d = self.det
        with trace_range("remote_ingest"):
            frames = self._ingest_for(key)(batch)
        if d.wire in ("shm", "devshm"):
            with trace_range("remote_preprocess"):
                x, xf = preprocess(frames, (d.h, d.w), d.mode2d, d.scaling, torch.float32,
                                   "NHWC" if d.nhwc else "NCHW")
                if d.nhwc:
                    x = x.permute(0, 2, 3, 1)
            with trace_range("remote_rpc"):
                region, slot, layout, resps = self._rpc_shm(x, n)
            post_fn = lambda: self._post_shm(region, slot, layout, resps, n, xf)  # noqa: E731
        else:
            with trace_range("remote_preprocess"):
                inputs, xf = self._model_input(frames)
                torch.cuda.current_stream(self.device).synchronize()  # the inputs are in host memory
            with trace_range("remote_rpc"):
                responses = self._rpc(inputs)
            post_fn = lambda: self._post(responses, xf)  # noqa: E731
        with getattr(self.det.post, "lock", self.lock), trace_range("remote_postprocess"):
            res = post_fn()
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
