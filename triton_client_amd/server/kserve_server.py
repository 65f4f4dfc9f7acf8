"""In-process / standalone KServe-v2 (Triton-protocol) gRPC server.

Replaces the external Triton server the reference talks to
(``README.md:62-67``; gRPC :8001, metrics :8002).  Implements
``GRPCInferenceService`` with generic handlers over the runtime-built
protobuf types (``triton_client_amd.proto``): ServerLive/Ready, ModelReady,
ServerMetadata, ModelMetadata, ModelConfig, ModelInfer, ModelStreamInfer,
ModelStatistics, RepositoryIndex/Load/Unload.  The same server doubles as
the test backend with an optional fault injector (delay /
drop / corrupt — SURVEY §5.3) and exports Triton-named Prometheus metrics.

Run standalone::

    python -m triton_client_amd.server --models YOLOv5nCOCO,pointpillar_kitti --port 8001
"""
from __future__ import annotations

import random
import threading
import time
from concurrent import futures
from dataclasses import dataclass
from typing import Dict, List, Optional

import grpc
import numpy as np

from ..proto import KSERVE_TO_NP, SERVICE, service_pb2 as pb
from .model import PROFILE, InferError, ServedModel
from .repository import ModelRepository

_BF16 = "BF16"


@dataclass
class FaultInjector:
    delay_s: float = 0.0
    drop_rate: float = 0.0
    corrupt_rate: float = 0.0
    seed: int = 0

    def __post_init__(self):
        self._rng = random.Random(self.seed)
        self._lock = threading.Lock()

    def roll(self, p: float) -> bool:
        if p <= 0:
            return False
        with self._lock:
            return self._rng.random() < p


def _np_dtype(dt: str):
    if dt == _BF16:
        return np.dtype(np.uint16)
    return np.dtype(KSERVE_TO_NP[dt])


def _kserve_dtype(a: np.ndarray) -> str:
    from ..proto import NP_TO_KSERVE
    return NP_TO_KSERVE[str(a.dtype)]


def decode_inputs(req, shm=None) -> Dict[str, np.ndarray]:
    """Inputs of a protobuf ModelInferRequest: shared-memory references become
    views of the registered region, raw contents views of the message (raw
    contents are indexed over the inputs that carry no region), else the
    typed contents."""
    from .shm import tensor_shm
    out = {}
    raw = list(req.raw_input_contents)
    k = 0
    for t in req.inputs:
        shape = tuple(int(s) for s in t.shape)
        ref = tensor_shm(t.parameters)
        if ref is not None:
            if shm is None:
                raise InferError("shared memory inputs are not supported by this server")
            region, off, nbytes = ref
            dt = _np_dtype(t.datatype)
            if nbytes != int(np.prod(shape)) * dt.itemsize:
                raise InferError(f"input '{t.name}': {nbytes} shared memory bytes do not match shape {list(shape)}")
            out[t.name] = shm.get(region).view(off, nbytes, dt, shape)
            continue
        i, k = k, k + 1
        if i < len(raw) and raw:
            a = np.frombuffer(raw[i], dtype=_np_dtype(t.datatype))
        else:  # typed contents
            c = t.contents
            src = {"FP32": c.fp32_contents, "FP64": c.fp64_contents, "INT32": c.int_contents,
                   "INT64": c.int64_contents, "UINT32": c.uint_contents, "UINT64": c.uint64_contents,
                   "BOOL": c.bool_contents}.get(t.datatype)
            if src is None:
                raise InferError(f"unsupported typed contents for {t.datatype}")
            a = np.asarray(src, dtype=_np_dtype(t.datatype))
        if a.size != int(np.prod(shape)):
            raise InferError(f"input '{t.name}': {a.size} elements do not match shape {list(shape)}")
        out[t.name] = a.reshape(shape)
    return out


def request_regions(req) -> List[str]:
    """Names of the shared-memory regions a request's inputs and outputs reference."""
    from .shm import tensor_shm
    names = []
    for t in list(req.inputs) + list(req.outputs):
        ref = tensor_shm(t.parameters)
        if ref is not None:
            names.append(ref[0])
    return names


def output_slices(req, shm) -> Optional[Dict[str, np.ndarray]]:
    """{output name: uint8 view of its shared-memory slice} for the outputs a request
    asks to receive in shared memory (None: none does)."""
    from .shm import tensor_shm
    if shm is None:
        return None
    out = {}
    for o in req.outputs:
        ref = tensor_shm(o.parameters)
        if ref is not None:
            region, off, nbytes = ref
            out[o.name] = shm.get(region).view(off, nbytes, np.uint8, (nbytes,))
    return out or None


def encode_response(model: ServedModel, req, outputs: Dict[str, np.ndarray], corrupt: bool = False, shm=None):
    """Protobuf response; an output requested into a shared-memory region is
    written there and answered with its shape / datatype (and the region
    parameters) but no raw contents, as Triton does."""
    from .shm import tensor_shm
    resp = pb.ModelInferResponse(model_name=model.name, model_version=model.version, id=req.id)
    names = [o.name for o in req.outputs] or list(outputs.keys())
    params = {o.name: o.parameters for o in req.outputs}
    for n in names:
        if n not in outputs:
            raise InferError(f"unknown output '{n}' for model '{model.name}'")
        a = outputs[n]
        ref = tensor_shm(params[n]) if n in params else None
        reg = shm.get(ref[0]) if (ref is not None and shm is not None) else None
        if reg is not None and reg.device and getattr(a, "is_cuda", False):
            # device output for a device region: written there by the model (or copied on the device)
            import torch
            dt = np.dtype(str(a.dtype).replace("torch.", ""))
            t = resp.outputs.add(name=n, datatype=_kserve_dtype(np.empty(0, dt)))
            t.shape.extend(a.shape)
            region, off, nbytes = ref
            size = a.numel() * a.element_size()
            if size > nbytes:
                raise InferError(f"output '{n}': {size} bytes exceed the {nbytes}-byte shared memory slice")
            dst = reg.view(off, size, dt, tuple(a.shape))
            if corrupt:
                dst.zero_()
            elif dst.data_ptr() != a.data_ptr():
                dst.copy_(a)
                torch.cuda.current_stream(dst.device).synchronize()
            for key in ("shared_memory_region", "shared_memory_offset", "shared_memory_byte_size"):
                if key in params[n]:
                    t.parameters[key].CopyFrom(params[n][key])
            continue
        if getattr(a, "is_cuda", False):
            a = a.cpu()
        a = np.ascontiguousarray(a.numpy() if hasattr(a, "numpy") and not isinstance(a, np.ndarray) else a)
        t = resp.outputs.add(name=n, datatype=_kserve_dtype(a))
        t.shape.extend(a.shape)
        if ref is not None:
            if shm is None:
                raise InferError("shared memory outputs are not supported by this server")
            region, off, nbytes = ref
            if a.nbytes > nbytes:
                raise InferError(f"output '{n}': {a.nbytes} bytes exceed the {nbytes}-byte shared memory slice")
            dst = shm.get(region).view(off, a.nbytes, a.dtype, a.shape)
            if corrupt:
                dst[...] = 0
            elif reg is not None and reg.device:
                import torch
                dst.copy_(torch.from_numpy(a))
                torch.cuda.current_stream(dst.device).synchronize()
            elif dst.ctypes.data != a.ctypes.data:  # not already written there by the device
                np.copyto(dst, a)
            for key in ("shared_memory_region", "shared_memory_offset", "shared_memory_byte_size"):
                if key in params[n]:
                    t.parameters[key].CopyFrom(params[n][key])
            continue
        b = a.tobytes()
        if corrupt and len(b):
            b = bytes(len(b))  # zeroed payload: detectable by clients, keeps the shape contract
        resp.raw_output_contents.append(b)
    return resp


class GRPCInferenceServicer:
    def __init__(self, repo: ModelRepository, fault: Optional[FaultInjector] = None, metrics=None,
                 server_name: str = "triton_client_amd", version: str = "0.1.0"):
        self.repo = repo
        self.fault = fault or FaultInjector()
        self.metrics = metrics
        self.server_name, self.version = server_name, version
        from .shm import SharedMemoryRegistry
        dev_id = None
        try:
            import torch
            d = torch.device(getattr(repo, "device", "cpu") or "cpu")
            if d.type == "cuda" and torch.cuda.is_available():
                dev_id = d.index if d.index is not None else torch.cuda.current_device()
        except Exception:  # noqa: BLE001 - a CPU-only server has no device regions to check
            dev_id = None
        self.shm = SharedMemoryRegistry(device_id=dev_id)

    # -------------------------------------------------------------- health / metadata
    def ServerLive(self, req, ctx):
        return pb.ServerLiveResponse(live=True)

    def ServerReady(self, req, ctx):
        return pb.ServerReadyResponse(ready=self.repo.all_ready())

    def ModelReady(self, req, ctx):
        m = self.repo.get(req.name, req.version)
        return pb.ModelReadyResponse(ready=bool(m and m.ready))

    def ServerMetadata(self, req, ctx):
        return pb.ServerMetadataResponse(name=self.server_name, version=self.version,
                                         extensions=["classification", "model_repository", "statistics",
                                                     "binary_tensor_data", "schedule_policy", "system_shared_memory"])

    def _model(self, name, version, ctx) -> ServedModel:
        m = self.repo.get(name, version)
        if m is None:
            ctx.abort(grpc.StatusCode.NOT_FOUND, f"Request for unknown model: '{name}' is not found")
        if not m.ready:
            ctx.abort(grpc.StatusCode.UNAVAILABLE, f"Request for unknown model: '{name}' is not ready")
        return m

    def ModelMetadata(self, req, ctx):
        return self._model(req.name, req.version, ctx).metadata()

    def ModelConfig(self, req, ctx):
        return pb.ModelConfigResponse(config=self._model(req.name, req.version, ctx).config())

    def ModelStatistics(self, req, ctx):
        resp = pb.ModelStatisticsResponse()
        for m in self.repo.models(req.name or None):
            st = m.stats
            ms = resp.model_stats.add(name=m.name, version=m.version, last_inference=st.last_inference_ms,
                                      inference_count=st.inference_count, execution_count=st.execution_count)
            ms.inference_stats.success.count = st.inference_count
            ms.inference_stats.success.ns = st.success_ns
            ms.inference_stats.fail.count = st.fail_count
            ms.inference_stats.compute_infer.count = st.execution_count
            ms.inference_stats.compute_infer.ns = st.compute_ns
        return resp

    def RepositoryIndex(self, req, ctx):
        resp = pb.RepositoryIndexResponse()
        for name, state in self.repo.index():
            if req.ready and state != "READY":
                continue
            resp.models.add(name=name, version="1", state=state)
        return resp

    def RepositoryModelLoad(self, req, ctx):
        try:
            self.repo.load(req.model_name)
        except KeyError as e:
            ctx.abort(grpc.StatusCode.NOT_FOUND, str(e))
        return pb.RepositoryModelLoadResponse()

    def RepositoryModelUnload(self, req, ctx):
        try:
            self.repo.unload(req.model_name)
        except InferError as e:  # a batch stuck on the device: the model stays loaded, not ready
            ctx.abort(grpc.StatusCode.DEADLINE_EXCEEDED, str(e))
        return pb.RepositoryModelUnloadResponse()

    # -------------------------------------------------------------- inference
    def _infer(self, req, ctx):
        t0 = time.perf_counter()
        m = self._model(req.model_name, req.model_version, ctx)
        if self.fault.delay_s:
            time.sleep(self.fault.delay_s)
        if self.fault.roll(self.fault.drop_rate):
            ctx.abort(grpc.StatusCode.UNAVAILABLE, "fault injection: dropped request")
        leased = []
        try:
            # device regions stay mapped until this request's batch has run and its response is
            # encoded, even if the client (or another one) unregisters them meanwhile
            leased = self.shm.lease(request_regions(req))
            inputs = decode_inputs(req, self.shm)
            if PROFILE.on:
                PROFILE.add("pb.decode_inputs", time.perf_counter() - t0)
            corrupt = self.fault.roll(self.fault.corrupt_rate)
            resp = m(inputs, [o.name for o in req.outputs],
                     encode=lambda outputs: encode_response(m, req, outputs, corrupt=corrupt, shm=self.shm),
                     out_dst=None if corrupt else output_slices(req, self.shm))
        except InferError as e:
            if self.metrics:
                self.metrics.request(m.name, False, time.perf_counter() - t0)
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        finally:
            self.shm.release(leased)
        if self.metrics:
            self.metrics.request(m.name, True, time.perf_counter() - t0)
        return resp

    def ModelInfer(self, req, ctx):
        return self._infer(req, ctx)

    # ------------------------------------------------- system shared memory
    def SystemSharedMemoryStatus(self, req, ctx):
        resp = pb.SystemSharedMemoryStatusResponse()
        try:
            regions = self.shm.status(req.name)
        except InferError as e:
            ctx.abort(grpc.StatusCode.NOT_FOUND, str(e))
        for r in regions:
            st = resp.regions[r.name]
            st.name, st.key, st.offset, st.byte_size = r.name, r.key, r.offset, r.byte_size
        return resp

    def SystemSharedMemoryRegister(self, req, ctx):
        try:
            self.shm.register(req.name, req.key, int(req.offset), int(req.byte_size))
        except InferError as e:
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        return pb.SystemSharedMemoryRegisterResponse()

    def SystemSharedMemoryUnregister(self, req, ctx):
        self.shm.unregister(req.name, device=False)
        return pb.SystemSharedMemoryUnregisterResponse()

    # ------------------------------------------------- device shared memory (HIP IPC)
    def CudaSharedMemoryStatus(self, req, ctx):
        resp = pb.CudaSharedMemoryStatusResponse()
        try:
            regions = self.shm.status(req.name, device=True)
        except InferError as e:
            ctx.abort(grpc.StatusCode.NOT_FOUND, str(e))
        for r in regions:
            st = resp.regions[r.name]
            st.name, st.device_id, st.byte_size = r.name, r.device_id, r.byte_size
        return resp

    def CudaSharedMemoryRegister(self, req, ctx):
        try:
            self.shm.register_device(req.name, bytes(req.raw_handle), int(req.device_id), int(req.byte_size))
        except InferError as e:
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        return pb.CudaSharedMemoryRegisterResponse()

    def CudaSharedMemoryUnregister(self, req, ctx):
        self.shm.unregister(req.name, device=True)
        return pb.CudaSharedMemoryUnregisterResponse()

    def ModelInferBytes(self, data: bytes, ctx) -> bytes:
        """ModelInfer on the raw wire bytes through the C++ codec: inputs are
        views into the request (no protobuf objects, no tensor copies until
        the model stages them for the device), the response is written
        straight from the output tensors."""
        from ..channel.wire import encode_response, parse_request

        t0 = time.perf_counter()
        try:
            req = parse_request(data)
        except ValueError as e:
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        if PROFILE.on:
            PROFILE.add("wire.parse", time.perf_counter() - t0)
        if req.has_params:  # shared-memory references: a small message, the protobuf path reads them
            t1 = time.perf_counter()
            pr = pb.ModelInferRequest.FromString(data)
            t2 = time.perf_counter()
            out = self._infer(pr, ctx)
            t3 = time.perf_counter()
            out = out.SerializeToString()
            if PROFILE.on:
                PROFILE.add("pb.from_string", t2 - t1)
                PROFILE.add("pb.infer", t3 - t2)
                PROFILE.add("pb.serialize", time.perf_counter() - t3)
                PROFILE.add("request_total", time.perf_counter() - t0)
            return out
        m = self._model(req.model_name, req.model_version, ctx)
        if self.fault.delay_s:
            time.sleep(self.fault.delay_s)
        if self.fault.roll(self.fault.drop_rate):
            ctx.abort(grpc.StatusCode.UNAVAILABLE, "fault injection: dropped request")
        try:
            for name, a in req.inputs.items():
                if a.size == 0 and 0 not in a.shape:
                    raise InferError(f"input '{name}': no raw contents")
            corrupt = self.fault.roll(self.fault.corrupt_rate)

            def encode(outputs):
                names = req.outputs or list(outputs.keys())
                for n in names:
                    if n not in outputs:
                        raise InferError(f"unknown output '{n}' for model '{m.name}'")
                outs = [(n, np.zeros(tuple(outputs[n].shape), np.asarray(outputs[n]).dtype) if corrupt else outputs[n])
                        for n in names]
                return encode_response(m.name, outs, m.version, req.id)
            resp = m(req.inputs, req.outputs, encode=encode)
        except InferError as e:
            if self.metrics:
                self.metrics.request(m.name, False, time.perf_counter() - t0)
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        if self.metrics:
            self.metrics.request(m.name, True, time.perf_counter() - t0)
        if PROFILE.on:
            PROFILE.add("request_total", time.perf_counter() - t0)
        return resp

    def ModelStreamInfer(self, req_iter, ctx):
        for req in req_iter:
            try:
                resp = self._infer(req, _StreamCtx(ctx))
                yield pb.ModelStreamInferResponse(infer_response=resp)
            except _StreamAbort as e:
                yield pb.ModelStreamInferResponse(error_message=str(e))


class _StreamAbort(Exception):
    pass


class _StreamCtx:
    """Per-request errors on a stream become error_message responses."""

    def __init__(self, ctx):
        self._ctx = ctx

    def abort(self, code, details):
        raise _StreamAbort(details)


def _handlers(servicer: GRPCInferenceServicer, raw_infer: bool = True):
    from ..proto import SERVICE_METHODS
    h = {}
    for rpc, req, resp, cs, ss in SERVICE_METHODS:
        if rpc == "ModelInfer" and raw_infer:  # bytes in, bytes out through the C++ codec
            h[rpc] = grpc.unary_unary_rpc_method_handler(servicer.ModelInferBytes, request_deserializer=None,
                                                         response_serializer=None)
            continue
        fn = getattr(servicer, rpc)
        de = getattr(pb, req).FromString
        ser = getattr(pb, resp).SerializeToString
        if cs and ss:
            h[rpc] = grpc.stream_stream_rpc_method_handler(fn, request_deserializer=de, response_serializer=ser)
        else:
            h[rpc] = grpc.unary_unary_rpc_method_handler(fn, request_deserializer=de, response_serializer=ser)
    return grpc.method_handlers_generic_handler(SERVICE, h)


class KServeServer:
    def __init__(self, repo: ModelRepository, address: str = "127.0.0.1:8001", max_workers: int = 8,
                 max_message_bytes: int = 512 << 20, fault: Optional[FaultInjector] = None,
                 metrics_port: Optional[int] = None, raw_infer: bool = True, switch_interval_s: Optional[float] = None):
        """raw_infer: serve ModelInfer through the C++ codec on the wire bytes
        (False: the protobuf runtime, as a Triton-like reference path)."""
        self.repo = repo
        self.address = address
        if switch_interval_s is None:
            switch_interval_s = 2e-4  # GIL hand-off between the gRPC threads and the batchers
        self.switch_interval_s = switch_interval_s
        metrics = None
        if metrics_port is not None:
            from ..utils.metrics import ServerMetrics
            metrics = ServerMetrics(port=metrics_port)
        self.servicer = GRPCInferenceServicer(repo, fault, metrics)
        opts = [("grpc.max_send_message_length", max_message_bytes),
                ("grpc.max_receive_message_length", max_message_bytes),
                ("grpc.so_reuseport", 1)]  # `python -m triton_client_amd.server --procs N` shares the port
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=opts)
        self.server.add_generic_rpc_handlers((_handlers(self.servicer, raw_infer),))
        self.port = self.server.add_insecure_port(address)
        if self.port == 0:
            raise RuntimeError(f"could not bind {address}")

    @property
    def target(self) -> str:
        host = self.address.rsplit(":", 1)[0]
        return f"{host}:{self.port}"

    def start(self) -> "KServeServer":
        # GIL hand-off: a batcher thread returning from a device wait (or a request thread
        # from a socket read) otherwise waits up to the 5 ms default switch interval for a
        # thread running Python to yield — several times per batch (measured on the served
        # bench: ~6 ms of every 15 ms PointPillars execution, TCA_SERVER_PROFILE)
        import sys
        if sys.getswitchinterval() > self.switch_interval_s:
            sys.setswitchinterval(self.switch_interval_s)
        self.server.start()
        return self

    def stop(self, grace: float = 0.5) -> None:
        self.server.stop(grace)

    def wait(self) -> None:
        self.server.wait_for_termination()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
