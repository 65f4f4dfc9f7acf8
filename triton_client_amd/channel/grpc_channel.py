"""KServe-v2 gRPC channel (reference ``communicator/channel/grpc_channel.py:8-78``).

API parity with the reference ``GRPCChannel``: construction opens the
channel, fetches ``ModelMetadata`` + ``ModelConfig`` and pre-builds a
reusable ``ModelInferRequest`` (``.request``, ``.input``, ``.output``,
``.response`` are public and mutated by the inference drivers exactly like
the reference's); ``do_inference()`` is a unary ``ModelInfer``.

Additions: server liveness / model readiness probes at start,
an optional per-RPC deadline with bounded exponential-backoff retries,
``do_inference_async()`` (the legacy ``.future`` path, ``evaluate.py:166``),
``stream_inference()`` (``ModelStreamInfer``, ``evaluate.py:143``), and
``infer_raw()`` — the zero-copy fast path through the C++ wire codec.
Message-size limits are derived from the model's tensor sizes instead of the
reference's fixed ``batch_size * 8568044`` (README TODO at ``README.md:118``:
a 1333x800 fp32 input is 12.8 MB).
"""
from __future__ import annotations

import time
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import grpc
import numpy as np

from ..proto import SERVICE, SERVICE_METHODS, model_config_pb2 as mc, service_pb2 as pb
from .base import BaseChannel
from .wire import ParsedResponse, encode_request, parse_response

REFERENCE_MAX_MSG = 8568044  # one YOLOv5-COCO-640 fp32 output + protobuf overhead
RETRYABLE = {grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED, grpc.StatusCode.RESOURCE_EXHAUSTED}


class GRPCInferenceServiceStub:
    """Client stub for ``inference.GRPCInferenceService`` (generated-stub
    equivalent) plus ``ModelInferRaw`` taking/returning serialized bytes."""

    def __init__(self, channel: grpc.Channel):
        for rpc, req, resp, cs, ss in SERVICE_METHODS:
            path = f"/{SERVICE}/{rpc}"
            ser = getattr(pb, req).SerializeToString
            de = getattr(pb, resp).FromString
            if cs and ss:
                fn = channel.stream_stream(path, request_serializer=ser, response_deserializer=de)
            else:
                fn = channel.unary_unary(path, request_serializer=ser, response_deserializer=de)
            setattr(self, rpc, fn)
        self.ModelInferRaw = channel.unary_unary(f"/{SERVICE}/ModelInfer", request_serializer=None,
                                                 response_deserializer=None)


def _flag(FLAGS, name, default):
    v = getattr(FLAGS, name, default) if FLAGS is not None else default
    return default if v is None else v


class GRPCChannel(BaseChannel):
    def __init__(self, params: dict, FLAGS, timeout_s: Optional[float] = None, retries: int = 2,
                 wait_ready_s: float = 10.0, connect: bool = True):
        super().__init__(params, FLAGS)
        self._meta_data = {}
        self._grpc_stub = None
        self._channel = None
        self.timeout_s = timeout_s
        self.retries = retries
        self.wait_ready_s = wait_ready_s
        self.model_name = str(_flag(FLAGS, "model_name", ""))
        self.model_version = str(_flag(FLAGS, "model_version", ""))
        self.batch_size = int(_flag(FLAGS, "batch_size", 1))
        self.request = self.input = self.output = self.response = None
        if connect:
            self.register_channel()
            self.wait_for_server(self.wait_ready_s)
            self._grpc_metadata()

    # ------------------------------------------------------------ reference API
    def register_channel(self, max_message_bytes: Optional[int] = None):
        limit = max_message_bytes or max(REFERENCE_MAX_MSG * self.batch_size, 64 << 20)
        opts = [("grpc.max_send_message_length", limit), ("grpc.max_receive_message_length", limit)]
        self._channel = grpc.insecure_channel(self.params["grpc_channel"], options=opts)
        self._grpc_stub = GRPCInferenceServiceStub(self._channel)
        return self._grpc_stub

    def fetch_channel(self):
        return self._grpc_stub

    def get_metadata(self) -> dict:
        return self._meta_data

    def do_inference(self):
        return self._call(self._grpc_stub.ModelInfer, self.request)

    # ------------------------------------------------------------ additions
    def _call(self, fn, req, **kw):
        delay = 0.05
        for attempt in range(self.retries + 1):
            try:
                return fn(req, timeout=self.timeout_s, **kw)
            except grpc.RpcError as e:
                if e.code() not in RETRYABLE or attempt == self.retries:
                    raise
                time.sleep(delay)
                delay *= 2

    def wait_for_server(self, timeout_s: float = 10.0) -> bool:
        """Poll ServerLive (and ModelReady when a model is named) until ready."""
        deadline = time.monotonic() + timeout_s
        last = None
        while True:
            try:
                live = self._grpc_stub.ServerLive(pb.ServerLiveRequest(), timeout=1.0).live
                ready = True
                if self.model_name:
                    ready = self._grpc_stub.ModelReady(
                        pb.ModelReadyRequest(name=self.model_name, version=self.model_version), timeout=1.0).ready
                if live and ready:
                    return True
            except grpc.RpcError as e:
                last = e
            if time.monotonic() > deadline:
                raise ConnectionError(f"KServe server at {self.params['grpc_channel']} not ready"
                                      f" (model {self.model_name!r}): {last}")
            time.sleep(0.1)

    def _grpc_metadata(self):
        self._meta_data["metadata_request"] = pb.ModelMetadataRequest(name=self.model_name,
                                                                      version=self.model_version)
        self._meta_data["metadata_response"] = self._call(self._grpc_stub.ModelMetadata,
                                                          self._meta_data["metadata_request"])
        self._meta_data["config_request"] = pb.ModelConfigRequest(name=self.model_name, version=self.model_version)
        self._meta_data["config_response"] = self._call(self._grpc_stub.ModelConfig,
                                                        self._meta_data["config_request"])
        self._set_grpc_members()

    def _set_grpc_members(self):
        self.input = pb.ModelInferRequest.InferInputTensor()
        self.request = pb.ModelInferRequest(model_name=self.model_name, model_version=self.model_version)
        self.output = pb.ModelInferRequest.InferRequestedOutputTensor()

    def do_inference_async(self):
        """grpc future for the current request (legacy ``ModelInfer.future``)."""
        return self._grpc_stub.ModelInfer.future(self.request, timeout=self.timeout_s)

    def stream_inference(self, requests: Iterable) -> Iterator:
        """Bidirectional ``ModelStreamInfer``: yields ModelStreamInferResponse."""
        return self._grpc_stub.ModelStreamInfer(iter(requests), timeout=self.timeout_s)

    def infer_raw(self, inputs: Sequence[Tuple[str, np.ndarray]], outputs: Sequence[str] = (),
                  datatypes: Optional[Sequence[str]] = None, request_id: str = "") -> ParsedResponse:
        """Fast path: serialize with the C++ codec, parse the response into
        zero-copy ndarray views."""
        raw = encode_request(self.model_name, inputs, outputs, self.model_version, request_id, datatypes)
        data = self._call(self._grpc_stub.ModelInferRaw, raw)
        return parse_response(data)

    def send_raw(self, raw: bytes) -> ParsedResponse:
        """One pre-encoded request (see channel.wire.encode_request) → parsed response."""
        return parse_response(self._call(self._grpc_stub.ModelInferRaw, raw))

    def send_raw_async(self, raw: bytes):
        """grpc future of a pre-encoded request (``.result()`` → response bytes)."""
        return self._grpc_stub.ModelInferRaw.future(raw, timeout=self.timeout_s)

    def server_metadata(self):
        return self._grpc_stub.ServerMetadata(pb.ServerMetadataRequest(), timeout=self.timeout_s)

    # ------------------------------------------------- system shared memory
    def register_system_shared_memory(self, name: str, key: str, byte_size: int, offset: int = 0):
        return self._call(self._grpc_stub.SystemSharedMemoryRegister,
                          pb.SystemSharedMemoryRegisterRequest(name=name, key=key, offset=offset, byte_size=byte_size))

    def unregister_system_shared_memory(self, name: str = ""):
        return self._call(self._grpc_stub.SystemSharedMemoryUnregister,
                          pb.SystemSharedMemoryUnregisterRequest(name=name))

    def system_shared_memory_status(self, name: str = ""):
        return self._call(self._grpc_stub.SystemSharedMemoryStatus, pb.SystemSharedMemoryStatusRequest(name=name))

    def register_cuda_shared_memory(self, name: str, raw_handle: bytes, device_id: int, byte_size: int):
        """Device shared memory (Triton's CudaSharedMemoryRegister; here a HIP IPC handle,
        ``utils.hip_ipc.DeviceAllocation``)."""
        return self._call(self._grpc_stub.CudaSharedMemoryRegister,
                          pb.CudaSharedMemoryRegisterRequest(name=name, raw_handle=raw_handle, device_id=device_id,
                                                             byte_size=byte_size))

    def unregister_cuda_shared_memory(self, name: str = ""):
        return self._call(self._grpc_stub.CudaSharedMemoryUnregister, pb.CudaSharedMemoryUnregisterRequest(name=name))

    def cuda_shared_memory_status(self, name: str = ""):
        return self._call(self._grpc_stub.CudaSharedMemoryStatus, pb.CudaSharedMemoryStatusRequest(name=name))

    def model_statistics(self, name: str = ""):
        return self._grpc_stub.ModelStatistics(pb.ModelStatisticsRequest(name=name), timeout=self.timeout_s)

    def close(self):
        if self._channel is not None:
            self._channel.close()
            self._channel = None


def input_geometry(model_metadata, model_config) -> Tuple[int, int, int, int, str]:
    """(c, h, w, format, datatype) of a single image input (for stats/tests)."""
    inp = model_metadata.inputs[0]
    fmt = model_config.input[0].format
    s = list(inp.shape)
    if len(s) == 4:
        s = s[1:]
    if fmt == mc.ModelInput.FORMAT_NHWC:
        h, w, c = s
    else:
        c, h, w = s
    return c, h, w, fmt, inp.datatype
