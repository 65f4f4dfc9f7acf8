"""Zero-copy KServe-v2 request/response (de)serialisation through the C++
wire codec (``csrc/runtime/kserve_wire.cpp``).

Client:

* :func:`encode_request` — one pass, ONE copy of each tensor: the C++
  encoder writes a serialized ``ModelInferRequest`` whose
  ``raw_input_contents`` come straight from the given memory (numpy arrays or
  CPU torch tensors — typically the pinned ``hipHostMalloc`` staging the GPU
  preprocess landed in) directly into the ``bytes`` object handed to gRPC
  (allocated uninitialised through the CPython API, so there is no
  ``bytearray`` → ``bytes`` second copy).
* :func:`parse_response` — ``{name: np.ndarray}`` views into the response
  bytes (``np.frombuffer``, no copy), replacing the reference's per-element
  ``struct.unpack`` decoders (``clients/postprocess/base_postprocess.py:15-37``).

Server (the same codec, mirrored): :func:`parse_request` gives views of every
``raw_input_contents`` inside the request bytes; :func:`encode_response`
writes the response straight from the output tensors' memory.

All fall back to the protobuf runtime when the native library is absent
(CPU-only hosts without hipcc); results are identical bytes.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native
from ..proto import KSERVE_TO_NP, NP_TO_KSERVE, service_pb2

_BF16 = "BF16"


def _np_dtype(kserve: str):
    if kserve == _BF16:
        return np.dtype(np.uint16)
    return np.dtype(KSERVE_TO_NP[kserve])


def kserve_dtype(arr: np.ndarray) -> str:
    return NP_TO_KSERVE[str(arr.dtype)]


def _rt():
    try:
        return _native.runtime()
    except Exception:
        return None


_TORCH_KSERVE = {"torch.float32": "FP32", "torch.float16": "FP16", "torch.float64": "FP64", "torch.int32": "INT32",
                 "torch.int64": "INT64", "torch.uint8": "UINT8", "torch.int8": "INT8", "torch.int16": "INT16",
                 "torch.bool": "BOOL", "torch.bfloat16": _BF16}

_PyBytes_FromStringAndSize = ctypes.pythonapi.PyBytes_FromStringAndSize
_PyBytes_FromStringAndSize.restype = ctypes.py_object
_PyBytes_FromStringAndSize.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_PyBytes_AsString = ctypes.pythonapi.PyBytes_AsString
_PyBytes_AsString.restype = ctypes.c_void_p
_PyBytes_AsString.argtypes = [ctypes.py_object]


def _new_bytes(size: int):
    """An uninitialised, not-yet-shared ``bytes`` of ``size`` and its buffer
    address (CPython's own pattern for filling a bytes object in place)."""
    b = _PyBytes_FromStringAndSize(None, size)
    return b, _PyBytes_AsString(b)


class _Mem:
    """Pointer / shape / byte size / KServe dtype of a host tensor, without copying it."""
    __slots__ = ("ptr", "shape", "nbytes", "dtype", "keep")

    def __init__(self, a, dtype: Optional[str] = None):
        if type(a).__module__.startswith("torch"):
            if a.device.type != "cpu":
                raise ValueError("wire tensors must be host memory (copy device results into pinned staging first)")
            if not a.is_contiguous():
                a = a.contiguous()
            self.ptr, self.shape = a.data_ptr(), tuple(a.shape)
            self.nbytes = a.numel() * a.element_size()
            self.dtype = dtype or _TORCH_KSERVE[str(a.dtype)]
        else:
            a = np.ascontiguousarray(a)
            self.ptr, self.shape, self.nbytes = a.ctypes.data, a.shape, a.nbytes
            self.dtype = dtype or kserve_dtype(a)
        self.keep = a

    def view(self) -> bytes:
        return ctypes.string_at(self.ptr, self.nbytes)


def _c_tables(items: Sequence[Tuple[str, "_Mem"]]):
    n = len(items)
    names = (ctypes.c_char_p * max(n, 1))(*[nm.encode() for nm, _ in items])
    dtypes = (ctypes.c_char_p * max(n, 1))(*[m.dtype.encode() for _, m in items])
    shapes = np.asarray([d for _, m in items for d in m.shape] or [0], np.int64)
    ndims = np.asarray([len(m.shape) for _, m in items] or [0], np.int32)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[m.ptr for _, m in items])
    nbytes = np.asarray([m.nbytes for _, m in items] or [0], np.int64)
    return names, dtypes, shapes, ndims, ptrs, nbytes


def encode_request(model_name: str, inputs: Sequence[Tuple[str, object]], outputs: Sequence[str] = (),
                   model_version: str = "", request_id: str = "", datatypes: Optional[Sequence[str]] = None) -> bytes:
    """inputs: (name, numpy array or CPU torch tensor); each tensor's bytes are
    copied exactly once, into the returned request."""
    dts = list(datatypes) if datatypes else [None] * len(inputs)
    items = [(n, _Mem(a, dt)) for (n, a), dt in zip(inputs, dts)]
    rt = _rt()
    if rt is None:
        req = service_pb2.ModelInferRequest(model_name=model_name, model_version=model_version, id=request_id)
        for name, m in items:
            t = req.inputs.add(name=name, datatype=m.dtype)
            t.shape.extend(m.shape)
            req.raw_input_contents.append(m.view())
        for o in outputs:
            req.outputs.add(name=o)
        return req.SerializeToString()
    n_in, n_out = len(items), len(outputs)
    names, dtypes, shapes, ndims, ptrs, nbytes = _c_tables(items)
    onames = (ctypes.c_char_p * max(n_out, 1))(*[o.encode() for o in outputs])
    mn, mv, rid = model_name.encode(), model_version.encode(), request_id.encode()
    size = rt.tca_kserve_request_size(mn, mv, rid, n_in, names, dtypes, shapes.ctypes.data, ndims.ctypes.data,
                                      nbytes.ctypes.data, n_out, onames)
    out, addr = _new_bytes(size)
    n = rt.tca_kserve_encode_request(mn, mv, rid, n_in, names, dtypes, shapes.ctypes.data, ndims.ctypes.data, ptrs,
                                     nbytes.ctypes.data, n_out, onames, addr, size)
    if n != size:
        raise RuntimeError(f"kserve encode failed ({n} != {size})")
    return out


def encode_response(model_name: str, outputs: Sequence[Tuple[str, object]], model_version: str = "",
                    request_id: str = "") -> bytes:
    """Serialized ModelInferResponse written straight from the output tensors'
    memory (one copy of each)."""
    items = [(n, _Mem(a)) for n, a in outputs]
    rt = _rt()
    if rt is None:
        resp = service_pb2.ModelInferResponse(model_name=model_name, model_version=model_version, id=request_id)
        for name, m in items:
            t = resp.outputs.add(name=name, datatype=m.dtype)
            t.shape.extend(m.shape)
            resp.raw_output_contents.append(m.view())
        return resp.SerializeToString()
    names, dtypes, shapes, ndims, ptrs, nbytes = _c_tables(items)
    mn, mv, rid = model_name.encode(), model_version.encode(), request_id.encode()
    size = rt.tca_kserve_response_size(mn, mv, rid, len(items), names, dtypes, shapes.ctypes.data, ndims.ctypes.data,
                                       nbytes.ctypes.data)
    out, addr = _new_bytes(size)
    n = rt.tca_kserve_encode_response(mn, mv, rid, len(items), names, dtypes, shapes.ctypes.data, ndims.ctypes.data,
                                      ptrs, nbytes.ctypes.data, addr, size)
    if n != size:
        raise RuntimeError(f"kserve response encode failed ({n} != {size})")
    return out


class ParsedRequest:
    """Server view of a ModelInferRequest: ``inputs`` are ndarray views into the request bytes."""

    def __init__(self):
        self.model_name = ""
        self.model_version = ""
        self.id = ""
        self.inputs: Dict[str, np.ndarray] = {}
        self.datatypes: Dict[str, str] = {}
        self.order: List[str] = []
        self.outputs: List[str] = []
        self.has_params = False  # a tensor carries parameters (shared-memory references): protobuf path


def parse_request(data: bytes, max_tensors: int = 64) -> ParsedRequest:
    out = ParsedRequest()
    rt = _rt()
    if rt is None:
        req = service_pb2.ModelInferRequest()
        req.ParseFromString(data)
        out.model_name, out.model_version, out.id = req.model_name, req.model_version, req.id
        for t, raw in zip(req.inputs, req.raw_input_contents):
            out.inputs[t.name] = np.frombuffer(raw, dtype=_np_dtype(t.datatype)).reshape(tuple(t.shape))
            out.datatypes[t.name] = t.datatype
            out.order.append(t.name)
        out.outputs = [o.name for o in req.outputs]
        out.has_params = (any(len(t.parameters) for t in req.inputs) or any(len(o.parameters) for o in req.outputs)
                          or len(req.raw_input_contents) < len(req.inputs))  # typed contents: protobuf path
        return out
    mv = memoryview(data)
    meta = np.zeros((max_tensors, 8), np.int64)
    shapes = np.zeros((max_tensors * 8,), np.int64)
    raw = np.zeros((max_tensors, 2), np.int64)
    req = np.zeros((max_tensors, 2), np.int64)
    counts = np.zeros((10,), np.int64)
    src = ctypes.c_char_p(data)
    rc = rt.tca_kserve_parse_request(ctypes.cast(src, ctypes.c_void_p), len(data), max_tensors, meta.ctypes.data,
                                     shapes.ctypes.data, shapes.size, raw.ctypes.data, req.ctypes.data,
                                     counts.ctypes.data)
    if rc != 0:
        raise ValueError(f"malformed ModelInferRequest ({rc})")
    n_in, n_raw, n_req = (int(v) for v in counts[:3])
    out.has_params = bool(counts[9])
    txt = lambda o, ln: bytes(mv[o:o + ln]).decode()  # noqa: E731
    out.model_name, out.model_version, out.id = (txt(int(counts[3 + 2 * k]), int(counts[4 + 2 * k])) for k in range(3))
    for k in range(n_in):
        no, nl, do, dl, nd, si = (int(v) for v in meta[k, :6])
        name, dt = txt(no, nl), txt(do, dl)
        shape = tuple(int(v) for v in shapes[si:si + nd])
        out.datatypes[name] = dt
        out.order.append(name)
        if k < n_raw:
            off, ln = int(raw[k, 0]), int(raw[k, 1])
            it = _np_dtype(dt).itemsize
            out.inputs[name] = np.frombuffer(data, dtype=_np_dtype(dt), count=ln // it, offset=off).reshape(shape)
    out.outputs = [txt(int(req[k, 0]), int(req[k, 1])) for k in range(n_req)]
    return out


class ParsedResponse:
    """name → ndarray view (plus .shapes/.datatypes/.model_name)."""

    def __init__(self):
        self.model_name = ""
        self.outputs: Dict[str, np.ndarray] = {}
        self.datatypes: Dict[str, str] = {}
        self.order: List[str] = []

    def __getitem__(self, k):
        return self.outputs[k] if isinstance(k, str) else self.outputs[self.order[k]]

    def __len__(self):
        return len(self.order)


def parse_response(data: bytes, max_outputs: int = 64) -> ParsedResponse:
    out = ParsedResponse()
    rt = _rt()
    if rt is None:
        resp = service_pb2.ModelInferResponse()
        resp.ParseFromString(data)
        out.model_name = resp.model_name
        for t, raw in zip(resp.outputs, resp.raw_output_contents):
            a = np.frombuffer(raw, dtype=_np_dtype(t.datatype)).reshape(tuple(t.shape))
            out.outputs[t.name] = a
            out.datatypes[t.name] = t.datatype
            out.order.append(t.name)
        return out
    mv = memoryview(data)
    meta = np.zeros((max_outputs, 8), np.int64)
    shapes = np.zeros((max_outputs * 8,), np.int64)
    raw = np.zeros((max_outputs, 2), np.int64)
    counts = np.zeros((4,), np.int64)
    src = ctypes.c_char_p(data)  # points at the bytes object's buffer (no copy)
    rc = rt.tca_kserve_parse_response(ctypes.cast(src, ctypes.c_void_p), len(data), max_outputs, meta.ctypes.data,
                                      shapes.ctypes.data, shapes.size, raw.ctypes.data, counts.ctypes.data)
    if rc != 0:
        raise ValueError(f"malformed ModelInferResponse ({rc})")
    n_out, n_raw = int(counts[0]), int(counts[1])
    out.model_name = bytes(mv[counts[2]:counts[2] + counts[3]]).decode()
    for k in range(n_out):
        no, nl, do, dl, nd, si = (int(v) for v in meta[k, :6])
        name = bytes(mv[no:no + nl]).decode()
        dt = bytes(mv[do:do + dl]).decode()
        shape = tuple(int(v) for v in shapes[si:si + nd])
        out.datatypes[name] = dt
        out.order.append(name)
        if k < n_raw:
            off, ln = int(raw[k, 0]), int(raw[k, 1])
            out.outputs[name] = np.frombuffer(data, dtype=_np_dtype(dt), count=ln // _np_dtype(dt).itemsize,
                                              offset=off).reshape(shape)
    return out
