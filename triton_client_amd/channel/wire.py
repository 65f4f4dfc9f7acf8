"""Zero-copy KServe-v2 request/response (de)serialisation through the C++
wire codec (``csrc/runtime/kserve_wire.cpp``).

* :func:`encode_request` — one pass, one copy of each tensor: writes a
  serialized ``ModelInferRequest`` whose ``raw_input_contents`` come straight
  from the given arrays (e.g. pinned staging written by the GPU).
* :func:`parse_response` — returns ``{name: np.ndarray}`` views into the
  response bytes (``np.frombuffer``, no copy), replacing the reference's
  per-element ``struct.unpack`` decoders
  (``clients/postprocess/base_postprocess.py:15-37``).

Both fall back to the protobuf runtime when the native library is absent
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


def encode_request(model_name: str, inputs: Sequence[Tuple[str, np.ndarray]], outputs: Sequence[str] = (),
                   model_version: str = "", request_id: str = "", datatypes: Optional[Sequence[str]] = None) -> bytes:
    arrs = [np.ascontiguousarray(a) for _, a in inputs]
    dts = list(datatypes) if datatypes else [kserve_dtype(a) for a in arrs]
    rt = _rt()
    if rt is None:
        req = service_pb2.ModelInferRequest(model_name=model_name, model_version=model_version, id=request_id)
        for (name, _), a, dt in zip(inputs, arrs, dts):
            t = req.inputs.add(name=name, datatype=dt)
            t.shape.extend(a.shape)
            req.raw_input_contents.append(a.tobytes())
        for o in outputs:
            req.outputs.add(name=o)
        return req.SerializeToString()
    n_in, n_out = len(arrs), len(outputs)
    names = (ctypes.c_char_p * n_in)(*[n.encode() for n, _ in inputs])
    dtypes = (ctypes.c_char_p * n_in)(*[d.encode() for d in dts])
    shapes = np.asarray([d for a in arrs for d in a.shape], np.int64)
    ndims = np.asarray([a.ndim for a in arrs], np.int32)
    ptrs = (ctypes.c_void_p * n_in)(*[a.ctypes.data for a in arrs])
    nbytes = np.asarray([a.nbytes for a in arrs], np.int64)
    onames = (ctypes.c_char_p * max(n_out, 1))(*[o.encode() for o in outputs])
    mn, mv, rid = model_name.encode(), model_version.encode(), request_id.encode()
    size = rt.tca_kserve_request_size(mn, mv, rid, n_in, names, dtypes, shapes.ctypes.data, ndims.ctypes.data,
                                      nbytes.ctypes.data, n_out, onames)
    buf = bytearray(size)
    cbuf = (ctypes.c_char * size).from_buffer(buf)
    n = rt.tca_kserve_encode_request(mn, mv, rid, n_in, names, dtypes, shapes.ctypes.data, ndims.ctypes.data, ptrs,
                                     nbytes.ctypes.data, n_out, onames, ctypes.addressof(cbuf), size)
    del cbuf
    if n != size:
        raise RuntimeError(f"kserve encode failed ({n} != {size})")
    return bytes(buf)


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
