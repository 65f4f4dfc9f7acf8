"""ROS1 message wire format (genpy serialisation) for the message types the
reference reads and writes in its bags (``communicator/bag_inference2d.py:34-35``,
``communicator/bag_inference3d.py:62-63,182-183``): sensor_msgs Image /
CompressedImage / PointCloud2, jsk_recognition_msgs BoundingBoxArray and
vision_msgs Detection2DArray / Detection3DArray (+ their dependencies).

* Schemas are the ``.msg`` definitions (comments stripped); :func:`md5sum`
  implements genmsg's MD5 rule (constants first, nested types replaced by
  their own MD5) — checked against the well-known sums of std_msgs/Header,
  sensor_msgs/Image, sensor_msgs/PointCloud2, ... in the tests.
* :func:`serialize` / :func:`deserialize` work on the dataclasses of
  :mod:`.msgs` (little-endian, ``uint32`` length prefixes for strings and
  variable arrays, ``uint8[]`` as raw bytes).  Where a ROS type carries fields
  the dataclasses do not model (``PoseWithCovariance.covariance``,
  ``Detection3D.source_cloud``) they are written as zeros / empty and
  dropped on read.
"""
from __future__ import annotations

import hashlib
import struct
import threading
from dataclasses import is_dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

from . import msgs

BUILTIN = {
    "bool": "?", "int8": "b", "uint8": "B", "byte": "b", "char": "B", "int16": "h", "uint16": "H",
    "int32": "i", "uint32": "I", "int64": "q", "uint64": "Q", "float32": "f", "float64": "d",
}
SPECIAL = ("string", "time", "duration")

DEFS: Dict[str, str] = {
    "std_msgs/Header": "uint32 seq\ntime stamp\nstring frame_id",
    "geometry_msgs/Point": "float64 x\nfloat64 y\nfloat64 z",
    "geometry_msgs/Vector3": "float64 x\nfloat64 y\nfloat64 z",
    "geometry_msgs/Quaternion": "float64 x\nfloat64 y\nfloat64 z\nfloat64 w",
    "geometry_msgs/Pose": "Point position\nQuaternion orientation",
    "geometry_msgs/Pose2D": "float64 x\nfloat64 y\nfloat64 theta",
    "geometry_msgs/PoseWithCovariance": "Pose pose\nfloat64[36] covariance",
    "sensor_msgs/Image": ("Header header\nuint32 height\nuint32 width\nstring encoding\nuint8 is_bigendian\n"
                          "uint32 step\nuint8[] data"),
    "sensor_msgs/CompressedImage": "Header header\nstring format\nuint8[] data",
    "sensor_msgs/PointField": ("uint8 INT8=1\nuint8 UINT8=2\nuint8 INT16=3\nuint8 UINT16=4\nuint8 INT32=5\n"
                               "uint8 UINT32=6\nuint8 FLOAT32=7\nuint8 FLOAT64=8\n"
                               "string name\nuint32 offset\nuint8 datatype\nuint32 count"),
    "sensor_msgs/PointCloud2": ("Header header\nuint32 height\nuint32 width\nPointField[] fields\nbool is_bigendian\n"
                                "uint32 point_step\nuint32 row_step\nuint8[] data\nbool is_dense"),
    "jsk_recognition_msgs/BoundingBox": ("Header header\ngeometry_msgs/Pose pose\ngeometry_msgs/Vector3 dimensions\n"
                                         "float32 value\nuint32 label"),
    "jsk_recognition_msgs/BoundingBoxArray": "Header header\nBoundingBox[] boxes",
    "vision_msgs/ObjectHypothesisWithPose": "int64 id\nfloat64 score\ngeometry_msgs/PoseWithCovariance pose",
    "vision_msgs/BoundingBox2D": "geometry_msgs/Pose2D center\nfloat64 size_x\nfloat64 size_y",
    "vision_msgs/Detection2D": ("Header header\nObjectHypothesisWithPose[] results\nBoundingBox2D bbox\n"
                                "sensor_msgs/Image source_img"),
    "vision_msgs/Detection2DArray": "Header header\nDetection2D[] detections",
    "vision_msgs/BoundingBox3D": "geometry_msgs/Pose center\ngeometry_msgs/Vector3 size",
    "vision_msgs/Detection3D": ("Header header\nObjectHypothesisWithPose[] results\nBoundingBox3D bbox\n"
                                "sensor_msgs/PointCloud2 source_cloud"),
    "vision_msgs/Detection3DArray": "Header header\nDetection3D[] detections",
}

# ROS type -> the msgs dataclass holding it (types without one decode to dicts)
DATACLASS = {
    "std_msgs/Header": msgs.Header, "geometry_msgs/Point": msgs.Point, "geometry_msgs/Vector3": msgs.Vector3,
    "geometry_msgs/Quaternion": msgs.Quaternion, "geometry_msgs/Pose": msgs.Pose, "geometry_msgs/Pose2D": msgs.Pose2D,
    "sensor_msgs/Image": msgs.Image, "sensor_msgs/CompressedImage": msgs.CompressedImage,
    "sensor_msgs/PointField": msgs.PointField, "sensor_msgs/PointCloud2": msgs.PointCloud2,
    "jsk_recognition_msgs/BoundingBox": msgs.BoundingBox, "jsk_recognition_msgs/BoundingBoxArray": msgs.BoundingBoxArray,
    "vision_msgs/ObjectHypothesisWithPose": msgs.ObjectHypothesisWithPose,
    "vision_msgs/BoundingBox2D": msgs.BoundingBox2D, "vision_msgs/Detection2D": msgs.Detection2D,
    "vision_msgs/Detection2DArray": msgs.Detection2DArray, "vision_msgs/BoundingBox3D": msgs.BoundingBox3D,
    "vision_msgs/Detection3D": msgs.Detection3D, "vision_msgs/Detection3DArray": msgs.Detection3DArray,
}
TYPE_OF = {v: k for k, v in DATACLASS.items()}


class Field:
    __slots__ = ("type", "name", "base", "array", "size")

    def __init__(self, type_: str, name: str, pkg: str):
        self.type, self.name = type_, name
        base, self.array, self.size = type_, False, None
        if type_.endswith("]"):
            base, dim = type_[:-1].split("[")
            self.array, self.size = True, (int(dim) if dim else None)
        self.base = resolve(base, pkg)


def resolve(base: str, pkg: str) -> str:
    if base in BUILTIN or base in SPECIAL:
        return base
    if base == "Header":
        return "std_msgs/Header"
    return base if "/" in base else f"{pkg}/{base}"


_SPECS: Dict[str, Tuple[List[Tuple[str, str, str]], List[Field]]] = {}


def spec(msg_type: str):
    """(constants [(type, name, value)], fields) of a registered type."""
    if msg_type not in _SPECS:
        if msg_type not in DEFS:
            raise KeyError(f"no schema for {msg_type}")
        pkg = msg_type.split("/")[0]
        consts, flds = [], []
        for line in DEFS[msg_type].splitlines():
            line = line.split("#")[0].strip()
            if not line:
                continue
            t, rest = line.split(None, 1)
            if "=" in rest:
                n, v = rest.split("=", 1)
                consts.append((t, n.strip(), v.strip()))
            else:
                flds.append(Field(t, rest.strip(), pkg))
        _SPECS[msg_type] = (consts, flds)
    return _SPECS[msg_type]


def md5_text(msg_type: str) -> str:
    consts, flds = spec(msg_type)
    lines = [f"{t} {n}={v}" for t, n, v in consts]
    for f in flds:
        if f.base in BUILTIN or f.base in SPECIAL:
            lines.append(f"{f.type} {f.name}")
        else:
            lines.append(f"{md5sum(f.base)} {f.name}")
    return "\n".join(lines)


def md5sum(msg_type: str) -> str:
    return hashlib.md5(md5_text(msg_type).encode()).hexdigest()


def full_definition(msg_type: str) -> str:
    """The message_definition text rosbag stores in a connection record:
    the type's own definition, then every dependency once."""
    out, seen, order = [DEFS[msg_type]], {msg_type}, []

    def walk(t):
        for f in spec(t)[1]:
            if f.base not in BUILTIN and f.base not in SPECIAL and f.base not in seen:
                seen.add(f.base)
                order.append(f.base)
                walk(f.base)
    walk(msg_type)
    for d in order:
        out.append("=" * 80 + f"\nMSG: {d}\n" + DEFS[d])
    return "\n".join(out) + "\n"


# ------------------------------------------------------------------ adapters between dataclasses and ROS fields
def _get(msg: Any, name: str, ros_type: str, field: Field):
    if isinstance(msg, dict):
        return msg.get(name)
    if ros_type == "vision_msgs/ObjectHypothesisWithPose" and name == "pose":
        return {"pose": getattr(msg, "pose", None), "covariance": [0.0] * 36}
    return getattr(msg, name, None)


def _write(buf: bytearray, value: Any, f: Field, parent: str) -> None:
    if f.array:
        if f.base in ("uint8", "char") and f.size is None:
            b = bytes(value or b"")
            buf += struct.pack("<I", len(b))
            buf += b
            return
        items = list(value or [])
        if f.size is None:
            buf += struct.pack("<I", len(items))
        elif len(items) != f.size:
            items = (items + [0] * f.size)[: f.size]
        if f.base in BUILTIN:
            buf += struct.pack("<%d%s" % (len(items), BUILTIN[f.base]), *items)
        else:
            for it in items:
                _write_scalar(buf, it, f.base)
        return
    _write_scalar(buf, value, f.base)


def _write_scalar(buf: bytearray, value: Any, base: str) -> None:
    if base in BUILTIN:
        buf += struct.pack("<" + BUILTIN[base], value if value is not None else 0)
    elif base == "string":
        b = (value or "").encode() if isinstance(value, str) else bytes(value or b"")
        buf += struct.pack("<I", len(b))
        buf += b
    elif base in ("time", "duration"):
        secs = getattr(value, "secs", 0) if value is not None else 0
        nsecs = getattr(value, "nsecs", 0) if value is not None else 0
        if isinstance(value, dict):
            secs, nsecs = value.get("secs", 0), value.get("nsecs", 0)
        buf += struct.pack("<Ii" if base == "duration" else "<II", secs, nsecs)
    else:
        _write_msg(buf, value, base)


def _write_jsk_columns(buf: bytearray, msg: Any) -> None:
    """BoundingBoxArray whose boxes are still columns (``msgs.ArrayList`` from the
    live driver): every box record is fixed-size (its header is the array's), so
    the whole array is one packed structured-array write."""
    import numpy as np

    cols = msg.boxes.columns
    hdr = bytearray()
    _write_msg(hdr, msg.header, "std_msgs/Header")
    n = len(cols["value"])
    rec = np.zeros(n, np.dtype([("h", f"V{len(hdr)}"), ("p", "<f8", 3), ("q", "<f8", 4), ("d", "<f8", 3),
                                ("v", "<f4"), ("l", "<u4")]))
    if n:
        rec["h"] = np.frombuffer(bytes(hdr), f"V{len(hdr)}")[0]
        rec["p"], rec["q"], rec["d"] = cols["position"], cols["orientation"], cols["dimensions"]
        rec["v"], rec["l"] = cols["value"], cols["label"]
    buf += hdr
    buf += struct.pack("<I", n)
    buf += rec.tobytes()


def _write_msg(buf: bytearray, msg: Any, msg_type: str) -> None:
    if (msg_type == "jsk_recognition_msgs/BoundingBoxArray" and isinstance(getattr(msg, "boxes", None), msgs.ArrayList)
            and not msg.boxes.built and msg.boxes.columns is not None and "position" in msg.boxes.columns):
        _write_jsk_columns(buf, msg)
        return
    for f in spec(msg_type)[1]:
        _write(buf, _get(msg, f.name, msg_type, f) if msg is not None else None, f, msg_type)


def serialize(msg: Any, msg_type: Optional[str] = None) -> bytes:
    msg_type = msg_type or TYPE_OF[type(msg)]
    buf = bytearray()
    _write_msg(buf, msg, msg_type)
    return bytes(buf)


# ------------------------------------------------------------------ read
def _read_msg(mv: memoryview, off: int, msg_type: str):
    d = {}
    for f in spec(msg_type)[1]:
        d[f.name], off = _read(mv, off, f)
    return _build(msg_type, d), off


def _read_scalar(mv: memoryview, off: int, base: str):
    if base in BUILTIN:
        fmt = "<" + BUILTIN[base]
        return struct.unpack_from(fmt, mv, off)[0], off + struct.calcsize(fmt)
    if base == "string":
        (n,) = struct.unpack_from("<I", mv, off)
        return bytes(mv[off + 4: off + 4 + n]).decode("utf-8", "replace"), off + 4 + n
    if base in ("time", "duration"):
        s, ns = struct.unpack_from("<Ii" if base == "duration" else "<II", mv, off)
        return msgs.Time(s, ns), off + 8
    return _read_msg(mv, off, base)


def _read(mv: memoryview, off: int, f: Field):
    if not f.array:
        return _read_scalar(mv, off, f.base)
    if f.size is None:
        (n,) = struct.unpack_from("<I", mv, off)
        off += 4
    else:
        n = f.size
    if f.base in ("uint8", "char"):
        alloc = getattr(_TLS, "alloc", None)
        if alloc is _ZERO_COPY and n >= ALLOC_MIN:
            return mv[off: off + n], off + n
        if alloc is not None and n >= ALLOC_MIN:
            buf = alloc(n)  # e.g. the DP host ring's ingest arena: the payload lands where every rank reads it
            if buf is not None:
                buf[:] = mv[off: off + n]
                return memoryview(buf), off + n
        return bytes(mv[off: off + n]), off + n
    if f.base in BUILTIN:
        fmt = "<%d%s" % (n, BUILTIN[f.base])
        return list(struct.unpack_from(fmt, mv, off)), off + struct.calcsize(fmt)
    out = []
    for _ in range(n):
        v, off = _read_scalar(mv, off, f.base)
        out.append(v)
    return out, off


def _build(msg_type: str, d: dict):
    if msg_type == "geometry_msgs/PoseWithCovariance":
        return d  # adapted by its parent
    if msg_type == "vision_msgs/ObjectHypothesisWithPose":
        d = dict(d, pose=d["pose"]["pose"])
    cls = DATACLASS.get(msg_type)
    if cls is None or not is_dataclass(cls):
        return d
    names = {f for f in cls.__dataclass_fields__}
    return cls(**{k: v for k, v in d.items() if k in names})


_TLS = threading.local()
ALLOC_MIN = 64 << 10  # byte arrays from this size go to ``alloc`` (image rows, JPEG bytes, PointCloud2 data)


_ZERO_COPY = object()


def deserialize(data: bytes, msg_type: str, alloc: Optional[Callable[[int], Any]] = None, zero_copy: bool = False):
    """``alloc(n)``: optional destination for large uint8 arrays (a writable buffer of n
    bytes, or None to keep ``bytes``); the message's field then views that buffer.
    ``zero_copy``: large uint8 arrays are views of ``data`` itself (which the message
    then keeps alive).  Image / CompressedImage / PointCloud2 go through the native parse
    (:func:`deserialize_many`) when the runtime library is built."""
    if msg_type in NATIVE_TYPES and _native_rt() is not None:
        return deserialize_many([data], msg_type, alloc, zero_copy)[0]
    return deserialize_py(data, msg_type, alloc, zero_copy)


def deserialize_py(data: bytes, msg_type: str, alloc: Optional[Callable[[int], Any]] = None, zero_copy: bool = False):
    """The schema-driven Python reader (every registered type; the reference semantics the
    native parse is tested against)."""
    mv = memoryview(data)
    _TLS.alloc = _ZERO_COPY if zero_copy else alloc
    try:
        msg, off = _read_msg(mv, 0, msg_type)
    finally:
        _TLS.alloc = None
    if off != len(data):
        raise ValueError(f"{msg_type}: {len(data) - off} trailing bytes")
    return msg


# ------------------------------------------------------------------ native batch parse (sensor messages)
NATIVE_TYPES = {"sensor_msgs/Image": 1, "sensor_msgs/CompressedImage": 2, "sensor_msgs/PointCloud2": 3}
COPY_THREADS = 8  # threads of one batch's payload copy into caller buffers
_STR_CACHE: Dict[bytes, str] = {}
_FIELDS_CACHE: Dict[bytes, List[msgs.PointField]] = {}


def _native_rt():
    try:
        from .. import _native
        return _native.runtime(auto_build=False)
    except Exception:  # noqa: BLE001 - no runtime library: the Python reader below stays exact
        return None


def _str(a, o: int, n: int) -> str:
    b = a[o:o + n].tobytes()
    s = _STR_CACHE.get(b)
    if s is None:
        s = b.decode("utf-8", "replace")
        if len(_STR_CACHE) < 4096:
            _STR_CACHE[b] = s
    return s


def _point_fields(a, o: int, e: int) -> List[msgs.PointField]:
    b = a[o:e].tobytes()
    f = _FIELDS_CACHE.get(b)
    if f is None:
        f, _ = _read(memoryview(b), 0, Field("PointField[]", "fields", "sensor_msgs"))
        if len(_FIELDS_CACHE) < 256:
            _FIELDS_CACHE[b] = f
    return [msgs.PointField(x.name, x.offset, x.datatype, x.count) for x in f]


def deserialize_many(datas, msg_type: str, alloc: Optional[Callable[[int], Any]] = None, zero_copy: bool = False,
                     threads: int = COPY_THREADS) -> list:
    """Deserialise a batch of ``sensor_msgs/Image`` / ``CompressedImage`` / ``PointCloud2``
    wire buffers with one native parse (``tca_ros_parse``, csrc/runtime/ros_wire.cpp) and one
    multi-threaded payload copy (``tca_host_gather_copy``), both outside the GIL.  Same
    result as :func:`deserialize` per message: ``alloc`` puts payloads of ``ALLOC_MIN`` bytes
    or more into caller buffers (the DP ingest arena), ``zero_copy`` makes every payload a
    view of its input (a mapped bag file: nothing is read until a consumer touches it)."""
    import numpy as np

    t = NATIVE_TYPES.get(msg_type)
    rt = _native_rt() if t is not None else None
    if rt is None:
        return [deserialize_py(d, msg_type, alloc, zero_copy) for d in datas]
    n = len(datas)
    if n == 0:
        return []
    arrs = [np.frombuffer(d, np.uint8) for d in datas]
    ptrs = np.fromiter((a.ctypes.data for a in arrs), np.uint64, n)
    lens = np.fromiter((a.size for a in arrs), np.int64, n)
    meta = np.empty((n, 16), np.int64)
    rc = rt.tca_ros_parse(t, n, ptrs.ctypes.data, lens.ctypes.data, meta.ctypes.data)
    if rc != 0:
        if rc > 0:  # the Python reader names what is wrong with that message
            deserialize_py(datas[rc - 1], msg_type)
        raise ValueError(f"{msg_type}: message {rc - 1} does not parse")
    rows = meta.tolist()
    out = []
    cd, cs, cn = [], [], []
    for i, m in enumerate(rows):
        a = arrs[i]
        do, dl = m[11], m[12]
        data = None
        if zero_copy and dl >= ALLOC_MIN:
            data = memoryview(datas[i])[do:do + dl]
        elif alloc is not None and dl >= ALLOC_MIN:
            buf = alloc(dl)
            if buf is not None:
                cd.append(buf.ctypes.data)
                cs.append(int(ptrs[i]) + do)
                cn.append(dl)
                data = memoryview(buf)
        if data is None:
            data = a[do:do + dl].tobytes()
        hdr = msgs.Header(m[0], msgs.Time(m[1], m[2]), _str(a, m[3], m[4]))
        if t == 1:
            out.append(msgs.Image(hdr, m[5], m[6], _str(a, m[7], m[8]), m[9], m[10], data))
        elif t == 2:
            out.append(msgs.CompressedImage(hdr, _str(a, m[5], m[6]), data))
        else:
            out.append(msgs.PointCloud2(hdr, m[5], m[6], _point_fields(a, m[7], m[8]), bool(m[9]), m[10], m[13],
                                        data, bool(m[14])))
    if cd:
        k = len(cd)
        d_ = np.asarray(cd, np.uint64)
        s_ = np.asarray(cs, np.uint64)
        n_ = np.asarray(cn, np.int64)
        if rt.tca_host_gather_copy(k, d_.ctypes.data, s_.ctypes.data, n_.ctypes.data, int(threads)) != 0:
            raise ValueError("tca_host_gather_copy: bad arguments")
    return out
