"""ROS message types used by the reference, as plain dataclasses with the
same field names (sensor_msgs, std_msgs, geometry_msgs, jsk_recognition_msgs,
vision_msgs).  When a real ROS1 install is present, ``ros.compat`` uses the
genuine message classes instead; these mirror them for the GPU box / CI.
"""
from __future__ import annotations

import time as _time
from dataclasses import dataclass, field, fields, is_dataclass
from typing import Any, Dict, List


class ArrayList(list):
    """A message's list field (``BoundingBoxArray.boxes``, ``Detection2DArray.detections``)
    kept as the detector's columns until something reads it.

    The live drivers publish one message per frame at thousands of frames/s;
    building every ``BoundingBox`` / ``Detection2D`` object up front costs more
    host time than the GPU step.  This list is built by ``build()`` on first
    access (iteration, indexing, ``len`` is known without building), so a
    subscriber that reads the field sees ordinary message objects, while one
    that only forwards or serialises the message never pays for them
    (``ros.rosmsg`` serialises an unbuilt BoundingBoxArray straight from the
    columns).  ``columns`` holds the arrays it was made from."""

    def __init__(self, n: int, build, columns=None):
        super().__init__()
        self._n, self._build, self.columns = int(n), build, columns

    @property
    def built(self) -> bool:
        return self._build is None

    def _fill(self) -> None:
        b = self._build
        if b is not None:
            self._build = None
            list.extend(self, b())

    def __len__(self):
        return self._n if self._build is not None else list.__len__(self)

    def __bool__(self):
        return len(self) > 0

    def __reduce__(self):  # pickles / deep-copies as a plain list of messages
        self._fill()
        return (list, (list(list.__iter__(self)),))


def _filled(name):
    base = getattr(list, name)

    def method(self, *a, **kw):
        self._fill()
        return base(self, *a, **kw)
    method.__name__ = name
    return method


for _m in ("__iter__", "__getitem__", "__contains__", "__eq__", "__ne__", "__repr__", "__reversed__", "__add__",
           "__mul__", "__rmul__", "__iadd__", "__imul__", "__setitem__", "__delitem__", "__lt__", "__le__",
           "__gt__", "__ge__", "index", "count", "copy", "append", "extend", "insert", "pop", "remove", "sort",
           "reverse", "clear"):
    setattr(ArrayList, _m, _filled(_m))
ArrayList.__hash__ = None


@dataclass
class Time:
    secs: int = 0
    nsecs: int = 0

    @staticmethod
    def now() -> "Time":
        t = _time.time_ns()
        return Time(t // 1_000_000_000, t % 1_000_000_000)

    @staticmethod
    def from_sec(s: float) -> "Time":
        return Time(int(s), int(round((s - int(s)) * 1e9)))

    def to_sec(self) -> float:
        return self.secs + self.nsecs * 1e-9

    def to_nsec(self) -> int:
        return self.secs * 1_000_000_000 + self.nsecs


@dataclass
class Header:
    seq: int = 0
    stamp: Time = field(default_factory=Time)
    frame_id: str = ""


# ---------------------------------------------------------------- sensor_msgs
@dataclass
class Image:
    header: Header = field(default_factory=Header)
    height: int = 0
    width: int = 0
    encoding: str = "rgb8"
    is_bigendian: int = 0
    step: int = 0
    data: bytes = b""


@dataclass
class CompressedImage:
    header: Header = field(default_factory=Header)
    format: str = "jpeg"
    data: bytes = b""


@dataclass
class PointField:
    INT8 = 1
    UINT8 = 2
    INT16 = 3
    UINT16 = 4
    INT32 = 5
    UINT32 = 6
    FLOAT32 = 7
    FLOAT64 = 8
    name: str = ""
    offset: int = 0
    datatype: int = 7
    count: int = 1


@dataclass
class PointCloud2:
    header: Header = field(default_factory=Header)
    height: int = 1
    width: int = 0
    fields: List[PointField] = field(default_factory=list)
    is_bigendian: bool = False
    point_step: int = 16
    row_step: int = 0
    data: bytes = b""
    is_dense: bool = False


# ---------------------------------------------------------------- geometry_msgs
@dataclass
class Point:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


@dataclass
class Vector3:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0


@dataclass
class Quaternion:
    x: float = 0.0
    y: float = 0.0
    z: float = 0.0
    w: float = 1.0


@dataclass
class Pose:
    position: Point = field(default_factory=Point)
    orientation: Quaternion = field(default_factory=Quaternion)


@dataclass
class Pose2D:
    x: float = 0.0
    y: float = 0.0
    theta: float = 0.0


# ---------------------------------------------------------------- jsk_recognition_msgs
@dataclass
class BoundingBox:
    header: Header = field(default_factory=Header)
    pose: Pose = field(default_factory=Pose)
    dimensions: Vector3 = field(default_factory=Vector3)
    value: float = 0.0
    label: int = 0


@dataclass
class BoundingBoxArray:
    header: Header = field(default_factory=Header)
    boxes: List[BoundingBox] = field(default_factory=list)


# ---------------------------------------------------------------- vision_msgs
@dataclass
class ObjectHypothesisWithPose:
    id: int = 0
    score: float = 0.0
    pose: Pose = field(default_factory=Pose)


@dataclass
class BoundingBox2D:
    center: Pose2D = field(default_factory=Pose2D)
    size_x: float = 0.0
    size_y: float = 0.0


@dataclass
class Detection2D:
    header: Header = field(default_factory=Header)
    results: List[ObjectHypothesisWithPose] = field(default_factory=list)
    bbox: BoundingBox2D = field(default_factory=BoundingBox2D)
    source_img: Image = field(default_factory=Image)


@dataclass
class Detection2DArray:
    header: Header = field(default_factory=Header)
    detections: List[Detection2D] = field(default_factory=list)


@dataclass
class BoundingBox3D:
    center: Pose = field(default_factory=Pose)
    size: Vector3 = field(default_factory=Vector3)


@dataclass
class Detection3D:
    header: Header = field(default_factory=Header)
    results: List[ObjectHypothesisWithPose] = field(default_factory=list)
    bbox: BoundingBox3D = field(default_factory=BoundingBox3D)


@dataclass
class Detection3DArray:
    header: Header = field(default_factory=Header)
    detections: List[Detection3D] = field(default_factory=list)


MSG_TYPES: Dict[str, type] = {
    "sensor_msgs/Image": Image, "sensor_msgs/CompressedImage": CompressedImage,
    "sensor_msgs/PointCloud2": PointCloud2, "sensor_msgs/PointField": PointField,
    "std_msgs/Header": Header, "jsk_recognition_msgs/BoundingBoxArray": BoundingBoxArray,
    "jsk_recognition_msgs/BoundingBox": BoundingBox, "vision_msgs/Detection2DArray": Detection2DArray,
    "vision_msgs/Detection3DArray": Detection3DArray,
}
TYPE_NAMES = {v: k for k, v in MSG_TYPES.items()}


def to_dict(msg: Any) -> Any:
    if is_dataclass(msg):
        return {f.name: to_dict(getattr(msg, f.name)) for f in fields(msg)}
    if isinstance(msg, list):
        return [to_dict(m) for m in msg]
    return msg


def from_dict(cls, d: Any):
    """Rebuild a dataclass message from to_dict() output."""
    import typing

    if not is_dataclass(cls):
        return d
    hints = typing.get_type_hints(cls)
    kw = {}
    for f in fields(cls):
        if f.name not in d:
            continue
        t = hints[f.name]
        v = d[f.name]
        origin = getattr(t, "__origin__", None)
        if origin in (list, List):
            (inner,) = t.__args__
            kw[f.name] = [from_dict(inner, x) for x in v]
        elif is_dataclass(t):
            kw[f.name] = from_dict(t, v)
        else:
            kw[f.name] = v
    return cls(**kw)
