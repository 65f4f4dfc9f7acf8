"""rospy / cv_bridge / point_cloud2 surface used by the inference drivers.

If a real ROS1 environment is importable (``rospy``), the drivers use it
unchanged; otherwise this module provides the same calls over the
in-process :class:`~triton_client_amd.ros.bus.TopicBus`:
``init_node, Subscriber, Publisher, spin, loginfo/logwarn/logerr, get_param,
is_shutdown, signal_shutdown, Time`` plus cv_bridge-style image conversion
and PointCloud2 construction.
"""
from __future__ import annotations

import io
import logging
import threading
from typing import Optional, Sequence

import numpy as np

from . import msgs
from .bus import default_bus

try:  # pragma: no cover - real ROS is not installed on the dev/GPU hosts
    import rospy as _rospy  # type: ignore
    HAVE_ROSPY = True
except Exception:
    _rospy = None
    HAVE_ROSPY = False

log = logging.getLogger("triton_client_amd.ros")
_PARAMS = {}
_NODE = {"name": None}
Time = msgs.Time


def init_node(name: str, anonymous: bool = False, **kw) -> None:
    if HAVE_ROSPY:
        _rospy.init_node(name, anonymous=anonymous, **kw)
    _NODE["name"] = name


def get_param(name: str, default=None):
    if HAVE_ROSPY:
        return _rospy.get_param(name, default)
    return _PARAMS.get(name.lstrip("~/"), default)


def set_param(name: str, value) -> None:
    _PARAMS[name.lstrip("~/")] = value


def loginfo(msg, *a):
    (_rospy.loginfo if HAVE_ROSPY else log.info)(msg, *a)


def logwarn(msg, *a):
    (_rospy.logwarn if HAVE_ROSPY else log.warning)(msg, *a)


def logerr(msg, *a):
    (_rospy.logerr if HAVE_ROSPY else log.error)(msg, *a)


def _raw_ingest(msg_type, callback, ingest):
    """rospy ``AnyMsg`` callback: the wire bytes of an Image / CompressedImage / PointCloud2 parsed
    by the native ROS parser (csrc/runtime/ros_wire.cpp, GIL released) with the payload copied
    straight into ``ingest(n)`` buffers -- the data-parallel ring's ingest arena -- instead of
    genpy's per-field Python deserialiser building a ``bytes`` payload that the ring then copies
    again."""
    from . import rosmsg

    def cb(raw):
        # the publisher's actual type (AnyMsg keeps the connection header): an Image topic
        # subscribed as CompressedImage is parsed as what it is
        hdr = getattr(raw, "_connection_header", None) or {}
        return callback(rosmsg.deserialize(raw._buff, hdr.get("type", msg_type), alloc=ingest))
    return cb


class Subscriber:
    def __init__(self, topic: str, msg_type, callback, queue_size: Optional[int] = None, bus=None, ingest=None):
        """``ingest(n)``: with a real ROS master, sensor messages are received as raw bytes
        (``rospy.AnyMsg``) and deserialised natively with their payloads in ``ingest`` buffers
        (the data-parallel drivers pass the host ring's ``ingest_buffer``)."""
        self.topic = topic
        if HAVE_ROSPY and bus is None:
            from . import rosmsg
            name = msg_type if isinstance(msg_type, str) else (getattr(msg_type, "_type", None)
                                                               or rosmsg.TYPE_OF.get(msg_type))
            if ingest is not None and name in rosmsg.NATIVE_TYPES:
                cb = _raw_ingest(name, callback, ingest)
                self._impl = _rospy.Subscriber(topic, _rospy.AnyMsg, cb, queue_size=queue_size)
            else:
                self._impl = _rospy.Subscriber(topic, msg_type, callback, queue_size=queue_size)
            self._bus = None
        else:
            self._bus = bus or default_bus()
            self._impl = self._bus.subscribe(topic, callback, queue_size)

    def unregister(self):
        if self._bus is not None:
            self._bus.unsubscribe(self.topic, self._impl)
        else:
            self._impl.unregister()


class Publisher:
    def __init__(self, topic: str, msg_type, queue_size: Optional[int] = None, bus=None):
        self.topic = topic
        if HAVE_ROSPY and bus is None:
            self._impl = _rospy.Publisher(topic, msg_type, queue_size=queue_size)
            self._bus = None
        else:
            self._bus = bus or default_bus()
            self._impl = None

    def publish(self, msg) -> None:
        if self._bus is not None:
            self._bus.publish(self.topic, msg)
        else:
            if isinstance(getattr(msg, "data", None), memoryview):  # genpy packs uint8[] from bytes
                msg.data = msg.data.tobytes()
            self._impl.publish(msg)

    def get_num_connections(self) -> int:
        return self._bus.num_subscribers(self.topic) if self._bus is not None else self._impl.get_num_connections()


def is_shutdown(bus=None) -> bool:
    if HAVE_ROSPY and bus is None:
        return _rospy.is_shutdown()
    return (bus or default_bus()).shutdown_event.is_set()


def signal_shutdown(reason: str = "", bus=None) -> None:
    if HAVE_ROSPY and bus is None:
        _rospy.signal_shutdown(reason)
    (bus or default_bus()).shutdown_event.set()


def spin(bus=None, timeout: Optional[float] = None) -> None:
    if HAVE_ROSPY and bus is None:
        _rospy.spin()
        return
    (bus or default_bus()).shutdown_event.wait(timeout)


# ---------------------------------------------------------------- cv_bridge equivalents
def imgmsg_to_numpy(msg: msgs.Image, desired_encoding: str = "rgb8") -> np.ndarray:
    ch = {"rgb8": 3, "bgr8": 3, "rgba8": 4, "bgra8": 4, "mono8": 1}[msg.encoding]
    a = np.frombuffer(msg.data, np.uint8).reshape(msg.height, msg.step // 1)[:, : msg.width * ch]
    a = a.reshape(msg.height, msg.width, ch)
    if ch == 1:
        a = np.repeat(a, 3, axis=2)
    a = a[..., :3]
    if desired_encoding == "rgb8" and msg.encoding.startswith("bgr"):
        a = a[..., ::-1]
    elif desired_encoding == "bgr8" and msg.encoding.startswith("rgb"):
        a = a[..., ::-1]
    return np.ascontiguousarray(a)


def numpy_to_imgmsg(img: np.ndarray, encoding: str = "rgb8", header: Optional[msgs.Header] = None) -> msgs.Image:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape[:2]
    return msgs.Image(header=header or msgs.Header(), height=h, width=w, encoding=encoding, step=img.strides[0],
                      data=img.tobytes())


def jpeg_encode(img_rgb: np.ndarray, quality: int = 90) -> bytes:
    from PIL import Image as PILImage

    buf = io.BytesIO()
    PILImage.fromarray(img_rgb).save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def jpeg_decode_rgb(data: bytes) -> np.ndarray:
    """CompressedImage → RGB uint8 (the reference: cv2.imdecode + BGR→RGB,
    ros_inference.py:119-131).  Decoded on the host (libjpeg via PIL); rocJPEG
    is not available in this ROCm image."""
    from PIL import Image as PILImage

    return np.asarray(PILImage.open(io.BytesIO(data)).convert("RGB"))


def compressed_to_numpy(msg: msgs.CompressedImage) -> np.ndarray:
    return jpeg_decode_rgb(msg.data)


# ---------------------------------------------------------------- point clouds
XYZI_FIELDS = [msgs.PointField("x", 0, 7, 1), msgs.PointField("y", 4, 7, 1), msgs.PointField("z", 8, 7, 1),
               msgs.PointField("intensity", 12, 7, 1)]


def create_cloud_xyzi(points: np.ndarray, header: Optional[msgs.Header] = None) -> msgs.PointCloud2:
    p = np.ascontiguousarray(points[:, :4], np.float32)
    return msgs.PointCloud2(header=header or msgs.Header(), height=1, width=p.shape[0], fields=list(XYZI_FIELDS),
                            point_step=16, row_step=16 * p.shape[0], data=p.tobytes(), is_dense=False)


def cloud_layout(msg: msgs.PointCloud2, names: Sequence[str] = ("x", "y", "z", "intensity")):
    """PointLayout (offsets/datatypes of the requested fields) of a PointCloud2."""
    from ..ops.lidar import PointLayout

    by = {f.name: f for f in msg.fields}
    missing = [n for n in names if n not in by]
    if missing:
        raise ValueError(f"PointCloud2 lacks fields {missing}")
    return PointLayout(msg.point_step, tuple(by[n].offset for n in names), tuple(by[n].datatype for n in names))


_PF_NP = {1: "i1", 2: "u1", 3: "<i2", 4: "<u2", 5: "<i4", 6: "<u4", 7: "<f4", 8: "<f8"}


def cloud_to_numpy(msg: msgs.PointCloud2, names: Sequence[str] = ("x", "y", "z", "intensity"),
                   skip_nans: bool = True, normalize_intensity: bool = False, z_offset: float = 0.0) -> np.ndarray:
    """Vectorised ``read_points(field_names, skip_nans)`` → [N, len(names)] float32
    via a strided structured view of the payload (the reference builds the
    array from a Python generator, 138 ms per 64-beam sweep).
    Optional reference post-steps: intensity /= max, z += offset
    (ros_inference3d.py:127-128)."""
    by = {f.name: f for f in msg.fields}
    n = msg.width * msg.height
    dt = np.dtype({"names": list(names), "formats": [_PF_NP[by[k].datatype] for k in names],
                   "offsets": [by[k].offset for k in names], "itemsize": msg.point_step})
    rec = np.frombuffer(msg.data, dtype=dt, count=n)
    out = np.empty((n, len(names)), np.float32)
    for j, k in enumerate(names):
        out[:, j] = rec[k]
    if skip_nans:
        out = out[~np.isnan(out).any(1)]
    if normalize_intensity and len(names) > 3 and len(out):
        m = out[:, 3].max()
        if m > 0:
            out[:, 3] /= m
    if z_offset and len(names) > 2:
        out[:, 2] += z_offset
    return out


def yaw2quaternion(yaw: float) -> msgs.Quaternion:
    """Rotation about +z (reference ros_inference3d.py:117-118 via pyquaternion)."""
    return msgs.Quaternion(0.0, 0.0, float(np.sin(yaw / 2)), float(np.cos(yaw / 2)))
