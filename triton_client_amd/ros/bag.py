"""Bag files: record / replay topic streams (reference: ``rosbag.Bag`` in
``communicator/bag_inference{2d,3d}.py``, ``tools/bag_stitch.py``).

``Bag(path, 'r'|'w')``, ``write(topic, msg, t)``, ``read_messages(topics=...)``
→ ``(topic, msg, t)``, ``get_message_count``, ``get_type_and_topic_info`` —
the ``rosbag.Bag`` API, over two formats:

* **ROS bag v2.0** (:mod:`.rosbag_v2`, pure Python): what real recordings
  are; read whenever the file carries the ``#ROSBAG V2.0`` magic, written for
  paths ending in ``.bag`` (or ``fmt="rosbag"``).
* **TCABAG1**: a compact self-describing fallback — a magic header, then
  length-prefixed msgpack records ``{topic, type, t_ns, msg}`` where ``msg``
  is the message's field dict (bytes payloads stay binary, no pickling — a
  bag never executes code when read); written for other paths.

Reading streams record by record / chunk by chunk (large bags are never
loaded whole).
"""
from __future__ import annotations

import struct
from typing import Iterator, Optional, Sequence, Tuple

import msgpack
import numpy as np

from . import msgs, rosbag_v2, rosmsg

MAGIC = b"TCABAG1\n"


def Bag(path: str, mode: str = "r", fmt: Optional[str] = None, compression: str = "none"):
    """Open a bag: ROS bag v2.0 (read by magic; written for ``*.bag`` or
    ``fmt="rosbag"``) or the TCABAG1 fallback."""
    if mode not in ("r", "w", "a"):
        raise ValueError("mode must be r, w or a")
    if mode == "r":
        return RosBag(path, "r") if rosbag_v2.is_rosbag(path) else TcaBag(path, "r")
    fmt = fmt or ("rosbag" if path.endswith(".bag") else "tcabag")
    if fmt == "rosbag":
        if mode == "a":
            raise ValueError("appending to a ROS bag is not supported")
        return RosBag(path, "w", compression)
    return TcaBag(path, mode)


class RosBag:
    """rosbag.Bag-like wrapper over :mod:`.rosbag_v2`."""

    def __init__(self, path: str, mode: str = "r", compression: str = "none"):
        self.path, self.mode = path, mode
        self._w = rosbag_v2.RosBagWriter(path, compression) if mode == "w" else None
        self._r = rosbag_v2.RosBagReader(path) if mode == "r" else None

    def write(self, topic: str, msg, t: Optional[msgs.Time] = None) -> None:
        self._w.write(topic, msg, t)

    def read_messages(self, topics: Optional[Sequence[str]] = None, start_seq: int = 0, alloc=None,
                      readers: int = 0, mapped: bool = False):
        """``alloc(n)``: where large payloads are deserialised to (e.g. the DP ring's
        ``ingest_buffer``); None keeps ``bytes``.  ``readers``: threads that read uncompressed
        chunks ahead into ``alloc`` buffers (0: the calling thread reads).  ``mapped``: sensor
        payloads stay in the file, as views of its read-only mapping (sharded DP replay)."""
        k = 0
        for topic, m, t in rosbag_v2.read_messages(self._r, topics, alloc, readers, mapped):
            k += 1
            if k <= start_seq:
                continue
            yield topic, m, t

    def get_message_count(self, topic_filters: Optional[Sequence[str]] = None) -> int:
        return sum(1 for c, _, _ in self._r.raw_messages() if not topic_filters or c.topic in topic_filters)

    def get_type_and_topic_info(self):
        info = {}
        for c, _, _ in self._r.raw_messages():
            d = info.setdefault(c.topic, {"type": c.type, "count": 0, "md5sum": c.md5sum})
            d["count"] += 1
        return info

    def close(self) -> None:
        if self._w is not None:
            self._w.close()
        if self._r is not None:
            self._r.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class TcaBag:
    def __init__(self, path: str, mode: str = "r"):
        self.path, self.mode = path, mode
        self._f = open(path, {"r": "rb", "w": "wb", "a": "ab"}[mode])
        if mode == "w":
            self._f.write(MAGIC)
        elif mode == "r":
            if self._f.read(len(MAGIC)) != MAGIC:
                raise ValueError(f"{path}: neither a ROS bag v2.0 nor a triton_client_amd bag")

    def write(self, topic: str, msg, t: Optional[msgs.Time] = None) -> None:
        t = t or getattr(getattr(msg, "header", None), "stamp", None) or msgs.Time.now()
        rec = msgpack.packb({"topic": topic, "type": msgs.TYPE_NAMES.get(type(msg), type(msg).__name__),
                             "t": t.to_nsec(), "msg": msgs.to_dict(msg)}, use_bin_type=True)
        self._f.write(struct.pack("<Q", len(rec)))
        self._f.write(rec)

    def _records(self) -> Iterator[dict]:
        self._f.seek(len(MAGIC))
        while True:
            hdr = self._f.read(8)
            if len(hdr) < 8:
                return
            (n,) = struct.unpack("<Q", hdr)
            yield msgpack.unpackb(self._f.read(n), raw=False)

    def read_messages(self, topics: Optional[Sequence[str]] = None, start_seq: int = 0,
                      alloc=None, readers: int = 0, mapped: bool = False) -> Iterator[Tuple[str, object, msgs.Time]]:
        """Yields (topic, msg, t).  ``start_seq`` resumes a replay after the
        first ``start_seq`` matching messages."""
        k = 0
        for r in self._records():
            if topics and r["topic"] not in topics:
                continue
            k += 1
            if k <= start_seq:
                continue
            cls = msgs.MSG_TYPES.get(r["type"])
            m = msgs.from_dict(cls, r["msg"]) if cls else r["msg"]
            raw = getattr(m, "data", None)
            if alloc is not None and isinstance(raw, (bytes, bytearray)) and len(raw) >= rosmsg.ALLOC_MIN:
                buf = alloc(len(raw))
                if buf is not None:
                    buf[:] = np.frombuffer(raw, np.uint8)
                    m.data = memoryview(buf)
            t = msgs.Time(r["t"] // 1_000_000_000, r["t"] % 1_000_000_000)
            yield r["topic"], m, t

    def get_message_count(self, topic_filters: Optional[Sequence[str]] = None) -> int:
        return sum(1 for r in self._records() if not topic_filters or r["topic"] in topic_filters)

    def get_type_and_topic_info(self):
        info = {}
        for r in self._records():
            d = info.setdefault(r["topic"], {"type": r["type"], "count": 0})
            d["count"] += 1
        return info

    def close(self) -> None:
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def stitch(src: str, dst: str, n: int = 500, topics: Optional[Sequence[str]] = None) -> int:
    """Copy the first n messages (reference tools/bag_stitch.py)."""
    k = 0
    with Bag(src) as bi, Bag(dst, "w") as bo:
        for topic, m, t in bi.read_messages(topics):
            if k >= n:
                break
            bo.write(topic, m, t)
            k += 1
    return k
