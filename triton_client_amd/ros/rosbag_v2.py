"""ROS1 bag format 2.0 reader / writer, pure Python (``rosbag`` is not installed).

The reference replays and records real ``.bag`` files
(``communicator/bag_inference2d.py:34-35``, ``communicator/bag_inference3d.py:62-63,182-183``,
``tools/bag_stitch.py:4-5``, ``tools/pc_extractor.py:30``).  Record layout (bag
format 2.0): ``#ROSBAG V2.0\\n``, then records ``<u32 header_len><header><u32
data_len><data>``, a header being ``<u32 len>name=value`` fields with an
``op`` byte:

* 0x03 bag header — ``index_pos`` (u64), ``conn_count``, ``chunk_count``;
  padded to 4096 bytes;
* 0x05 chunk — ``compression`` (none / bz2 / lz4), ``size``; its data is
  connection + message-data records;
* 0x07 connection — ``conn``, ``topic``; data = a field block with ``topic``,
  ``type``, ``md5sum``, ``message_definition``;
* 0x02 message data — ``conn``, ``time`` (u32 sec, u32 nsec); data = the
  serialised message (:mod:`.rosmsg`);
* 0x04 index data (per connection after each chunk: ``ver`` 1, ``conn``,
  ``count``; data = (time, offset-in-chunk) pairs) and 0x06 chunk info (in
  the index section: ``ver``, ``chunk_pos``, ``start_time``, ``end_time``,
  ``count``; data = (conn, msg_count) pairs).

Reading streams chunk by chunk (a bag is never loaded whole); messages of
types without a schema come back as :class:`RawMessage`.  bz2 chunks are
read with the stdlib; lz4 only if the ``lz4`` module is importable.
"""
from __future__ import annotations

import bz2
import os
import struct
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

from . import msgs, rosmsg

MAGIC = b"#ROSBAG V2.0\n"
OP_MSG, OP_BAG_HEADER, OP_INDEX, OP_CHUNK, OP_CHUNK_INFO, OP_CONNECTION = 0x02, 0x03, 0x04, 0x05, 0x06, 0x07
HEADER_LEN = 4096
CHUNK_THRESHOLD = 768 * 1024


@dataclass
class RawMessage:
    type: str
    md5sum: str
    data: bytes


@dataclass
class Connection:
    id: int
    topic: str
    type: str
    md5sum: str
    definition: str


def _fields(d: Dict[str, bytes]) -> bytes:
    out = bytearray()
    for k, v in d.items():
        f = k.encode() + b"=" + v
        out += struct.pack("<I", len(f)) + f
    return bytes(out)


def _parse_fields(b: bytes) -> Dict[str, bytes]:
    if not isinstance(b, bytes):
        b = bytes(b)
    d, off = {}, 0
    while off < len(b):
        (n,) = struct.unpack_from("<I", b, off)
        f = b[off + 4: off + 4 + n]
        k, _, v = f.partition(b"=")
        d[k.decode()] = v
        off += 4 + n
    return d


def _record(header: Dict[str, bytes], data: bytes) -> bytes:
    h = _fields(header)
    return struct.pack("<I", len(h)) + h + struct.pack("<I", len(data)) + data


def _u32(v: int) -> bytes:
    return struct.pack("<I", v)


def _time(t: msgs.Time) -> bytes:
    return struct.pack("<II", t.secs, t.nsecs)


def _read_time(b: bytes) -> msgs.Time:
    s, ns = struct.unpack("<II", b)
    return msgs.Time(s, ns)


class RosBagWriter:
    def __init__(self, path: str, compression: str = "none", chunk_threshold: int = CHUNK_THRESHOLD):
        if compression not in ("none", "bz2"):
            raise ValueError("compression: none or bz2")
        self.f = open(path, "wb")
        self.compression, self.threshold = compression, chunk_threshold
        self.conns: Dict[Tuple[str, str], Connection] = {}
        self.chunk_infos: List[Tuple[int, msgs.Time, msgs.Time, Dict[int, int]]] = []
        self._chunk = bytearray()
        self._chunk_conns: set = set()
        self._index: Dict[int, List[Tuple[msgs.Time, int]]] = {}
        self._t0 = self._t1 = None
        self.f.write(MAGIC)
        self._write_bag_header(0, 0, 0)

    def _write_bag_header(self, index_pos: int, conn_count: int, chunk_count: int) -> None:
        h = _fields({"op": bytes([OP_BAG_HEADER]), "index_pos": struct.pack("<Q", index_pos),
                     "conn_count": _u32(conn_count), "chunk_count": _u32(chunk_count)})
        pad = HEADER_LEN - 4 - len(h) - 4
        self.f.write(struct.pack("<I", len(h)) + h + struct.pack("<I", pad) + b" " * pad)

    def _conn_record(self, c: Connection) -> bytes:
        data = _fields({"topic": c.topic.encode(), "type": c.type.encode(), "md5sum": c.md5sum.encode(),
                        "message_definition": c.definition.encode()})
        return _record({"op": bytes([OP_CONNECTION]), "conn": _u32(c.id), "topic": c.topic.encode()}, data)

    def write(self, topic: str, msg, t: Optional[msgs.Time] = None) -> None:
        t = t or getattr(getattr(msg, "header", None), "stamp", None) or msgs.Time.now()
        if isinstance(msg, RawMessage):
            mtype, md5, data, definition = msg.type, msg.md5sum, msg.data, ""
        else:
            mtype = rosmsg.TYPE_OF[type(msg)]
            md5, data, definition = rosmsg.md5sum(mtype), rosmsg.serialize(msg, mtype), rosmsg.full_definition(mtype)
        key = (topic, mtype)
        c = self.conns.get(key)
        if c is None:
            c = self.conns[key] = Connection(len(self.conns), topic, mtype, md5, definition)
        if c.id not in self._chunk_conns:
            self._chunk += self._conn_record(c)
            self._chunk_conns.add(c.id)
        self._index.setdefault(c.id, []).append((t, len(self._chunk)))
        self._chunk += _record({"op": bytes([OP_MSG]), "conn": _u32(c.id), "time": _time(t)}, data)
        ns = t.to_nsec()
        self._t0 = t if self._t0 is None or ns < self._t0.to_nsec() else self._t0
        self._t1 = t if self._t1 is None or ns > self._t1.to_nsec() else self._t1
        if len(self._chunk) >= self.threshold:
            self._flush_chunk()

    def _flush_chunk(self) -> None:
        if not self._chunk:
            return
        raw = bytes(self._chunk)
        data = bz2.compress(raw) if self.compression == "bz2" else raw
        pos = self.f.tell()
        self.f.write(_record({"op": bytes([OP_CHUNK]), "compression": self.compression.encode(),
                              "size": _u32(len(raw))}, data))
        counts = {}
        for cid, entries in sorted(self._index.items()):
            body = b"".join(_time(t) + _u32(off) for t, off in entries)
            self.f.write(_record({"op": bytes([OP_INDEX]), "ver": _u32(1), "conn": _u32(cid),
                                  "count": _u32(len(entries))}, body))
            counts[cid] = len(entries)
        self.chunk_infos.append((pos, self._t0, self._t1, counts))
        self._chunk, self._chunk_conns, self._index = bytearray(), set(), {}
        self._t0 = self._t1 = None

    def close(self) -> None:
        if self.f.closed:
            return
        self._flush_chunk()
        index_pos = self.f.tell()
        for c in sorted(self.conns.values(), key=lambda c: c.id):
            self.f.write(self._conn_record(c))
        for pos, t0, t1, counts in self.chunk_infos:
            body = b"".join(_u32(cid) + _u32(n) for cid, n in sorted(counts.items()))
            self.f.write(_record({"op": bytes([OP_CHUNK_INFO]), "ver": _u32(1), "chunk_pos": struct.pack("<Q", pos),
                                  "start_time": _time(t0), "end_time": _time(t1), "count": _u32(len(counts))},
                                 body))
        self.f.seek(len(MAGIC))
        self._write_bag_header(index_pos, len(self.conns), len(self.chunk_infos))
        self.f.close()


class RosBagReader:
    def __init__(self, path: str):
        self.path = os.path.abspath(path)
        self.f = open(path, "rb")
        if self.f.read(len(MAGIC)) != MAGIC:
            raise ValueError(f"{path}: not a ROS bag v2.0")
        self.conns: Dict[int, Connection] = {}
        self.mm = None

    def _read_record(self, f, alloc=None) -> Optional[Tuple[Dict[str, bytes], bytes]]:
        """``alloc``: an uncompressed chunk is read straight into ``alloc(n)`` (the DP ring's
        ingest arena) and its messages are views of it -- no copy between the file and the ring."""
        b = f.read(4)
        if len(b) < 4:
            return None
        (hl,) = struct.unpack("<I", b)
        h = _parse_fields(f.read(hl))
        (dl,) = struct.unpack("<I", f.read(4))
        if (alloc is not None and dl >= rosmsg.ALLOC_MIN and h.get("op", b"\0")[0] == OP_CHUNK
                and h.get("compression", b"none") == b"none"):
            buf = alloc(dl)
            if buf is not None:
                if f.readinto(memoryview(buf)) != dl:
                    raise ValueError("truncated ROS bag chunk")
                return h, memoryview(buf)
        return h, f.read(dl)

    def _conn(self, h, data) -> Connection:
        d = _parse_fields(data)
        cid = struct.unpack("<I", h["conn"])[0]
        c = Connection(cid, h["topic"].decode(), d["type"].decode(), d.get("md5sum", b"*").decode(),
                       d.get("message_definition", b"").decode("utf-8", "replace"))
        self.conns[cid] = c
        return c

    @staticmethod
    def _decompress(kind: str, data: bytes) -> bytes:
        if kind == "none":
            return data
        if kind == "bz2":
            return bz2.decompress(data)
        if kind == "lz4":
            try:
                import lz4.frame  # noqa: F401
            except ImportError as e:
                raise RuntimeError("lz4-compressed bag chunk and the lz4 module is not installed") from e
            import lz4.frame
            return lz4.frame.decompress(data)
        raise ValueError(f"unknown chunk compression {kind!r}")

    def _iter_payload(self, blob: bytes) -> Iterator[Tuple[Connection, msgs.Time, bytes]]:
        off = 0
        n = len(blob)
        while off + 8 <= n:
            (hl,) = struct.unpack_from("<I", blob, off)
            h = _parse_fields(bytes(blob[off + 4: off + 4 + hl]))
            (dl,) = struct.unpack_from("<I", blob, off + 4 + hl)
            data = blob[off + 8 + hl: off + 8 + hl + dl]
            off += 8 + hl + dl
            op = h["op"][0]
            if op == OP_CONNECTION:
                self._conn(h, data)
            elif op == OP_MSG:
                cid = struct.unpack("<I", h["conn"])[0]
                yield self.conns[cid], _read_time(h["time"]), data

    def _records(self) -> Iterator[Tuple[Dict[str, bytes], int, int]]:
        """(header, data offset, data length) of every record, reading headers only."""
        f = self.f
        f.seek(len(MAGIC))
        while True:
            b = f.read(4)
            if len(b) < 4:
                return
            (hl,) = struct.unpack("<I", b)
            h = _parse_fields(f.read(hl))
            b = f.read(4)
            if len(b) < 4:
                return
            (dl,) = struct.unpack("<I", b)
            off = f.tell()
            yield h, off, dl
            f.seek(off + dl)

    def _prefetched(self, alloc, readers: int, ahead: int):
        """Records with the data of uncompressed chunks read ahead by ``readers`` threads
        (``os.preadv`` into ``alloc`` buffers, GIL released) -- a single reader thread bounds bag
        replay at one core's copy rate otherwise (``tools/fanout_bench.py --bag``)."""
        import collections
        from concurrent.futures import ThreadPoolExecutor

        fd = self.f.fileno()

        def read_into(buf, off, n):
            mv = memoryview(buf)
            got = 0
            while got < n:
                k = os.preadv(fd, [mv[got:]], off + got)
                if k <= 0:
                    raise ValueError("truncated ROS bag chunk")
                got += k
            return mv

        recs = list(self._records())
        pending = collections.deque()
        with ThreadPoolExecutor(readers, thread_name_prefix="bagread") as pool:
            it = iter(recs)

            def fill():
                while len(pending) < ahead:
                    r = next(it, None)
                    if r is None:
                        return
                    h, off, dl = r
                    fut = None
                    if (dl >= rosmsg.ALLOC_MIN and h.get("op", b"\0")[0] == OP_CHUNK
                            and h.get("compression", b"none") == b"none"):
                        buf = alloc(dl)
                        if buf is not None:
                            fut = pool.submit(read_into, buf, off, dl)
                    pending.append((h, off, dl, fut))
            fill()
            while pending:
                h, off, dl, fut = pending.popleft()
                if fut is not None:
                    data = fut.result()
                else:
                    data = os.pread(fd, dl, off)
                fill()
                yield h, data

    def raw_messages(self, alloc=None, readers: int = 0, ahead: int = 8) -> Iterator[Tuple[Connection, msgs.Time, bytes]]:
        """(connection, time, serialised bytes) in file order (memoryviews into ``alloc``
        buffers for uncompressed chunks when ``alloc`` is given; with ``readers`` > 0 those
        chunks are read ahead by that many threads, up to ``ahead`` records in flight)."""
        if alloc is not None and readers > 0:
            for h, data in self._prefetched(alloc, readers, ahead):
                op = h["op"][0]
                if op == OP_CHUNK:
                    yield from self._iter_payload(self._decompress(h["compression"].decode(), data))
                elif op == OP_CONNECTION:
                    self._conn(h, data)
                elif op == OP_MSG:
                    cid = struct.unpack("<I", h["conn"])[0]
                    yield self.conns[cid], _read_time(h["time"]), data
            return
        self.f.seek(len(MAGIC))
        while True:
            rec = self._read_record(self.f, alloc)
            if rec is None:
                return
            h, data = rec
            op = h["op"][0]
            if op == OP_CHUNK:
                yield from self._iter_payload(self._decompress(h["compression"].decode(), data))
            elif op == OP_CONNECTION:
                self._conn(h, data)
            elif op == OP_MSG:
                cid = struct.unpack("<I", h["conn"])[0]
                yield self.conns[cid], _read_time(h["time"]), data
            # bag header, index data, chunk info: nothing to replay

    def mapping(self):
        """The bag file's read-only shared mapping (made on first use; random access advice,
        so touching a message's first page does not read its payload ahead)."""
        if self.mm is None:
            import mmap
            self.mm = mmap.mmap(self.f.fileno(), 0, access=mmap.ACCESS_READ)
            try:
                self.mm.madvise(mmap.MADV_RANDOM)
            except (AttributeError, OSError):
                pass
            from ..parallel.host_ring import FileMaps
            FileMaps.register(self.path, self.mm)
        return self.mm

    WINDOW = 64  # messages parsed per native call batch (per type) in mapped_messages

    def mapped_messages(self, topics: Optional[Sequence[str]] = None) -> Iterator[Tuple[Connection, msgs.Time, object]]:
        """(connection, time, message) in file order, with the sensor messages' payloads left in
        the file: each ``data`` is a view of :meth:`mapping` and nothing of it is read until a
        consumer touches it.  One native pass (``tca_bag_index``) walks the top-level records and
        the records inside uncompressed chunks; windows of up to :attr:`WINDOW` messages are
        parsed with one native call per message type (``rosmsg.deserialize_many``).  So this
        reads only record headers and message prefixes.  Sharded data-parallel replay
        (``parallel/ring_dp.py``): rank 0 orders and publishes these messages, and every rank
        reads its own shard's payloads from its own mapping of the file.  Compressed chunks
        (and hosts without the runtime library) take the ordinary path."""
        import numpy as np

        rt = rosmsg._native_rt()
        if rt is None or not hasattr(rt, "tca_bag_index"):
            for c, t, data in self.raw_messages():
                if not topics or c.topic in topics:
                    yield c, t, self.decode(c, data)
            return
        mm = self.mapping()
        mv = memoryview(mm)
        base = np.frombuffer(mm, np.uint8).ctypes.data if len(mm) else 0
        want = None if not topics else set(topics)
        cap = 1024
        cols = [np.empty(cap, t) for t in (np.int32, np.int32, np.uint32, np.uint32, np.int64, np.int64, np.int64,
                                           np.int64)]
        ptrs = [c.ctypes.data for c in cols]
        state = np.array([len(MAGIC), 0], np.int64)
        pending: List[Tuple[Connection, msgs.Time, int, int]] = []
        conns = self.conns

        def flush():
            if not pending:
                return []
            groups: Dict[str, List[int]] = {}
            for i, (c, _, _, _) in enumerate(pending):
                groups.setdefault(c.type, []).append(i)
            parsed: List[object] = [None] * len(pending)
            for typ, idx in groups.items():
                ms = rosmsg.deserialize_many([mv[pending[i][2]:pending[i][2] + pending[i][3]] for i in idx], typ,
                                             zero_copy=True)
                for i, m in zip(idx, ms):
                    parsed[i] = m
            out = [(c, t, m) for (c, t, _, _), m in zip(pending, parsed)]
            pending.clear()
            return out
        while True:
            k = int(rt.tca_bag_index(base, len(mm), state.ctypes.data, cap, *ptrs))
            if k < 0:
                raise ValueError(f"{self.path}: malformed record near byte {int(state[0])}")
            if k == 0:
                break
            ops, cids, secs, nsecs, hoffs, hlens, doffs, dlens = (c[:k].tolist() for c in cols)
            for i in range(k):
                o = ops[i]
                if o == OP_MSG:
                    c = conns[cids[i]]
                    if want is not None and c.topic not in want:
                        continue
                    t = msgs.Time(secs[i], nsecs[i])
                    if c.type in rosmsg.NATIVE_TYPES:
                        pending.append((c, t, doffs[i], dlens[i]))
                        if len(pending) >= self.WINDOW:
                            yield from flush()
                    else:
                        yield from flush()
                        yield c, t, self.decode(c, mv[doffs[i]:doffs[i] + dlens[i]])
                elif o == OP_CONNECTION:
                    if cids[i] not in conns:
                        h0 = hoffs[i]
                        self._conn(_parse_fields(bytes(mv[h0:h0 + hlens[i]])), bytes(mv[doffs[i]:doffs[i] + dlens[i]]))
                elif o == OP_CHUNK:  # compressed: the ordinary path
                    yield from flush()
                    h = _parse_fields(bytes(mv[hoffs[i]:hoffs[i] + hlens[i]]))
                    blob = self._decompress(h["compression"].decode(), bytes(mv[doffs[i]:doffs[i] + dlens[i]]))
                    for c, t, data in self._iter_payload(blob):
                        if want is None or c.topic in want:
                            yield c, t, self.decode(c, data)
        yield from flush()

    @staticmethod
    def decode(conn: Connection, data: bytes, alloc=None):
        if conn.type in rosmsg.DEFS:
            if isinstance(data, memoryview):  # a view of an arena chunk: payloads stay views of it
                return rosmsg.deserialize(data, conn.type, zero_copy=True)
            return rosmsg.deserialize(data, conn.type, alloc)
        return RawMessage(conn.type, conn.md5sum, data)

    def close(self) -> None:
        if self.mm is not None:
            from ..parallel.host_ring import FileMaps
            FileMaps.unregister(self.mm)
            try:
                self.mm.close()
            except BufferError:  # messages still view the file: the mapping goes with them
                pass
            self.mm = None
        self.f.close()


def is_rosbag(path: str) -> bool:
    with open(path, "rb") as f:
        return f.read(len(MAGIC)) == MAGIC


def read_messages(reader: RosBagReader, topics: Optional[Sequence[str]] = None, alloc=None, readers: int = 0,
                  mapped: bool = False):
    """``alloc``: see :func:`rosmsg.deserialize` (large payloads written into caller buffers);
    ``readers``: threads reading uncompressed chunks ahead into ``alloc`` buffers;
    ``mapped``: payloads stay in the file (:meth:`RosBagReader.mapped_messages`)."""
    if mapped:
        for c, m, t in ((c, m, t) for c, t, m in reader.mapped_messages(topics)):
            yield c.topic, m, t
        return
    for c, t, data in reader.raw_messages(alloc, readers):
        if topics and c.topic not in topics:
            continue
        yield c.topic, reader.decode(c, data, alloc), t
