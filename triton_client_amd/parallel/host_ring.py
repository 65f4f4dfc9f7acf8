"""The node's shared host ring: how a batch of sensor messages reaches every GPU.

Data-parallel drivers run one process per GPU (``torchrun`` / self-launch).
The ROS subscriber lives in rank 0; instead of copying the node batch to rank
0's GPU and scattering it over xGMI (what the bench's ``--ingest rccl``
measures), rank 0 writes the batch's raw message payloads — JPEG bytes, rgb8
rows, PointCloud2 records — into one slot of a POSIX shared-memory ring, and
every rank pulls *its own shard* straight out of that mapping over its own
PCIe link (the mapping is page-locked in every process, so the H2D is a DMA
from the shared pages).  Each rank decodes its own JPEGs on its own (NUMA-
local) cores.  Annotated frames come back the same way: each rank DMAs them
into the slot's output area.  Only the detections travel over RCCL.

Shared-memory files per ring:

* control ``/dev/shm/<name>_ctl``: a header page, then per slot a 64 KiB
  control block — the slot's ``ready`` sequence word, one ``ack`` word per
  rank (each on its own cache line), a 64-int header and the item table;
* data ``/dev/shm/<name>_d<gen>``: per slot ``slot_bytes`` of payload + output
  area.  When a batch needs more room rank 0 starts a new generation (after
  every slot has drained); the header names the generation and peers attach
  to it on sight.
* ingest arena ``/dev/shm/<name>_in`` (optional, fixed size): rank 0's
  deserialisers write message payloads straight into it (:class:`IngestArena`),
  so the step records offsets there instead of copying payloads into the slot.

Signalling is by 32-bit sequence words with release/acquire ordering and
futex sleep/wake (``csrc/runtime/host_ring.cpp``): rank 0 writes a slot, then
``publish(ready, seq)``; a rank waits for ``ready >= seq``, reads its shard,
writes its outputs and ``publish(ack[rank], seq)``; rank 0 reuses a slot only
after every participant's ack of its previous sequence number.

Reference: none — the reference has no parallelism; this is the
"host ring shared by the sensor process" of SURVEY §5.8 / ``parallel/dp.py``.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import weakref
from typing import Iterable, List, Optional

import numpy as np

from .. import _native

MAGIC = 0x54434152494E4731  # "TCARING1"
CTL_SLOT = 1 << 16
HDR_INTS = 64
ITEM_INTS = 8
ITEMS_OFF = 8192
MAX_ITEMS = (CTL_SLOT - ITEMS_OFF) // (ITEM_INTS * 8)
ACK_OFF, ACK_STRIDE = 64, 64  # bytes: ack word of rank r at ACK_OFF + r * ACK_STRIDE
HDR_OFF = ACK_OFF + 64 * ACK_STRIDE
PATH_OFF = HDR_OFF + HDR_INTS * 8  # the step's source file (sharded replay): <u32 length><utf-8 path>
PATH_MAX = ITEMS_OFF - PATH_OFF - 4


def _rt():
    return _native.runtime()


class RingSpaceError(RuntimeError):
    """/dev/shm cannot hold a ring file (Docker's default /dev/shm is 64 MB)."""


def _reserve(fd: int, path: str, size: int) -> None:
    """Back the whole file with tmpfs pages now: a sparse file that later runs out of
    /dev/shm space would SIGBUS inside the payload copy or a D2H into the mapping."""
    try:
        os.posix_fallocate(fd, 0, size)
    except OSError as e:
        import errno
        if e.errno in (errno.ENOSPC, errno.EFBIG, errno.ENOMEM):
            free = None
            try:
                st = os.statvfs(os.path.dirname(path))
                free = st.f_bavail * st.f_frsize
            except OSError:
                pass
            raise RingSpaceError(
                f"{path}: cannot reserve {size / 2**20:.1f} MiB in {os.path.dirname(path)} "
                f"({'unknown' if free is None else f'{free / 2**20:.1f} MiB'} free); the data-parallel drivers need "
                "about 4 x 1.25 x (one node batch of payloads + annotated frames) -- give the container a larger "
                "/dev/shm (docker run --shm-size=...)") from e
        if e.errno not in (errno.EOPNOTSUPP, errno.EINVAL):  # filesystems without fallocate: stay sparse
            raise
        os.ftruncate(fd, size)


def _open(path: str, size: int, create: bool) -> mmap.mmap:
    flags = os.O_RDWR | (os.O_CREAT | os.O_TRUNC if create else 0)
    fd = os.open(path, flags, 0o600)
    try:
        if create:
            try:
                _reserve(fd, path, size)
            except BaseException:
                os.close(fd)
                fd = -1
                os.unlink(path)
                raise
        elif os.fstat(fd).st_size < size:
            raise RuntimeError(f"{path}: {os.fstat(fd).st_size} bytes, expected {size}")
        return mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    finally:
        if fd >= 0:
            os.close(fd)


def _host_register(mm: mmap.mmap, size: int) -> bool:
    """Page-lock a mapping for DMA in this process (hipHostRegister)."""
    try:
        import torch
        if not torch.cuda.is_available():
            return False
        addr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
        return int(torch.cuda.cudart().cudaHostRegister(addr, size, 0)) == 0
    except Exception:  # noqa: BLE001 - an unpinned ring still works (the copies are staged)
        return False


def _host_unregister(mm: mmap.mmap) -> None:
    try:
        import torch
        torch.cuda.cudart().cudaHostUnregister(ctypes.addressof(ctypes.c_char.from_buffer(mm)))
    except Exception:  # noqa: BLE001
        pass


class DataRing:
    """One generation's payload / output area: ``nslots`` slots of ``slot_bytes``."""

    def __init__(self, path: str, nslots: int, slot_bytes: int, create: bool, pin: bool):
        self.path, self.nslots, self.slot_bytes = path, nslots, slot_bytes
        self.mm = _open(path, nslots * slot_bytes, create)
        self.buf = np.frombuffer(self.mm, np.uint8)
        self.base = self.buf.ctypes.data
        self.pinned = _host_register(self.mm, nslots * slot_bytes) if pin else False

    def slot(self, s: int) -> np.ndarray:
        return self.buf[s * self.slot_bytes:(s + 1) * self.slot_bytes]

    def close(self, unlink: bool = False) -> None:
        if self.pinned:
            _host_unregister(self.mm)
            self.pinned = False
        self.buf = None
        try:
            self.mm.close()
        except BufferError:  # views still published (zero-copy messages): the mapping goes with them
            pass
        if unlink:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class IngestArena:
    """Rank 0's deserialisers write message payloads straight into this area.

    Without it a payload is copied twice in rank 0: the wire / bag record into a
    ``bytes`` object (the deserialiser), then into the ring slot (``_write_step``,
    one process copying the whole node batch: 6.6 GPUs fed with raw rgb8 frames,
    ``profiles/r5/fanout/``).  With it the deserialiser's copy *is* the ring copy:
    ``alloc(n)`` hands out a buffer inside a shared, page-locked mapping that every
    rank attached at start-up, the message's ``data`` views it, and the step only
    records the payload's offset (item ``I_SRC`` = 1) -- rank 0's step copies
    nothing, and the one remaining copy runs in whichever threads deserialise.

    Allocation is a circular first-in-first-out arena: blocks are handed out in
    order and the tail advances over freed blocks, so frees may come out of order
    (a held message keeps only the blocks behind it).  A block is free when every
    view of its array is gone (``weakref.finalize``); rank 0 holds the messages of a
    step until every participant has acked it, so a peer never reads a freed block.
    A full arena returns None and the caller keeps an ordinary ``bytes`` payload
    (the slot-copy path): ingest never blocks on the arena."""

    ALIGN = 256

    def __init__(self, path: str, size: int, create: bool, pin: bool):
        import collections
        import threading

        self.path, self.size = path, int(size)
        self.mm = _open(path, self.size, create)
        self.buf = np.frombuffer(self.mm, np.uint8)
        self.base = self.buf.ctypes.data
        self.pinned = _host_register(self.mm, self.size) if pin else False
        # re-entrant: a block's finalizer can run inside alloc() (cyclic GC on an allocation there)
        self._lock = threading.RLock()
        self._live = collections.deque()  # [offset, bytes, freed] in allocation order
        self._head = 0
        self.stats = {"allocs": 0, "bytes": 0, "full": 0}

    def _fit(self, z: int) -> Optional[int]:
        if not self._live:
            self._head = 0
            return 0 if z <= self.size else None
        tail = self._live[0][0]
        if self._head > tail:  # live blocks are [tail, head): room after head, else wrap to 0
            if self._head + z <= self.size:
                return self._head
            return 0 if z <= tail else None
        return self._head if self._head + z <= tail else None  # wrapped: room up to the tail

    def alloc(self, n: int) -> Optional[np.ndarray]:
        """A writable uint8 array of ``n`` bytes inside the arena, or None when it is full."""
        n = int(n)
        z = max(self.ALIGN, (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN)
        if self.mm is None:
            return None
        with self._lock:
            off = self._fit(z)
            if off is None:
                self.stats["full"] += 1
                return None
            rec = [off, z, False]
            self._live.append(rec)
            self._head = off + z
            self.stats["allocs"] += 1
            self.stats["bytes"] += n
        # a fresh array over the mapping (not a slice of self.buf): numpy collapses view
        # chains to the last ndarray, so slices and memoryviews of *this* array keep it alive
        arr = np.frombuffer(self.mm, np.uint8, n, off)
        weakref.finalize(arr, self._free, rec)
        return arr

    def _free(self, rec) -> None:
        with self._lock:
            rec[2] = True
            while self._live and self._live[0][2]:
                self._live.popleft()

    def offset_of(self, payload, nbytes: int) -> Optional[int]:
        """The arena offset of a payload buffer that lies inside the arena, else None."""
        if self.mm is None or nbytes <= 0:
            return None
        try:
            addr = np.frombuffer(payload, np.uint8, 1).ctypes.data
        except (TypeError, ValueError):
            return None
        off = addr - self.base
        return off if 0 <= off and off + nbytes <= self.size else None

    def in_use(self) -> int:
        with self._lock:
            return sum(r[1] for r in self._live if not r[2])

    def close(self, unlink: bool = False) -> None:
        if self.pinned:
            _host_unregister(self.mm)
            self.pinned = False
        self.buf = None
        try:
            self.mm.close()
            self.mm = None
        except BufferError:  # payload views still alive: the mapping goes with them
            pass
        if unlink:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class FileMaps:
    """Read-only mappings of files whose payload bytes each rank reads for itself.

    Sharded bag replay: rank 0 maps the bag (:meth:`~triton_client_amd.ros.rosbag_v2.RosBagReader.mapping`)
    and publishes messages whose payloads are views of the mapping; the ring step records a
    payload's *file offset* (item ``I_SRC`` = 2) and the file's path instead of copying the
    bytes, and every rank -- rank 0 included -- maps the same file and gathers its own shard's
    payloads from it into its own pinned staging, on its own cores.  Rank 0 never touches a
    payload byte it does not run itself."""

    _lock = __import__("threading").Lock()
    _maps: list = []  # (path, mmap, base address, size); a file may be mapped more than once

    @classmethod
    def register(cls, path: str, mm) -> None:
        base = np.frombuffer(mm, np.uint8).ctypes.data if len(mm) else 0
        with cls._lock:
            cls._maps.append((os.path.abspath(path), mm, base, len(mm)))

    @classmethod
    def unregister(cls, mm) -> None:
        with cls._lock:
            cls._maps[:] = [e for e in cls._maps if e[1] is not mm]

    @classmethod
    def locate(cls, payload, nbytes: int):
        """(path, file offset) of a payload buffer inside a registered mapping, else None."""
        if nbytes <= 0 or not cls._maps:
            return None
        try:
            addr = np.frombuffer(payload, np.uint8, 1).ctypes.data
        except (TypeError, ValueError):
            return None
        with cls._lock:
            for path, _, base, size in cls._maps:
                off = addr - base
                if 0 <= off and off + nbytes <= size:
                    return path, off
        return None

    @classmethod
    def view(cls, path: str) -> np.ndarray:
        """The whole file as a read-only uint8 array (mapped on first use in this process)."""
        path = os.path.abspath(path)
        with cls._lock:
            ent = next((e for e in cls._maps if e[0] == path), None)
        if ent is None:
            with open(path, "rb") as f:
                mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
            try:
                mm.madvise(mmap.MADV_RANDOM)
            except (AttributeError, OSError):
                pass
            cls.register(path, mm)
            ent = (path, mm)
        return np.frombuffer(ent[1], np.uint8)


class HostRing:
    """Control ring + the current data generation (+ the ingest arena, when one was
    asked for).  Rank 0 ``create``s, the other ranks ``attach`` (after a barrier)."""

    def __init__(self, name: str, nslots: int = 4, world: int = 1, create: bool = False, pin: bool = True,
                 arena_bytes: int = 0):
        if not name or "/" in name:
            raise ValueError(f"ring name {name!r}")
        if world > 64:
            raise ValueError("at most 64 ranks share one host ring")
        self.name, self.pin = name, pin
        self.ctl_path = os.path.join("/dev/shm", name + "_ctl")
        size = 4096 + nslots * CTL_SLOT
        self.arena: Optional[IngestArena] = None
        self.arena_path = os.path.join("/dev/shm", name + "_in")
        if create:
            self.mm = _open(self.ctl_path, size, True)
            hdr = np.frombuffer(self.mm, np.int64, 4, 0)
            arena_bytes = (int(arena_bytes) + 4095) // 4096 * 4096
            if arena_bytes > 0:
                try:
                    self.arena = IngestArena(self.arena_path, arena_bytes, True, pin)
                except RingSpaceError as e:  # the ring still works: payloads are copied into the slots
                    import logging
                    logging.getLogger("triton_client_amd.host_ring").warning("no ingest arena: %s", e)
                    arena_bytes = 0
            hdr[:] = (MAGIC, nslots, world, arena_bytes)
        else:
            mm = _open(self.ctl_path, 4096, False)
            magic, nslots, world, arena_bytes = np.frombuffer(mm, np.int64, 4, 0).tolist()
            mm.close()
            if magic != MAGIC:
                raise RuntimeError(f"{self.ctl_path} is not a host ring")
            self.mm = _open(self.ctl_path, 4096 + nslots * CTL_SLOT, False)
            if arena_bytes > 0:
                self.arena = IngestArena(self.arena_path, arena_bytes, False, pin)
        self.nslots, self.world = int(nslots), int(world)
        self.ctl = np.frombuffer(self.mm, np.uint8)
        self.ctl_base = self.ctl.ctypes.data
        self.data: Optional[DataRing] = None
        self.gen = -1
        self.owner = create
        self.generation_switches = {"grow": 0, "leased": 0}  # rank 0: why a new data area was made

    # ------------------------------------------------------------------ layout
    def _blk(self, s: int) -> int:
        return 4096 + s * CTL_SLOT

    def ready_addr(self, s: int) -> int:
        return self.ctl_base + self._blk(s)

    def ack_addr(self, s: int, rank: int) -> int:
        return self.ctl_base + self._blk(s) + ACK_OFF + rank * ACK_STRIDE

    def header(self, s: int) -> np.ndarray:
        return np.frombuffer(self.mm, np.int64, HDR_INTS, self._blk(s) + HDR_OFF)

    def items(self, s: int) -> np.ndarray:
        return np.frombuffer(self.mm, np.int64, MAX_ITEMS * ITEM_INTS, self._blk(s) + ITEMS_OFF).reshape(
            MAX_ITEMS, ITEM_INTS)

    def set_path(self, s: int, path: str) -> None:
        """Rank 0: the file slot s's file-sourced items (``I_SRC`` = 2) are read from."""
        b = path.encode()
        if len(b) > PATH_MAX:
            raise ValueError(f"source path longer than {PATH_MAX} bytes")
        o = self._blk(s) + PATH_OFF
        self.ctl[o:o + 4] = np.frombuffer(np.uint32(len(b)).tobytes(), np.uint8)
        self.ctl[o + 4:o + 4 + len(b)] = np.frombuffer(b, np.uint8)

    def path(self, s: int) -> str:
        o = self._blk(s) + PATH_OFF
        n = int(np.frombuffer(self.mm, np.uint32, 1, o)[0])
        return bytes(self.ctl[o + 4:o + 4 + min(n, PATH_MAX)]).decode()

    # ------------------------------------------------------------------ data generations
    def data_path(self, gen: int) -> str:
        return os.path.join("/dev/shm", f"{self.name}_d{gen}")

    def new_generation(self, slot_bytes: int) -> DataRing:
        """Rank 0: a (larger) data area; the caller has drained every slot."""
        old = self.data
        slot_bytes = (int(slot_bytes) + 4095) // 4096 * 4096
        self.data = DataRing(self.data_path(self.gen + 1), self.nslots, slot_bytes, True, self.pin)
        self.gen += 1  # only once the new area exists: a failed reservation keeps the old one in use
        if old is not None:
            old.close(unlink=True)
        return self.data

    def use_generation(self, gen: int, slot_bytes: int) -> DataRing:
        """Peers: attach the generation a header names."""
        if gen != self.gen:
            if self.data is not None:
                self.data.close()
            self.data = DataRing(self.data_path(gen), self.nslots, slot_bytes, False, self.pin)
            self.gen = gen
        return self.data

    # ------------------------------------------------------------------ signalling
    def publish(self, s: int, seq: int) -> None:
        _rt().tca_ring_publish(self.ready_addr(s), seq & 0xFFFFFFFF)

    def wait_ready(self, s: int, seq: int, timeout_ms: int = -1) -> bool:
        return _rt().tca_ring_wait(self.ready_addr(s), seq & 0xFFFFFFFF, timeout_ms) == 0

    def ack(self, s: int, rank: int, seq: int) -> None:
        _rt().tca_ring_publish(self.ack_addr(s, rank), seq & 0xFFFFFFFF)

    def wait_acks(self, s: int, ranks: Iterable[int], seq: int, timeout_ms: int = -1) -> List[int]:
        """Ranks (of ``ranks``) that had not acked ``seq`` when the wait ended."""
        mask = 0
        for r in ranks:
            mask |= 1 << r
        if not mask:
            return []
        missing = ctypes.c_uint64(0)
        rc = _rt().tca_ring_wait_all(self.ack_addr(s, 0), ACK_STRIDE // 4, mask, seq & 0xFFFFFFFF, timeout_ms,
                                     ctypes.byref(missing))
        if rc < 0:
            raise RuntimeError("tca_ring_wait_all: bad arguments")
        return [r for r in range(64) if (missing.value >> r) & 1]

    def close(self) -> None:
        if self.data is not None:
            self.data.close(unlink=self.owner)
            self.data = None
        if self.arena is not None:
            self.arena.close(unlink=self.owner)
            self.arena = None
        try:
            self.mm.close()
        except BufferError:
            pass
        if self.owner:
            try:
                os.unlink(self.ctl_path)
            except FileNotFoundError:
                pass
