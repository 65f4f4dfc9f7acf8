"""KServe-v2 system shared-memory extension (Triton's ``SystemSharedMemory*``
RPCs and the ``shared_memory_region`` / ``shared_memory_offset`` /
``shared_memory_byte_size`` tensor parameters), and its device twin (Triton's
``CudaSharedMemory*`` RPCs): a client's GPU allocation, shared by a HIP IPC
memory handle, that the request's inputs are read from and its outputs
written into on the device (``utils/hip_ipc.py``).

A client on the same host registers a POSIX shared-memory object
(``/dev/shm/<key>``) as a named region; an inference request then names a
region slice for an input instead of carrying the tensor bytes, and may name a
slice for an output, which the server writes instead of putting the bytes in
the response.  The gRPC messages shrink to a few hundred bytes: for the
reference's YOLOv5 contract (FP32 [3, 640, 640] in, FP32 [1, 25200, 85] out,
``examples/YOLOv5/config.pbtxt``) that is 13.5 MB per frame that no longer
crosses the gRPC stack.  Mapped regions are also page-locked for the GPU when
a device is present (``hipHostRegister``), so the served models' H2D copies
read them directly.
"""
from __future__ import annotations

import mmap
import os
import threading
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

from .model import InferError

SHM_DIR = "/dev/shm"

# page-locked registered mappings, base address -> bytes: a request view inside one
# is DMA'd to the GPU straight from the client's memory (no staging copy)
_PINNED: Dict[int, int] = {}
_PINNED_LOCK = threading.Lock()


def _base(mm: mmap.mmap) -> int:
    import ctypes
    return ctypes.addressof(ctypes.c_char.from_buffer(mm))


def pinned_host(a: np.ndarray) -> bool:
    """True when ``a`` lies entirely inside a page-locked registered region."""
    if not isinstance(a, np.ndarray) or not a.flags.c_contiguous:
        return False
    p, n = a.ctypes.data, a.nbytes
    with _PINNED_LOCK:
        return any(b <= p and p + n <= b + sz for b, sz in _PINNED.items())


@dataclass
class Region:
    name: str
    key: str
    offset: int
    byte_size: int
    mm: Optional[mmap.mmap]
    pinned: bool = False
    dev: Optional[object] = None  # device region: utils.hip_ipc.OpenedHandle
    device_id: int = 0
    _views: Optional[dict] = None
    # device regions: requests holding a lease (their batch may still read / write the
    # mapping); an unregister while any is held defers the close to the last release
    inflight: int = 0
    closing: bool = False

    @property
    def device(self) -> bool:
        return self.dev is not None

    def view(self, offset: int, nbytes: int, dtype, shape):
        """ndarray view of a system region; for a device region a torch tensor on its GPU."""
        if offset < 0 or nbytes < 0 or offset + nbytes > self.byte_size:
            raise InferError(f"shared memory region '{self.name}': [{offset}, {offset + nbytes}) outside "
                             f"its {self.byte_size} bytes")
        dt = np.dtype(dtype)
        count = nbytes // dt.itemsize
        if self.dev is not None:  # cached: clients reuse a few slots, and torch views cost a dispatch each
            key = (offset, nbytes, dt.str, tuple(shape))
            v = self._views.get(key) if self._views is not None else None
            if v is None:
                import torch
                tdt = torch.from_numpy(np.empty(0, dt)).dtype
                v = self.dev.tensor[offset:offset + count * dt.itemsize].view(tdt).reshape(shape)
                if self._views is None:
                    self._views = {}
                if len(self._views) < 4096:
                    self._views[key] = v
            return v
        a = np.frombuffer(self.mm, dtype=dt, count=count, offset=self.offset + offset)
        return a.reshape(shape)


def shm_path(key: str) -> str:
    k = key.lstrip("/")
    if not k or "/" in k:
        raise InferError(f"invalid shared memory key '{key}'")
    return os.path.join(SHM_DIR, k)


def _host_register(mm: mmap.mmap, size: int) -> bool:
    """Page-lock the mapping for DMA (torch's hipHostRegister binding); best effort."""
    try:
        import ctypes

        import torch
        if not torch.cuda.is_available():
            return False
        addr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
        return int(torch.cuda.cudart().cudaHostRegister(addr, size, 0)) == 0
    except Exception:  # noqa: BLE001 - an unpinned region still works (staged copies)
        return False


def _host_unregister(mm: mmap.mmap) -> None:
    try:
        import ctypes

        import torch
        torch.cuda.cudart().cudaHostUnregister(ctypes.addressof(ctypes.c_char.from_buffer(mm)))
    except Exception:  # noqa: BLE001
        pass


class SharedMemoryRegistry:
    """``device_id``: the GPU the served models run on (device regions on another
    GPU are refused: the server's copy kernels read them as same-device memory)."""

    def __init__(self, pin: bool = True, device_id: Optional[int] = None):
        self._regions: Dict[str, Region] = {}
        self._lock = threading.Lock()
        self.pin = pin
        self.device_id = device_id

    def register(self, name: str, key: str, offset: int, byte_size: int) -> Region:
        if not name:
            raise InferError("shared memory region needs a name")
        with self._lock:
            if name in self._regions:
                raise InferError(f"shared memory region '{name}' already registered")
        path = shm_path(key)
        try:
            fd = os.open(path, os.O_RDWR)
        except OSError as e:
            raise InferError(f"unable to open shared memory key '{key}': {e}") from e
        try:
            size = os.fstat(fd).st_size
            if byte_size <= 0 or offset < 0 or offset + byte_size > size:
                raise InferError(f"shared memory key '{key}' has {size} bytes; [{offset}, {offset + byte_size}) "
                                 f"requested")
            mm = mmap.mmap(fd, offset + byte_size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        r = Region(name, key, int(offset), int(byte_size), mm)
        if self.pin:
            r.pinned = _host_register(mm, offset + byte_size)
            if r.pinned:
                with _PINNED_LOCK:
                    _PINNED[_base(mm)] = offset + byte_size
        with self._lock:
            self._regions[name] = r
        return r

    def register_device(self, name: str, raw_handle: bytes, device_id: int, byte_size: int) -> Region:
        """Map a client's device allocation (HIP IPC handle, Triton's CudaSharedMemoryRegister)."""
        if not name:
            raise InferError("shared memory region needs a name")
        with self._lock:
            if name in self._regions:
                raise InferError(f"shared memory region '{name}' already registered")
        if byte_size <= 0:
            raise InferError(f"device shared memory region '{name}': byte_size {byte_size}")
        if self.device_id is not None and int(device_id) != self.device_id:
            raise InferError(f"device shared memory region '{name}' is on device {device_id}; this server's models "
                             f"run on device {self.device_id}")
        try:
            from ..utils.hip_ipc import OpenedHandle
            h = OpenedHandle(raw_handle, byte_size, device_id)
        except Exception as e:  # noqa: BLE001 - a bad handle / no GPU is the client's error
            raise InferError(f"unable to open device shared memory handle for '{name}': {e}") from e
        r = Region(name, "", 0, int(byte_size), None, dev=h, device_id=int(device_id))
        with self._lock:
            if name in self._regions:
                h.close()
                raise InferError(f"shared memory region '{name}' already registered")
            self._regions[name] = r
        return r

    def lease(self, names) -> list:
        """Hold the device regions a request references until :meth:`release`:
        an unregister meanwhile removes the name but leaves the mapping open
        for this request's batch (closed by the last release)."""
        regs = []
        with self._lock:
            for n in set(names):
                r = self._regions.get(n)
                if r is None:
                    raise InferError(f"unable to find shared memory region '{n}'")
                if r.dev is not None:
                    regs.append(r)
            for r in regs:
                r.inflight += 1
        return regs

    def release(self, regs) -> None:
        done = []
        with self._lock:
            for r in regs:
                r.inflight -= 1
                if r.inflight == 0 and r.closing:
                    done.append(r)
        if done:
            self._close(done)

    def unregister(self, name: str = "", device: Optional[bool] = None) -> None:
        """Unregister ``name`` (or every region of the kind: device True / system False / both None).
        A device region a queued or running request still holds (:meth:`lease`) is
        closed when that request releases it."""
        with self._lock:
            names = [name] if name else [n for n, r in self._regions.items() if device is None or r.device == device]
            regs = [self._regions.pop(n) for n in names if n in self._regions]
            for r in regs:
                if r.dev is not None and r.inflight > 0:
                    r.closing = True
            regs = [r for r in regs if not r.closing]
        if regs:
            self._close(regs)

    def _close(self, regs) -> None:
        from .model import GPU_PHASE

        # An execution that chose the direct (pinned) path for a view of this region
        # may still be DMA'ing from it: unpin only when no execution is in flight.
        # Executions hold GPU_PHASE shared; one that starts after this block finds
        # the region gone from _PINNED and stages its copy instead.
        GPU_PHASE.acquire_exclusive()
        try:
            for r in regs:
                if r.dev is not None:
                    import torch
                    torch.cuda.synchronize(r.dev.device)  # no copy from / into it still queued
                    r._views = None
                    r.dev.close()
                if r.pinned:
                    with _PINNED_LOCK:
                        _PINNED.pop(_base(r.mm), None)
                    _host_unregister(r.mm)
                    r.pinned = False
        finally:
            GPU_PHASE.release_exclusive()
        for r in regs:
            if r.mm is None:
                continue
            try:
                r.mm.close()
            except BufferError:  # a response still references it: the mapping goes with the last view
                pass

    def get(self, name: str) -> Region:
        with self._lock:
            r = self._regions.get(name)
        if r is None:
            raise InferError(f"unable to find shared memory region '{name}'")
        return r

    def status(self, name: str = "", device: bool = False):
        with self._lock:
            if name and (name not in self._regions or self._regions[name].device != device):
                raise InferError(f"unable to find shared memory region '{name}'")
            return [r for n, r in self._regions.items() if (not name or n == name) and r.device == device]


def tensor_shm(params) -> Optional[tuple]:
    """(region, offset, byte_size) from a tensor's parameters map, or None."""
    if "shared_memory_region" not in params:
        return None
    region = params["shared_memory_region"].string_param
    nbytes = int(params["shared_memory_byte_size"].int64_param) if "shared_memory_byte_size" in params else -1
    off = int(params["shared_memory_offset"].int64_param) if "shared_memory_offset" in params else 0
    if nbytes < 0:
        raise InferError("shared_memory_byte_size is required with shared_memory_region")
    return region, off, nbytes
