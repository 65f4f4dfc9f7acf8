"""Client side of the KServe-v2 system shared-memory extension (the role of
``tritonclient.utils.shared_memory``): a POSIX shared-memory object under
/dev/shm that the client writes request tensors into and the server writes
responses into; requests carry only region references (server side:
``server/shm.py``).  On a GPU client the mapping is page-locked so the
preprocess kernel's D2H lands in it directly."""
from __future__ import annotations

import mmap
import os
import uuid
import weakref
from typing import Optional

import numpy as np

from ..server.shm import SHM_DIR, _host_register, _host_unregister


class DeviceShmRegion:
    """Client side of the device shared-memory transport: a dedicated GPU allocation
    whose HIP IPC handle the server maps (``register`` → Triton's
    CudaSharedMemoryRegister).  ``view`` returns torch tensors on the GPU; the
    preprocess writes the request inputs there and the server writes the outputs
    back there, device to device."""

    def __init__(self, byte_size: int, device="cuda", key: Optional[str] = None):
        from ..utils.hip_ipc import DeviceAllocation
        self.key = key or f"tca_dev_{os.getpid()}_{uuid.uuid4().hex[:12]}"
        self.byte_size = int(byte_size)
        self.alloc = DeviceAllocation(self.byte_size, device)
        self.device = self.alloc.device

    def register(self, channel) -> None:
        channel.register_cuda_shared_memory(self.key, self.alloc.handle, self.alloc.device_id, self.byte_size)

    def unregister(self, channel) -> None:
        channel.unregister_cuda_shared_memory(self.key)

    def view(self, offset: int, dtype, shape):
        import torch
        dt = np.dtype(dtype)
        n = int(np.prod(shape))
        if offset < 0 or offset + n * dt.itemsize > self.byte_size:
            raise ValueError(f"[{offset}, {offset + n * dt.itemsize}) outside the {self.byte_size}-byte region")
        tdt = torch.from_numpy(np.empty(0, dt)).dtype
        return self.alloc.tensor[offset:offset + n * dt.itemsize].view(tdt).reshape(shape)

    def close(self, unlink: bool = True) -> None:
        self.alloc.close()


def _unlink_quiet(path: str) -> None:
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass


class ShmRegion:
    def register(self, channel) -> None:
        channel.register_system_shared_memory(self.key, self.key, self.byte_size)

    def unregister(self, channel) -> None:
        channel.unregister_system_shared_memory(self.key)

    def __init__(self, byte_size: int, key: Optional[str] = None, pin: bool = True):
        self.key = key or f"tca_{os.getpid()}_{uuid.uuid4().hex[:12]}"
        self.byte_size = int(byte_size)
        self.path = os.path.join(SHM_DIR, self.key)
        fd = os.open(self.path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
        try:
            os.ftruncate(fd, self.byte_size)
            self.mm = mmap.mmap(fd, self.byte_size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.pinned = _host_register(self.mm, self.byte_size) if pin else False
        # a region nobody closed still leaves no file behind in /dev/shm (at GC or interpreter exit)
        self._unlink = weakref.finalize(self, _unlink_quiet, self.path)

    def view(self, offset: int, dtype, shape) -> np.ndarray:
        dt = np.dtype(dtype)
        n = int(np.prod(shape))
        if offset < 0 or offset + n * dt.itemsize > self.byte_size:
            raise ValueError(f"[{offset}, {offset + n * dt.itemsize}) outside the {self.byte_size}-byte region")
        return np.frombuffer(self.mm, dtype=dt, count=n, offset=offset).reshape(shape)

    def close(self, unlink: bool = True) -> None:
        if self.mm is None:
            return
        if self.pinned:
            _host_unregister(self.mm)
        try:
            self.mm.close()
        except BufferError:  # live views keep the mapping; the file is still unlinked below
            pass
        self.mm = None
        if unlink:
            self._unlink()
        else:
            self._unlink.detach()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def shm_params(t, region: str, offset: int, nbytes: int) -> None:
    """Set the extension's parameters on a request input / requested output."""
    t.parameters["shared_memory_region"].string_param = region
    t.parameters["shared_memory_byte_size"].int64_param = int(nbytes)
    if offset:
        t.parameters["shared_memory_offset"].int64_param = int(offset)
