"""HIP device memory shared between processes on one host (IPC memory handles).

The device side of the KServe shared-memory transport (Triton's
``CudaSharedMemory*`` extension, see ``server/shm.py``): a client allocates a
device buffer with ``hipMalloc``, exports its ``hipIpcMemHandle_t`` (64 bytes)
and registers it with the server, which maps the same memory with
``hipIpcOpenMemHandle``.  Request inputs the client's preprocess kernels wrote
there and the outputs the server's graphs write back never cross PCIe.
Both sides see the memory as a uint8 torch tensor (``__cuda_array_interface__``).

Needs ``HSA_ENABLE_IPC_MODE_LEGACY=0`` on hosts whose driver only offers dmabuf
IPC (exported on the MI355X boxes).
"""
from __future__ import annotations

import ctypes
import threading
from typing import Optional

import torch

HANDLE_BYTES = 64  # HIP_IPC_HANDLE_SIZE
_LAZY_PEER_ACCESS = 1  # hipIpcMemLazyEnablePeerAccess


class _Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * HANDLE_BYTES)]


_HIP: Optional[ctypes.CDLL] = None
_LOCK = threading.Lock()


def _hip() -> ctypes.CDLL:
    global _HIP
    if _HIP is None:
        with _LOCK:
            if _HIP is None:
                lib = None
                for cand in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
                    try:
                        lib = ctypes.CDLL(cand)
                        break
                    except OSError:
                        continue
                if lib is None:
                    raise RuntimeError("libamdhip64.so not found: device shared memory needs the HIP runtime")
                vp, pp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)
                for name, args in (("hipMalloc", [pp, ctypes.c_size_t]), ("hipFree", [vp]),
                                   ("hipIpcGetMemHandle", [ctypes.POINTER(_Handle), vp]),
                                   ("hipIpcOpenMemHandle", [pp, _Handle, ctypes.c_uint]),
                                   ("hipIpcCloseMemHandle", [vp]), ("hipSetDevice", [ctypes.c_int]),
                                   ("hipGetDevice", [ctypes.POINTER(ctypes.c_int)]),
                                   ("hipMemGetAddressRange", [pp, ctypes.POINTER(ctypes.c_size_t), vp]),
                                   ("hipGetErrorString", [ctypes.c_int])):
                    f = getattr(lib, name)
                    f.argtypes = args
                    f.restype = ctypes.c_char_p if name == "hipGetErrorString" else ctypes.c_int
                _HIP = lib
    return _HIP


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {_hip().hipGetErrorString(rc).decode()} ({rc})")


class _CudaArray:
    """``__cuda_array_interface__`` of [nbytes] uint8 at ``ptr`` (torch.as_tensor wraps it, no copy)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def device_tensor(ptr: int, nbytes: int, device) -> torch.Tensor:
    """A uint8 torch tensor over [ptr, ptr + nbytes) of device memory (not owned)."""
    return torch.as_tensor(_CudaArray(ptr, nbytes), device=torch.device(device))


def _device_index(device) -> int:
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


class DeviceAllocation:
    """A dedicated ``hipMalloc`` buffer and its IPC handle (the client side)."""

    def __init__(self, nbytes: int, device="cuda"):
        self.nbytes, self.device_id = int(nbytes), _device_index(device)
        self.device = torch.device("cuda", self.device_id)
        hip = _hip()
        _check(hip.hipSetDevice(self.device_id), "hipSetDevice")
        p = ctypes.c_void_p()
        _check(hip.hipMalloc(ctypes.byref(p), self.nbytes), "hipMalloc")
        self.ptr = int(p.value)
        h = _Handle()
        try:
            _check(hip.hipIpcGetMemHandle(ctypes.byref(h), ctypes.c_void_p(self.ptr)), "hipIpcGetMemHandle")
        except Exception:
            hip.hipFree(ctypes.c_void_p(self.ptr))
            raise
        self.handle = bytes(h)  # all 64 bytes (h.reserved would stop at the first NUL)
        self.tensor = device_tensor(self.ptr, self.nbytes, self.device)

    def close(self) -> None:
        if self.ptr:
            torch.cuda.synchronize(self.device)
            self.tensor = None
            _hip().hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = 0


class OpenedHandle:
    """The server side: another process's allocation mapped into this one.

    The client's declared ``nbytes`` is checked against the size of the
    allocation actually mapped (``hipMemGetAddressRange``), so a region view can
    never reach past it, and the calling thread's current device is restored
    afterwards (a gRPC worker thread must not be left on another GPU)."""

    def __init__(self, raw_handle: bytes, nbytes: int, device_id: int):
        if len(raw_handle) != HANDLE_BYTES:
            raise ValueError(f"raw_handle must be {HANDLE_BYTES} bytes, got {len(raw_handle)}")
        self.nbytes, self.device_id = int(nbytes), int(device_id)
        if self.nbytes <= 0:
            raise ValueError(f"byte_size {self.nbytes}")
        self.device = torch.device("cuda", self.device_id)
        self.ptr = 0
        hip = _hip()
        prev = ctypes.c_int(-1)
        _check(hip.hipGetDevice(ctypes.byref(prev)), "hipGetDevice")
        try:
            _check(hip.hipSetDevice(self.device_id), "hipSetDevice")
            h = _Handle()
            ctypes.memmove(ctypes.addressof(h), raw_handle, HANDLE_BYTES)
            p = ctypes.c_void_p()
            _check(hip.hipIpcOpenMemHandle(ctypes.byref(p), h, _LAZY_PEER_ACCESS), "hipIpcOpenMemHandle")
            self.ptr = int(p.value)
            base, size = ctypes.c_void_p(), ctypes.c_size_t()
            _check(hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(self.ptr)),
                   "hipMemGetAddressRange")
            mapped = int(base.value or 0) + int(size.value) - self.ptr
            if self.nbytes > mapped:
                raise ValueError(f"byte_size {self.nbytes} exceeds the {mapped} bytes the handle maps")
        except Exception:
            if self.ptr:
                hip.hipIpcCloseMemHandle(ctypes.c_void_p(self.ptr))
                self.ptr = 0
            raise
        finally:
            if prev.value >= 0:
                hip.hipSetDevice(prev.value)
        self.tensor = device_tensor(self.ptr, self.nbytes, self.device)

    def close(self) -> None:
        if self.ptr:
            self.tensor = None
            _hip().hipIpcCloseMemHandle(ctypes.c_void_p(self.ptr))
            self.ptr = 0
