"""roctx ranges / markers.

Named host-side ranges around every per-frame stage (decode, preprocess,
RPC, graph replay, postprocess, publish) show up on the rocprofv3 timeline
next to the kernels when the run is traced with ``--marker-trace``:

    rocprofv3 --marker-trace --kernel-trace -d out -o run -- python bag2d.py ...

The library (``librocprofiler-sdk-roctx``, falling back to the legacy
``libroctx64``) is loaded lazily with ctypes.  Without it, or with
``TCA_ROCTX=0``, every call is a no-op costing one attribute lookup.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")
_state = {"lib": None, "tried": False}
_lock = threading.Lock()


def _lib():
    if _state["tried"]:
        return _state["lib"]
    with _lock:
        if not _state["tried"]:
            _state["tried"] = True
            if os.environ.get("TCA_ROCTX", "1") != "0":
                for name in _LIBS:
                    for path in (os.path.join("/opt/rocm/lib", name), name):
                        try:
                            lib = ctypes.CDLL(path)
                        except OSError:
                            continue
                        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                        lib.roctxRangePushA.restype = ctypes.c_int
                        lib.roctxRangePop.restype = ctypes.c_int
                        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                        _state["lib"] = lib
                        break
                    if _state["lib"] is not None:
                        break
    return _state["lib"]


def available() -> bool:
    return _lib() is not None


def push(name: str) -> int:
    lib = _lib()
    return lib.roctxRangePushA(name.encode()) if lib is not None else -1


def pop() -> int:
    lib = _lib()
    return lib.roctxRangePop() if lib is not None else -1


def mark(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def trace_range(name: str):
    push(name)
    try:
        yield
    finally:
        pop()
