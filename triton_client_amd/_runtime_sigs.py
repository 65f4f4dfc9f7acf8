"""argtypes for libtca_runtime.so (filled in as runtime components land)."""
import ctypes

SIGS = {}


def declare(lib: ctypes.CDLL) -> None:
    for name, (res, args) in SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
