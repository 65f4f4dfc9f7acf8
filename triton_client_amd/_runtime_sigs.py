"""argtypes for libtca_runtime.so."""
import ctypes

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
CP = ctypes.c_char_p
PP = ctypes.POINTER(ctypes.c_char_p)

SIGS = {
    "tca_kserve_request_size": (L, [CP, CP, CP, I, PP, PP, P, P, P, I, PP]),
    "tca_kserve_encode_request": (L, [CP, CP, CP, I, PP, PP, P, P, P, P, I, PP, P, L]),
    "tca_kserve_parse_response": (I, [P, L, I, P, P, I, P, P]),
}


def declare(lib: ctypes.CDLL) -> None:
    for name, (res, args) in SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
