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
    "tca_kserve_response_size": (L, [CP, CP, CP, I, PP, PP, P, P, P]),
    "tca_kserve_encode_response": (L, [CP, CP, CP, I, PP, PP, P, P, P, P, P, L]),
    "tca_kserve_parse_request": (I, [P, L, I, P, P, I, P, P, P]),
    # baseline JPEG entropy decoder (csrc/runtime/jpeg_entropy.cpp)
    "tca_jpeg_probe": (I, [P, ctypes.c_int64, P]),
    "tca_jpeg_decode_coefs": (I, [P, ctypes.c_int64, P, ctypes.c_int64, P, P]),
    "tca_jpeg_decode_batch": (I, [P, P, I, P, ctypes.c_int64, P, P, P, I]),
    # batched host payload copies into pinned staging (csrc/runtime/host_copy.cpp)
    "tca_host_gather_copy": (I, [I, P, P, P, I]),
    # ROS1 wire parse of sensor messages / bag chunk record scan (csrc/runtime/ros_wire.cpp)
    "tca_ros_parse": (I, [I, I, P, P, P]),
    "tca_bag_scan": (ctypes.c_int64, [P, ctypes.c_int64, ctypes.c_int64, P, P, P, P, P, P, P, P]),
    "tca_bag_index": (ctypes.c_int64, [P, ctypes.c_int64, P, ctypes.c_int64, P, P, P, P, P, P, P, P]),
    # node host ring signalling (csrc/runtime/host_ring.cpp)
    "tca_ring_publish": (I, [P, ctypes.c_uint32]),
    "tca_ring_load": (ctypes.c_uint32, [P]),
    "tca_ring_wait": (I, [P, ctypes.c_uint32, ctypes.c_int64]),
    "tca_ring_wait_all": (I, [P, I, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64,
                              ctypes.POINTER(ctypes.c_uint64)]),
    # host preprocess for GPU-less hosts (csrc/runtime/cpu_image.cpp)
    "tca_cpu_preprocess": (I, [P, I, I, I, I, P, I, I, I, I, I, I, I, ctypes.c_float, I, P, P, I]),
    # native RCCL communicator (csrc/runtime/rccl_comm.cpp)
    "tca_rccl_unique_id_bytes": (I, []),
    "tca_rccl_get_unique_id": (I, [P]),
    "tca_rccl_comm_init": (I, [ctypes.POINTER(P), I, P, I]),
    "tca_rccl_comm_destroy": (I, [P]),
    "tca_rccl_comm_abort": (I, [P]),
    "tca_rccl_async_error": (I, [P]),
    "tca_rccl_error_string": (CP, [I]),
    "tca_rccl_comm_count": (I, [P, ctypes.POINTER(I)]),
    "tca_rccl_group_p2p": (I, [P, I, P, P, P, P, P]),
    "tca_rccl_allreduce_max_f64": (I, [P, P, ctypes.c_int64, P]),
    "tca_rccl_broadcast": (I, [P, P, ctypes.c_int64, I, P]),
}


def declare(lib: ctypes.CDLL) -> None:
    for name, (res, args) in SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
