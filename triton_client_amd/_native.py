"""ctypes bindings to the in-tree native libraries.

Every op in ``triton_client_amd.ops`` dispatches on the tensor's device:
GPU tensors go to the HIP kernels here — never silently to a PyTorch
fallback; if the library is missing on a machine with a GPU the call raises
(the CPU path exists only for CPU tensors, i.e. config 1 "CPU-only" runs and
the GPU-less CI host).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

from . import _build

_LOCK = threading.Lock()
_KERNELS: Optional[ctypes.CDLL] = None
_RUNTIME: Optional[ctypes.CDLL] = None
_HIP: Optional[ctypes.CDLL] = None

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float

# name -> argtypes (restype is always int = hipError_t)
_KERNEL_SIGS = {
    "tca_draw_boxes": [P, L, I, I, I, I, P, I, I, P, P, I, P],
    "tca_draw_annotations": [P, L, I, I, I, I, P, I, I, P, P, P, I, P, I, P],
    # JPEG pixel reconstruction (csrc/kernels/jpeg.hip)
    "tca_jpeg_idct": [P, P, P, P, L, L, I, P],
    "tca_jpeg_color": [P, P, P, L, L, I, P],
    "tca_image_preprocess": [P, L, I, I, I, I, I, P, I, I, I, I, I, I, I, I, I, I, F, I, F, F, F, F, F, F, P],
    # src, batch stride, src_h, src_w, row stride, src_c, swap_rb, dst_h, dst_w, B, top, left, reg_h, reg_w, pad,
    # quantize, sc0-2, b0-2, w0, bias0, act0, w1, bias1, act1, out, ldo, co_off, stream
    # ptrs[14], ints[24], stream (csrc/kernels/c3_fused.hip)
    "tca_c3_fused": [P, P, P],
    "tca_yolo_stem_fused": [P, L, I, I, I, I, I, I, I, I, I, I, I, I, F, I, F, F, F, F, F, F, P, P, I, P, P, I, P, I,
                            I, P],
    # x[3], ldx[3], x_off[3], cin[3], hw[6], w[3], bias[3], strides[3], anchors, B, na, nc, conf, class_mask,
    # cand box, score, cls, key, count, cap, stream
    "tca_yolo_detect_filter": [P, P, P, P, P, P, P, P, P, I, I, I, F, P, P, P, P, P, P, I, P],
    "tca_yolo_decode": [P, P, P, I, I, I, I, I, P, P, P, P, P, P],
    "tca_yolo_decode_filter": [P, P, P, I, I, I, I, I, P, P, P, P, F, I, P, P, P, P, P, P, I, P, P],
    # pred, confs, kind, B, N, ld, nc, conf, multi_label, class_mask, img_w, img_h, cand box/score/cls/key/count,
    # cap, stream (the remote client's postprocess of a decoded response, csrc/kernels/yolo.hip)
    "tca_yolo_filter_decoded": [P, P, I, I, I, I, I, F, I, P, F, F, P, P, P, P, P, I, P],
    "tca_topk_sort": [P, P, I, I, I, P, P, P],
    "tca_nms_mask": [I, P, I, P, P, P, I, I, I, F, I, P, I, P],
    "tca_nms_mask_rot": [P, I, P, P, P, I, I, I, F, I, P, P, P],
    "tca_nms_reduce": [P, P, P, I, I, P, I, P, P, I, I, P, P, P, P, P, P],
    "tca_box_iou": [P, I, P, I, P, P],
    "tca_nms_merge": [P, P, P, P, P, P, P, P, I, I, I, F, I, I, P, P, P, P, P, P],
    "tca_pc2_unpack": [P, P, P, I, I, I, P, P, I, F, P, I, P, P, P, P],
    "tca_pc2_blocks_per_frame": [I],
    "tca_vox_blocks_per_frame": [I],
    "tca_voxelize": [P, I, I, P, I, P, P, P, I, I, I, P, P, P, P, P, P, P, P, P, P, I, I, P, I, P],
    "tca_pillar_vfe_slots": [P, I, I, P, P, P, P, I, I, I, P, P, P, P, I, I, P, P, I, P],
    "tca_pillar_vfe_set_variant": [I],
    "tca_conv_s2sp": [P, I, I, I, I, I, I, P, P, I, P, I, I, I, P, I, P],  # returns the previous variant (not an error code)
    "tca_pillar_vfe_voxels": [P, P, P, P, I, I, I, P, P, P, P, I, I, P, P, I, P],
    "tca_pillar_canvas_clear": [P, P, I, I, I, I, I, P, I, P],
    "tca_pillar_vfe_slots_occ": [P, I, I, P, P, P, P, I, I, I, P, P, P, P, I, I, P, P, I, P, P],
    "tca_pillar_vfe_voxels_occ": [P, P, P, P, I, I, I, P, P, P, P, I, I, P, P, I, P, P],
    "tca_pillar_canvas_clear_occ": [P, P, I, I, I, I, I, P, I, P, P],
    "tca_pillar_occ_clear": [P, P, I, I, I, I, P, P],
    "tca_conv_nhwc": [P, I, I, I, I, I, I, P, P, I, I, I, I, I, I, P, I, I, I, I, I, P, I, I, I, I, P],
    "tca_conv_nhwc_x3": [P, I, I, I, I, I, I, P, P, I, I, I, I, I, I, P, I, I, I, I, I, P, I, I, I, I, P],
    "tca_conv_nhwc_x3p": [P, I, I, I, I, I, I, P, P, I, I, I, I, I, I, P, I, I, I, I, I, P, I, I, I, I, I, P],
    # in, B, H, W, Cin, ldi, ci_off, wfrag, bias, N, out, ldo, co_off, act, res, ldr, r_off, tile, stream
    "tca_conv_wino": [P, I, I, I, I, I, I, I, P, P, I, P, I, I, I, I, P, I, P, I, P],
    "tca_conv_hx3p": [P, I, I, I, I, I, I, P, P, I, P, I, I, I, P, I, I, I, P],
    # in, B, H, W, Cin, ldi, ci_off, wfrag, bias, N, out, ldo, co_off, act, uni, uni_min, uni_val, tile, stream
    "tca_conv_hx3p_uni": [P, I, I, I, I, I, I, P, P, I, P, I, I, I, P, I, P, I, P],
    # occ, B, H, W, maxd, depth, stream
    "tca_bev_uniform_depth": [P, I, I, I, I, P, P],
    # in, B, H, W, Cin, ldi, ci_off, wfrag, bias, N, out, ldo, co_off, act, res, ldr, r_off, occ, tile, stream
    "tca_conv_hx3s2p": [P, I, I, I, I, I, I, P, P, I, P, I, I, I, P, I, I, P, P, I, P, I, P],
    # n, dst[], src[], nbytes[], stream (csrc/kernels/copy.hip)
    "tca_copy_segments": [I, P, P, P, P],
    # coords, nump, vcount, B, V, P, nz, ny, nx, flags, stream
    "tca_voxel_check": [P, P, P, I, I, I, I, I, I, P, P],
    # cur, cs, cur_n, B, maxp, R, ring, ring_n, ring_t, ring_pose, head, clock, pose, dt, out, out_n, stream
    "tca_sweep_step": [P, I, P, I, I, I, P, P, P, P, P, P, P, ctypes.c_double, P, P, P],
    # src, B, H, W, dst, dst_dtype, dst_layout, sc0, sc1, sc2, b0, b1, b2, stream
    "tca_planar_affine": [P, I, I, I, P, I, I, F, F, F, F, F, F, P],
    "tca_conv_nhwc_x3p_occ": [P, I, I, I, I, I, I, P, P, I, I, I, I, I, I, P, I, I, I, I, I, P, I, I, I, I, I, P, P],
    "tca_zero_i32": [P, I, P],
    "tca_anchor_decode_filter": [P, P, P, I, I, I, I, I, I, I, I, I, I, I, P, F, F, F, F, F, F, F, P, P, P, P, P, I, P],
    "tca_anchor_decode_filter_keyed": [P, P, P, I, I, I, I, I, I, I, I, I, I, I, P, F, F, F, F, F, F, P, P, P, P, P, P, I,
                                       P],
    "tca_anchor_topk_threshold": [P, I, I, I, I, I, I, I, I, I, P, P, P],
    "tca_pfn2_slots": [P, I, I, P, P, P, P, I, I, I, P, P, P, P, P, P, I, I, P, P, I, P],
    "tca_pfn2_voxels": [P, I, P, P, P, I, I, I, P, P, P, P, P, P, I, I, P, P, I, P],
    "tca_centerhead_decode": [P, I, I, I, I, I, I, P, P, I, F, P, P, I, P, P, P, P, P, P, I, P],
    "tca_maxpool2d_nhwc": [P, I, I, I, I, I, I, I, I, I, P, I, I, I, I, I, P],
    "tca_retina_decode": [P, P, I, I, I, I, I, I, I, I, I, P, F, F, F, F, I, I, P, P, P, P, P, I, I, P],
    "tca_fcos_decode": [P, P, P, I, I, I, I, I, I, I, I, I, F, F, F, I, I, P, P, P, P, P, I, I, P],
    "tca_segment_merge": [P, P, P, P, I, I, P, P, I, I, I, P, P, P, P, P, I, P],
    "tca_group_norm_nhwc": [P, I, I, I, I, I, I, F, P, P, I, P, P, I, I, P],
    "tca_group_norm_nhwc_dt": [P, I, I, I, I, I, I, F, P, P, I, P, P, I, I, I, P],
    "tca_yolov4_decode": [P, P, P, I, I, I, P, P, P, F, F, I, I, P, P, P, P, P, P, P, I, P],
    # in, B, H, W, C, ldi, ci_off, k, out, ldo, o1, o2, o3, dtype, stream
    "tca_sppf_pool3": [P, I, I, I, I, I, I, I, P, I, I, I, I, I, P],
    "tca_maxpool_nhwc": [P, I, I, I, I, I, I, I, P, I, I, I, P],
    "tca_upsample2x_nhwc": [P, I, I, I, I, I, I, P, I, I, I, P],
    "tca_vox_slots_csr": [P, I, P, I, P, P, I, I, P, P, P, P, P, P, P, P, I, P],
    "tca_bev_neck_head": [I, P, P, P, P, P, P, P, P, P, I, P, I, I, I, I, I, P],
    "tca_bev_neck_head_x3": [I, P, P, P, P, P, P, P, P, P, I, P, I, I, I, I, I, P],
    "tca_bev_neck_head_x3p": [I, P, P, P, P, P, P, P, P, P, I, P, I, I, I, I, I, P],
    "tca_bev_neck_head_x3v": [I, P, P, P, P, P, P, P, P, P, I, P, I, I, I, I, I, I, I, P],
    # SECOND-IoU: sparse 3D backbone + RoI head (spconv.hip)
    "tca_sp_offsets": [P, I, P, P, P],
    "tca_sp_vfe_slots": [P, I, I, P, P, I, P, P, I, I, P, P, P, P, P, P],
    "tca_sp_vfe_voxels": [P, I, I, I, P, P, P, P, P, P, P, P],
    "tca_sp_claim": [P, P, I, P, P, P, P, P, I, P],
    "tca_sp_rulebook": [P, P, I, P, P, P, P, P, P],
    "tca_sp_grid_reset": [P, P, I, P, P, P],
    "tca_sp_bev_clear": [P, P, I, I, P, I, I, I, P],
    "tca_sp_gemm": [P, I, P, I, P, P, P, I, I, P, I, P, P, P, I, I, I, I, P],
    "tca_sp_vfe_slots_f32": [P, I, I, P, P, I, P, P, I, I, P, P, P, P, P, P],
    "tca_sp_vfe_voxels_f32": [P, I, I, I, P, P, P, P, P, P, P, P],
    "tca_sp_bev_clear_f32": [P, P, I, I, P, I, I, I, P],
    "tca_roi_grid_pool_f32": [P, I, I, I, I, I, I, P, I, P, I, F, F, F, F, I, P, P],
    "tca_sp_gemm_x3": [P, I, P, I, P, P, P, I, I, P, I, P, P, P, I, I, I, I, P],
    "tca_roi_grid_pool": [P, I, I, I, I, I, I, P, I, P, I, F, F, F, F, I, P, P],
    "tca_roi_rescore": [P, P, I, P, P, I, I, F, P, P, P, P, P, P],
}


class NativeError(RuntimeError):
    pass


def _load_hip() -> ctypes.CDLL:
    global _HIP
    if _HIP is None:
        with _LOCK:
            if _HIP is not None:
                return _HIP
            lib = None
            for cand in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
                try:
                    lib = ctypes.CDLL(cand)
                    break
                except OSError:
                    continue
            if lib is not None:
                lib.hipGetErrorString.restype = ctypes.c_char_p
                lib.hipGetErrorString.argtypes = [I]
                lib.hipGetLastError.restype = I
                lib.hipGetLastError.argtypes = []
            _HIP = lib  # published only once its signatures are declared
    return _HIP


def _lib_path(name: str) -> str:
    if name == "libtca_kernels.so" and os.environ.get("TCA_KERNELS_LIB"):
        return os.environ["TCA_KERNELS_LIB"]  # A/B runs against another build of the kernels
    return os.path.join(_build.LIBDIR, name)


def kernels(auto_build: bool = True) -> ctypes.CDLL:
    """The HIP kernel library. Builds it in-tree if missing (hipcc present)."""
    global _KERNELS
    if _KERNELS is not None:
        return _KERNELS
    with _LOCK:
        if _KERNELS is not None:
            return _KERNELS
        path = _lib_path("libtca_kernels.so")
        if not os.path.exists(path) and auto_build:
            _build.build(verbose=False)
        if not os.path.exists(path):
            raise NativeError(f"{path} is missing: run `python -m triton_client_amd._build` (hipcc, gfx950)")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _KERNEL_SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                # an older build (TCA_KERNELS_LIB A/B runs): a call of this entry fails loudly
                # (AttributeError) instead of the whole library failing to load
                if not os.environ.get("TCA_KERNELS_LIB"):
                    raise NativeError(f"{path}: no symbol {name}: rebuild (python -m triton_client_amd._build)")
                continue
            fn.argtypes = args
            fn.restype = I
        _KERNELS = lib
        return lib


def runtime(auto_build: bool = True) -> ctypes.CDLL:
    global _RUNTIME
    if _RUNTIME is not None:
        return _RUNTIME
    with _LOCK:
        if _RUNTIME is not None:
            return _RUNTIME
        path = _lib_path("libtca_runtime.so")
        if not os.path.exists(path) and auto_build:
            _build.build(verbose=False)
        if not os.path.exists(path):
            raise NativeError(f"{path} is missing: run `python -m triton_client_amd._build`")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        from . import _runtime_sigs  # noqa: F401  (declares argtypes)
        _runtime_sigs.declare(lib)
        # published only after argtypes are declared: another thread takes the
        # lock-free fast path above, and an undeclared pointer argument would be
        # truncated to a C int (a served-path segfault under concurrent requests)
        _RUNTIME = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        hip = _load_hip()
        msg = hip.hipGetErrorString(rc).decode() if hip is not None else f"code {rc}"
        raise NativeError(f"{what} failed: {msg} ({rc})")


def call(name: str, *args) -> None:
    """Launch through the C ABI.  The launchers report ``hipGetLastError()``
    after their launch; a stale error left by an earlier runtime call that
    its caller already handled (e.g. a pointer-attribute probe on pageable
    host memory inside a framework copy) would be misreported as this
    launch's failure, so the thread's error state is cleared first."""
    fn = getattr(kernels(), name)
    hip = _HIP if _HIP is not None else _load_hip()
    if hip is not None:
        hip.hipGetLastError()
    if args and _KERNEL_SIGS.get(name, [None])[-1] is P and _capturing():
        _check_capture_stream(name, args[-1])
    check(fn(*args), name)


def _capturing() -> bool:
    from .pipelines.graph import capturing_thread
    return capturing_thread()


def _check_capture_stream(name: str, stream) -> None:
    """While this thread captures a graph, a launch must target a capturing
    stream: one outside the capture would run once now, not on every replay."""
    from .pipelines.graph import GraphCaptureError, stream_is_capturing

    h = int(stream or 0)
    if not stream_is_capturing(h):
        raise GraphCaptureError(f"{name}: launched onto stream {hex(h)}, which is not part of the graph being "
                                "captured (its work would not replay)")


def ptr(t) -> int:
    """Device/host pointer of a tensor (0 for None)."""
    return 0 if t is None else int(t.data_ptr())


def stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def available() -> bool:
    try:
        kernels()
        return True
    except Exception:
        return False
