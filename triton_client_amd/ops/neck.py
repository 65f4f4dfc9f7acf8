"""Fused BEV neck + anchor head (HIP kernel K15, ``csrc/kernels/bev_neck.hip``).

Replaces BaseBEVBackbone's deblocks (transpose convs k = s, stride s, + BN +
ReLU, 128 channels each) and AnchorHeadSingle's merged 1x1 head with one
launch; the 384-channel concat is never written (reference config:
``data/pointpillar.yaml:48-72``).  :func:`neck_head_supported` says whether
a plan qualifies; :class:`FusedNeckHead` falls back to nothing — callers keep
the unfused plan for shapes outside the contract.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence

import torch

from .. import _native
from .conv import NHWC, FusedConv, split_pairs

CB = 128
NH_PAD = 80


def chunk32_perm() -> List[int]:
    """Position p in a 32-channel chunk -> source channel, matching the
    register layout the kernel repacks its deconv accumulators into."""
    out = []
    for g in range(4):
        for e in range(8):
            out.append(4 * g + e if e < 4 else 16 + 4 * g + (e - 4))
    return out


def permute_head_weight(w: torch.Tensor) -> torch.Tensor:
    """[nh, K] (K % 32 == 0) -> [80, K] zero-padded rows, columns permuted per 32-chunk."""
    nh, K = w.shape
    assert K % 32 == 0 and nh <= NH_PAD
    idx = torch.tensor([c * 32 + p for c in range(K // 32) for p in chunk32_perm()], dtype=torch.long)
    out = torch.zeros(NH_PAD, K, dtype=w.dtype)
    out[:nh] = w[:, idx]
    return out


def neck_head_supported(ups: Sequence[FusedConv], strides: Sequence[int], cins: Sequence[int], head: FusedConv,
                        H: int, W: int) -> bool:
    if not 1 <= len(ups) <= 3:
        return False
    S = max(strides)
    for u, s, c in zip(ups, strides, cins):
        if s < 1 or S % s or c % (32 if head.precision == "fp32" else 64) or u.cout_real != CB or u.Kp != c:
            return False
        if u.transpose and u.shuffle != s:
            return False
        if not u.transpose and (u.k != 1 or s != 1):
            return False
    return (head.k == 1 and head.N <= NH_PAD and head.N % 8 == 0 and head.Kp == CB * len(ups)
            and H % S == 0 and W % S == 0)


class FusedNeckHead:
    """out[b, y, x, :nh] = head(cat_i relu(deconv_i(x_i)))[b, y, x].

    Precision follows the convs: bf16 (``tca_bev_neck_head``) or fp32 split
    products (``tca_bev_neck_head_x3``, fp32 activations, split weights)."""

    def __init__(self, ups: Sequence[FusedConv], strides: Sequence[int], head: FusedConv, device,
                 grid: int = 0):
        self.ups, self.strides = list(ups), [int(s) for s in strides]
        self.precision = head.precision
        assert all(u.precision == self.precision for u in self.ups)
        self.dtype = head.dtype
        self.nbr = len(self.ups)
        self.nh = head.N
        # persistent kernel: workgroup slots over 3/4 of the CUs (a multiple of 8: tiles are split per XCD).
        # The neck runs beside the first down blocks of the next batch (bench.py --lidar-pipeline 5); leaving
        # them a quarter of the CUs measured +0.5% / +0.7% over the full grid on two boxes
        # (profiles/r6/knobs/sweep4_shapes.txt, sweep10_neck_grid.txt); TCA_NECK_GRID overrides
        if grid <= 0:
            grid = int(os.environ.get("TCA_NECK_GRID", "0")) or \
                torch.cuda.get_device_properties(torch.device(device)).multi_processor_count * 3 // 4
        self.grid = max(8, grid // 8 * 8)
        # fp32 tiling (bev_neck.hip tca_bev_neck_head_x3v): 0 = <8 waves, 2 stages>, 99.6 KiB LDS; 1 = <8, 3>,
        # 149 KiB; 2 = <4, 2>, two workgroups per CU (66 KiB each), the fastest alone (883 vs 1056 us).  In
        # round 5's step 0 measured best (4652 vs 4617 for 2, profiles/r5/neck_variant2_ab.txt); with round 6's
        # front and VFE beside it, 2 is ahead on two boxes: +1.2% and +0.6% over 5-6 alternating rounds each
        # (profiles/r6/knobs/), so it is the default now
        self.variant = int(os.environ.get("TCA_NECK_VARIANT", "2"))
        wh = permute_head_weight(head.w_f32_gemm[:, : head.Kp].float())
        if self.precision == "fp32":
            self.wh = split_pairs(wh).to(device)
        else:
            self.wh = wh.to(device, torch.bfloat16).contiguous()
        bh = torch.zeros(NH_PAD)
        bh[: head.N] = head.b_gemm.float().cpu()
        self.bh = bh.to(device).contiguous()
        n = self.nbr
        self._w = (ctypes.c_void_p * n)(*[u.w_gemm.data_ptr() for u in self.ups])
        self._b = (ctypes.c_void_p * n)(*[u.b_gemm.data_ptr() for u in self.ups])
        self._s = (ctypes.c_int * n)(*self.strides)
        self._cin = (ctypes.c_int * n)(*[u.Kp for u in self.ups])

    def __call__(self, xs: Sequence[NHWC], out: NHWC, stream=None) -> NHWC:
        n = self.nbr
        B, H, W, _ = out.shape
        for x, s in zip(xs, self.strides):
            assert x.shape[0] == B and x.shape[1] * s == H and x.shape[2] * s == W, (x.shape, s, out.shape)
        assert out.off == 0 and out.t.dtype == self.dtype and all(x.t.dtype == self.dtype for x in xs)
        pair = xs[0].pair
        if any(x.pair != pair for x in xs) or (pair and self.precision != "fp32") or out.pair:
            raise TypeError("neck inputs: all pair storage (fp32 mode) or none; output fp32")
        ptrs = (ctypes.c_void_p * n)(*[x.t.data_ptr() for x in xs])
        ldx = (ctypes.c_int * n)(*[x.t.shape[-1] for x in xs])
        offx = (ctypes.c_int * n)(*[x.off for x in xs])
        args = (n, ptrs, ldx, offx, self._cin, self._s, self._w, self._b, _native.ptr(self.wh),
                _native.ptr(self.bh), self.nh, _native.ptr(out.t), out.t.shape[-1], B, H, W, self.grid)
        if self.precision == "fp32":
            _native.call("tca_bev_neck_head_x3v", *args, int(pair), self.variant, _native.stream_ptr(stream))
        else:
            _native.call("tca_bev_neck_head", *args, _native.stream_ptr(stream))
        return out
