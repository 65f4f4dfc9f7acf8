"""Fused NHWC convolution (``csrc/kernels/conv_mfma.hip``), bf16 or fp32.

:class:`FusedConv` packs a (BN-folded) ``Conv2d`` / ``ConvTranspose2d``
(k == stride) into the kernel's GEMM layout once and runs
``act(conv(x) + bias) (+ residual)`` in one launch, reading and writing
channel slices of wider NHWC buffers (:class:`NHWC`), so the detectors'
concatenations are free.

Precision (``precision=``):

* ``"fp32"`` — fp32 activations; every product on the bf16 MFMA as three
  split terms (``xh*wh + xh*wl + xl*wh``, fp32 accumulate, see
  ``tca_conv_nhwc_x3``): the reference's fp32 serving precision
  (``examples/YOLOv5/config.pbtxt:7,16``) at 3x the bf16 MFMA work.
* ``"bf16"`` — bf16 activations and weights, fp32 accumulation.

CPU tensors take an fp32 PyTorch path with the same semantics (used for tests
on the GPU-less host).
"""
from __future__ import annotations

import os

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native
from ..models.common import ACT_LEAKY, ACT_NONE, ACT_RELU, ACT_SILU, apply_act


@dataclass
class NHWC:
    """A channel slice [off, off + c) of an NHWC buffer ``t`` [B, H, W, C].

    ``pair``: the fp32 buffer holds fp32-mode *pair* storage — per 8
    channels {hi bf16 x 8 | lo bf16 x 8}, the bytes of 8 fp32 (see
    :func:`to_pairs`); the split-product kernels read its halves as MFMA
    fragments directly.  ``tensor()`` is then the raw storage; ``values()``
    / ``nchw()`` decode it."""
    t: torch.Tensor
    off: int = 0
    c: Optional[int] = None
    pair: bool = False
    # optional uint8 [B, H, W] pixel occupancy (a sparse BEV canvas): pair convs read an
    # unmarked pixel as zeros without fetching it (conv_mfma.hip tca_conv_nhwc_x3p_occ)
    occ: Optional[torch.Tensor] = None

    def __post_init__(self):
        if self.c is None:
            self.c = self.t.shape[-1] - self.off
        if self.pair:
            assert self.t.dtype == torch.float32 and self.off % 8 == 0 and self.c % 8 == 0, (self.off, self.c)

    @property
    def shape(self):
        return (*self.t.shape[:3], self.c)

    def tensor(self) -> torch.Tensor:
        return self.t[..., self.off:self.off + self.c]

    def slice(self, off: int, c: int) -> "NHWC":
        return NHWC(self.t, self.off + off, c, self.pair)

    def values(self) -> torch.Tensor:
        """NHWC fp32 / bf16 values of the slice (pairs decoded)."""
        return from_pairs(self.tensor()) if self.pair else self.tensor()

    def nchw(self) -> torch.Tensor:
        return self.values().permute(0, 3, 1, 2)


def to_pairs(x: torch.Tensor) -> torch.Tensor:
    """[..., C] fp32 values (C % 8 == 0) -> [..., C] fp32 *storage* holding, per
    8 channels, hi = bf16(x) then lo = bf16(x - hi)."""
    *lead, C = x.shape
    assert C % 8 == 0, C
    v = x.float().reshape(*lead, C // 8, 1, 8)
    hi = v.to(torch.bfloat16)
    lo = (v - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], -2).reshape(*lead, 2 * C).view(torch.float32)


def from_pairs(p: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`to_pairs`: pair storage -> fp32 values (hi + lo)."""
    *lead, C = p.shape
    assert C % 8 == 0, C
    h = p.contiguous().view(torch.bfloat16).reshape(*lead, C // 8, 2, 8).float()
    return (h[..., 0, :] + h[..., 1, :]).reshape(*lead, C)


def _ceil(x, m):
    return (x + m - 1) // m * m


PRECISIONS = ("fp32", "bf16")
# split-product tiles with pair-storage instantiations (conv_mfma.hip launch_glds_x3p: global_load_lds
# kernels 20-42, buffer-descriptor DMA kernels 68-79)
PAIR_TILES = (20, 22, 24, 25, 26, 32, 37, 41, 42, 68, 69, 70, 71, 72, 73, 74, 75, 76, 77, 78, 79, 90, 91, 92, 93, 94, 95, 96, 97, 102)


# conv_hx3.hip (3x3 stride-1 / stride-2 pair convs with register-streamed fragment-order
# weights): the default for every eligible layer (HX3 / HX3S2 False: the conv_mfma.hip tiles,
# for A/B runs).  Tiles 110 (auto) and 111-116 (hx3_launch tiles 1-6) select the stride-1
# kernel explicitly, 120 and 121-124 (hx3s2_launch tiles 1-4) the stride-2 one.
HX3 = True
HX3S2 = True
HX3_TILES = (110, 111, 112, 113, 114, 115, 116)
HX3S2_TILES = (120, 121, 122, 123, 124)
# conv_wino.hip (3x3 stride-1 by 1-D Winograd F(2,3), 1.5x fewer MFMAs than hx3): the default for
# every eligible stride-1 layer (WINO False: hx3).  Tiles 130 (auto) and 131-134 select it explicitly.
WINO = os.environ.get("TCA_WINO", "1") != "0"  # TCA_WINO=0: hx3 for A/B runs
# conv_s2sp.hip (the sparse-gather stride-2 conv: only (pixel, tap) pairs whose input cell is
# occupied) for a stride-2 pair conv over an occupancy-marked canvas with N == 64 and Cin 32 / 64
# (the first PointPillars BEV conv).  Opt-in (S2SP True / TCA_S2SP=1): measured no faster than the
# dense occupancy-masked hx3s2 kernel in the step (profiles/r5/s2sp/), which stays the default.
# Tiles 140 (auto: 4 x 32 output tiles), 141 (8 x 32) and 142 (2 x 32) select it explicitly.
S2SP = os.environ.get("TCA_S2SP", "0") == "1"
S2SP_TILES = (140, 141, 142)
S2SP_TILE = int(os.environ.get("TCA_S2SP_TILE", "0"))
WINO_MIN_N = int(os.environ.get("TCA_WINO_MIN_N", "128"))  # narrower layers stay on hx3 (A/B: profiles/r5/wino_ab.md)
WINO_TILES = (130, 131, 132, 133, 134)
# sweep overrides of the auto tile choice (tools/gpu_knob_sweep.sh): hx3_launch / hx3s2_launch / wino_launch tile
# numbers applied where the caller asked for tile 0; unset = the kernels' own choice
HX3_TILE_AUTO = int(os.environ.get("TCA_HX3_TILE", "0"))
HX3S2_TILE_AUTO = int(os.environ.get("TCA_HX3S2_TILE", "0"))
WINO_TILE_AUTO = int(os.environ.get("TCA_WINO_TILE", "0"))


def wino_tile(H: int, W: int, N: int) -> int:
    """conv_wino.hip wino_launch tile for an H x W output with N channels: F(2,3) along the axis
    that pads less to 32 (tiles 2 / 4: along y), 32 (1, 2) or 16 (3, 4) channels per wave."""
    cm = (H + 31) // 32 * 32 * W <= (W + 31) // 32 * 32 * H
    return (2 if cm else 1) if N % 128 == 0 else (4 if cm else 3)


def wino_taps(W: torch.Tensor, cin: int, cm: bool) -> torch.Tensor:
    """[N, 9 * cin] GEMM weights (K order (ky * 3 + kx) * cin + ci) -> the F(2,3)-transformed taps
    [N, 3 line taps kl, 4 positions p, cin] in fp64.  The Winograd axis is y when ``cm`` (line taps
    kl = kx), else x (kl = ky): V0 = g0, V1 = (g0 + g1 + g2) / 2, V2 = (g0 - g1 + g2) / 2, V3 = g2."""
    N = W.shape[0]
    g = W[:, :9 * cin].double().reshape(N, 3, 3, cin)  # n, ky, kx, ci
    if cm:
        g = g.permute(0, 2, 1, 3)  # n, kl = kx, kf = ky, ci
    g0, g1, g2 = g[:, :, 0], g[:, :, 1], g[:, :, 2]
    return torch.stack([g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2], 2)


def wino_weights(W: torch.Tensor, cin: int, cm: bool) -> torch.Tensor:
    """The conv_wino.hip weight image: wino_taps in fragment order (frag_weights over
    K = (kl * 4 + p) * cin + ci)."""
    N = W.shape[0]
    return frag_weights(wino_taps(W, cin, cm).reshape(N, 12 * cin).float())


def frag_weights(W: torch.Tensor) -> torch.Tensor:
    """[N, Kp] fp32 GEMM weights (N % 16 == 0, Kp % 32 == 0) -> the split weights in MFMA
    fragment order, [Kp/32][N/16][hi, lo][64 lanes][8] bf16: lane = fq * 16 + fr holds
    output channel 16 g + fr, K indices 32 ks + 8 fq .. + 8 (the B operand of
    mfma_f32_16x16x32_bf16), so one fragment load is one contiguous 1 KiB."""
    N, Kp = W.shape
    assert N % 16 == 0 and Kp % 32 == 0, (N, Kp)
    hi, lo = split_bf16(W)
    t = torch.stack([hi, lo], 0).reshape(2, N // 16, 16, Kp // 32, 4, 8)  # h, g, fr, ks, fq, e
    return t.permute(3, 1, 0, 4, 2, 5).contiguous()  # ks, g, h, fq, fr, e


def act_dtype(precision: str) -> torch.dtype:
    """Activation dtype of a precision mode."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")
    return torch.float32 if precision == "fp32" else torch.bfloat16


def split_bf16(w: torch.Tensor):
    """fp32 -> (hi, lo) bf16 with hi = rne(w), lo = rne(w - hi)."""
    w = w.float()
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return hi, lo


def split_pairs(w: torch.Tensor) -> torch.Tensor:
    """[N, K] fp32 (K % 8 == 0) -> [N, 2K] bf16: per 8 columns, 8 hi then 8 lo —
    the split-weight layout of the fp32-mode kernels."""
    N, K = w.shape
    assert K % 8 == 0, K
    hi, lo = split_bf16(w)
    return torch.stack([hi.reshape(N, K // 8, 8), lo.reshape(N, K // 8, 8)], 2).reshape(N, 2 * K).contiguous()


def nhwc_dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 2
    raise TypeError(f"NHWC activations must be fp32 or bf16, got {t.dtype}")


class FusedConv:
    def __init__(self, conv: nn.Module, act: int = ACT_NONE, device="cuda", cin_pad: Optional[int] = None,
                 cout_pad: Optional[int] = None, post_res: bool = False, precision: str = "bf16"):
        w = conv.weight.detach().float()
        b = conv.bias.detach().float() if conv.bias is not None else None
        self.transpose = isinstance(conv, nn.ConvTranspose2d)
        self.device = torch.device(device)
        self.act = act
        self.post_res = post_res  # act(conv + residual): ResNet bottleneck output
        self.precision = precision
        self.dtype = act_dtype(precision)
        if self.transpose:
            cin, cout, kh, kw = w.shape
            s = conv.stride[0]
            assert kh == kw == s and conv.padding[0] == 0, "only k == stride transpose convs"
            self.shuffle, self.k, self.s, self.p = s, 1, 1, 0
            self.cout_real = cout
            # GEMM N index = (sy*s + sx)*cout + co
            wg = w.permute(2, 3, 1, 0).reshape(s * s * cout, cin)  # [N, Cin]
            bias = b.repeat(s * s) if b is not None else None
            self.ref = conv
        else:
            cout, cin, kh, kw = w.shape
            assert kh == kw
            self.shuffle, self.k, self.s, self.p = 0, kh, conv.stride[0], conv.padding[0]
            self.cout_real = cout
            wg = w
            bias = b
            self.ref = conv
        self.cin = cin
        self.cin_p = cin_pad or _ceil(cin, 8)
        if self.transpose:
            wk = torch.zeros(wg.shape[0], self.cin_p)
            wk[:, :cin] = wg
            K = self.cin_p
        else:
            wk = torch.zeros(cout, kh, kw, self.cin_p)
            wk[..., :cin] = wg.permute(0, 2, 3, 1)
            wk = wk.reshape(cout, -1)
            K = kh * kw * self.cin_p
        N = wk.shape[0]
        self.N = cout_pad or _ceil(N, 8)
        self.K, self.Kp = K, _ceil(K, 32)
        W = torch.zeros(self.N, self.Kp)
        W[:N, :K] = wk
        self.bias = torch.zeros(self.N)
        if bias is not None:
            self.bias[:N] = bias
        self.w_f32_gemm = W  # [N, Kp] fp32 (host): the fused neck re-packs from it
        if precision == "fp32":
            self.w_gemm = split_pairs(W).to(self.device)  # [N, 2*Kp] bf16 hi/lo
        else:
            self.w_gemm = W.to(self.device, torch.bfloat16).contiguous()
        self.b_gemm = self.bias.to(self.device).contiguous()
        # fragment-order weights of the hx3 kernel (built here, never inside a graph capture)
        self._w_frag = frag_weights(W).to(self.device) if self.hx3_ok() and self.device.type == "cuda" else None
        # fp32 copies for the CPU path
        self.w_f32, self.b_f32 = w, b

    def out_hw(self, H, W):
        if self.transpose:
            return H * self.shuffle, W * self.shuffle
        return (H + 2 * self.p - self.k) // self.s + 1, (W + 2 * self.p - self.k) // self.s + 1

    def out_channels(self) -> int:
        return self.cout_real if self.transpose else self.N

    def __call__(self, x: NHWC, out: Optional[NHWC] = None, res: Optional[NHWC] = None, tile: int = 0,
                 stream=None, uni=None) -> NHWC:
        """uni: optional (depth uint8 [B, Ho, Wo], min depth, pair value [N]) — hx3 tiles whose
        pixels all reach the depth store the value instead of computing it (conv_hx3.hip
        tca_conv_hx3p_uni; see _BEVBackbonePlan)."""
        B, H, W, C = x.shape
        Ho, Wo = self.out_hw(H, W)
        if out is None:
            out = NHWC(torch.empty((B, Ho, Wo, self.out_channels()), dtype=self.dtype, device=x.t.device))
        if x.t.device.type != "cuda":
            return self._cpu(x, out, res)
        assert C == self.cin_p, (C, self.cin_p)
        for t in (x.t, out.t) + ((res.t,) if res is not None else ()):
            if t.dtype != self.dtype:
                raise TypeError(f"{self.precision} conv needs {self.dtype} activations, got {t.dtype}")
        gh, gw = (H, W) if self.transpose else (Ho, Wo)
        act = self.act | (16 if (self.post_res and res is not None) else 0)
        rp = (_native.ptr(res.t if res is not None else None), res.t.shape[-1] if res is not None else 0,
              res.off if res is not None else 0)
        if (x.occ is None and res is None and self.wino_ok() and not self.transpose and
                (tile in WINO_TILES or (tile == 0 and WINO))):
            # F(2,3) stride-1 kernel: pair or fp32 storage on either side
            return self._wino(x, out, tile, stream, uni)
        if x.pair or out.pair:
            # pair storage: the global_load_lds split-product kernels (Cin % 32, K == Kp)
            if self.precision != "fp32" or not x.pair or (res is not None and res.pair != out.pair):
                raise TypeError("pair activations: fp32 convs reading pairs (output pairs or fp32)")
            if (res is None and x.occ is not None and self.s2sp_ok() and
                    (tile in S2SP_TILES or (tile == 0 and S2SP))):
                assert x.occ.dtype == torch.uint8 and tuple(x.occ.shape) == (B, H, W), (x.occ.shape, (B, H, W))
                _native.call("tca_conv_s2sp", _native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off,
                             _native.ptr(self.hx3_weights()), _native.ptr(self.b_gemm), self.N,
                             _native.ptr(out.t), out.t.shape[-1], out.off, self.act | (0 if out.pair else 32),
                             _native.ptr(x.occ), tile - 140 if tile in S2SP_TILES else S2SP_TILE,
                             _native.stream_ptr(stream))
                return out
            if ((out.pair or res is None) and self.hx3_ok() and self.s == 2 and
                    (tile in HX3S2_TILES or (tile == 0 and HX3S2))):
                occ = x.occ
                if occ is not None:
                    assert occ.dtype == torch.uint8 and tuple(occ.shape) == (B, H, W), (occ.shape, (B, H, W))
                # act | 32: fp32 storage out (the input of an F(2,3) layer)
                _native.call("tca_conv_hx3s2p", _native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off,
                             _native.ptr(self.hx3_weights()), _native.ptr(self.b_gemm), self.N,
                             _native.ptr(out.t), out.t.shape[-1], out.off, act | (0 if out.pair else 32), *rp,
                             _native.ptr(occ), *self._uni_args(uni, B, Ho, Wo, res),
                             tile - 120 if tile in HX3S2_TILES else HX3S2_TILE_AUTO, _native.stream_ptr(stream))
                return out
            if (out.pair and x.occ is None and self.hx3_ok() and self.s == 1 and
                    (tile in HX3_TILES or (tile == 0 and HX3))):
                if uni is not None and res is None:
                    depth, dmin, val = uni
                    assert depth.dtype == torch.uint8 and tuple(depth.shape) == (B, Ho, Wo), depth.shape
                    assert val.dtype == torch.float32 and val.numel() == self.N, (val.dtype, val.shape)
                    _native.call("tca_conv_hx3p_uni", _native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off,
                                 _native.ptr(self.hx3_weights()), _native.ptr(self.b_gemm), self.N,
                                 _native.ptr(out.t), out.t.shape[-1], out.off, act, _native.ptr(depth), dmin,
                                 _native.ptr(val), tile - 110 if tile in HX3_TILES else HX3_TILE_AUTO,
                                 _native.stream_ptr(stream))
                    return out
                _native.call("tca_conv_hx3p", _native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off,
                             _native.ptr(self.hx3_weights()), _native.ptr(self.b_gemm), self.N,
                             _native.ptr(out.t), out.t.shape[-1], out.off, act, *rp,
                             tile - 110 if tile in HX3_TILES else HX3_TILE_AUTO, _native.stream_ptr(stream))
                return out
            args = (_native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off, _native.ptr(self.w_gemm),
                    _native.ptr(self.b_gemm), self.N, self.k, self.k, self.s, self.p, self.Kp, _native.ptr(out.t), gh,
                    gw, out.t.shape[-1], out.off, act, *rp, self.shuffle, tile if tile in PAIR_TILES else 0,
                    int(out.pair))
            if x.occ is not None and not self.transpose:
                assert x.occ.dtype == torch.uint8 and tuple(x.occ.shape) == (B, H, W), (x.occ.shape, (B, H, W))
                _native.call("tca_conv_nhwc_x3p_occ", *args, _native.ptr(x.occ), _native.stream_ptr(stream))
            else:
                _native.call("tca_conv_nhwc_x3p", *args, _native.stream_ptr(stream))
            return out
        fn = "tca_conv_nhwc_x3" if self.precision == "fp32" else "tca_conv_nhwc"
        _native.call(fn, _native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off,
                     _native.ptr(self.w_gemm), _native.ptr(self.b_gemm), self.N, self.k, self.k, self.s, self.p,
                     self.Kp, _native.ptr(out.t), gh, gw, out.t.shape[-1], out.off, act, *rp, self.shuffle, tile,
                     _native.stream_ptr(stream))
        return out

    def hx3_ok(self) -> bool:
        """conv_hx3.hip takes this conv: fp32, 3x3 stride 1 or 2, pad 1, Cin % 32, N % 64."""
        return (self.precision == "fp32" and not self.transpose and self.k == 3 and self.s in (1, 2) and self.p == 1
                and self.cin_p % 32 == 0 and self.K == self.Kp and self.N % 64 == 0)

    def _uni_args(self, uni, B, Ho, Wo, res=None):
        """(depth, uni_min, value) pointers of an optional uniform-tile skip (see _BEVBackbonePlan)."""
        if uni is None or res is not None:
            return None, 0, None
        depth, dmin, val = uni
        assert depth.dtype == torch.uint8 and tuple(depth.shape) == (B, Ho, Wo), depth.shape
        assert val.dtype == torch.float32 and val.numel() == self.N, (val.dtype, val.shape)
        return _native.ptr(depth), dmin, _native.ptr(val)

    def wino_ok(self) -> bool:
        """conv_wino.hip takes this conv: hx3's shapes at stride 1, ReLU or no activation."""
        return self.hx3_ok() and self.s == 1 and self.act in (ACT_NONE, ACT_RELU) and self.N >= WINO_MIN_N

    def _wino(self, x: NHWC, out: NHWC, tile: int, stream, uni) -> NHWC:
        B, H, W, _ = x.shape
        t = tile - 130 if tile in WINO_TILES[1:] else (WINO_TILE_AUTO or wino_tile(H, W, self.N))
        cm = t in (2, 4)
        if not hasattr(self, "_w_wino"):
            self._w_wino = {}
        wf = self._w_wino.get(cm)
        if wf is None:  # built on first use, never inside a graph capture (the plans warm up first)
            wf = self._w_wino[cm] = wino_weights(self.w_f32_gemm, self.cin_p, cm).to(self.device)
        depth, dmin, val = uni if uni is not None else (None, 0, None)
        if uni is not None:
            assert depth.dtype == torch.uint8 and tuple(depth.shape) == (B, H, W), depth.shape
            assert val.dtype == torch.float32 and val.numel() == self.N, (val.dtype, val.shape)
        _native.call("tca_conv_wino", _native.ptr(x.t), B, H, W, self.cin_p, x.t.shape[-1], x.off, int(x.pair),
                     _native.ptr(wf), _native.ptr(self.b_gemm), self.N, _native.ptr(out.t), out.t.shape[-1], out.off,
                     int(out.pair), self.act, _native.ptr(depth), dmin, _native.ptr(val), t,
                     _native.stream_ptr(stream))
        return out

    def hx3_weights(self) -> torch.Tensor:
        if self._w_frag is None:
            self._w_frag = frag_weights(self.w_f32_gemm).to(self.device)
        return self._w_frag

    def s2sp_ok(self) -> bool:
        """The sparse-gather stride-2 kernel takes this conv (conv_s2sp.hip: 3x3 stride 2 pad 1,
        N == 64, Cin 32 / 64, pair weights)."""
        return (self.precision == "fp32" and not self.transpose and self.k == 3 and self.s == 2 and self.p == 1
                and self.N == 64 and self.cin_p in (32, 64) and self.K == self.Kp
                and self.act in (ACT_NONE, ACT_RELU, ACT_SILU, ACT_LEAKY))

    def pair_ok(self) -> bool:
        """The pair-storage kernels take this conv (Cin % 32, K == Kp)."""
        return self.precision == "fp32" and self.cin_p % 32 == 0 and self.K == self.Kp

    def _cpu(self, x: NHWC, out: NHWC, res: Optional[NHWC]) -> NHWC:
        xi = x.nchw().float()[:, : self.cin]
        if self.transpose:
            y = F.conv_transpose2d(xi, self.w_f32, self.b_f32, stride=self.shuffle)
        else:
            y = F.conv2d(xi, self.w_f32, self.b_f32, stride=self.s, padding=self.p)
        if res is not None and self.post_res:
            y = apply_act(y + res.nchw().float()[:, : y.shape[1]], self.act)
        else:
            y = apply_act(y, self.act)
            if res is not None:
                y = y + res.nchw().float()[:, : y.shape[1]]
        out.tensor()[..., : y.shape[1]].copy_(y.permute(0, 2, 3, 1).to(out.t.dtype))
        return out


def sppf_pools(y0: NHWC, dst: torch.Tensor, cs: int, k: int = 5, stream=None) -> None:
    """YOLOv5 SPPF: y1 = pool(y0), y2 = pool(y1), y3 = pool(y2) (k x k, stride 1) into the channel
    slices [cs, 2cs), [2cs, 3cs), [3cs, 4cs) of dst.  One launch (nhwc_ops.hip tca_sppf_pool3) when
    the image plane fits its LDS, else three max-pools; the same bits either way."""
    B, H, W, C = y0.shape
    e = 4 if y0.t.dtype == torch.float32 else 8
    if (y0.t.is_cuda and C % (4 * e) == 0 and 2 * H * W * 64 <= 64 * 1024 and y0.off % e == 0
            and y0.t.shape[-1] % e == 0 and dst.shape[-1] % e == 0 and cs % e == 0):
        _native.call("tca_sppf_pool3", _native.ptr(y0.t), B, H, W, C, y0.t.shape[-1], y0.off, k, _native.ptr(dst),
                     dst.shape[-1], cs, 2 * cs, 3 * cs, nhwc_dtype_code(y0.t), _native.stream_ptr(stream))
        return
    y1 = maxpool_nhwc(y0, NHWC(dst, cs, cs), k, stream)
    y2 = maxpool_nhwc(y1, NHWC(dst, 2 * cs, cs), k, stream)
    maxpool_nhwc(y2, NHWC(dst, 3 * cs, cs), k, stream)


def maxpool_nhwc(x: NHWC, out: NHWC, k: int = 5, stream=None) -> NHWC:
    """k x k max-pool, stride 1, pad k//2 (SPPF), slice → slice."""
    B, H, W, C = x.shape
    if x.t.device.type != "cuda":
        y = F.max_pool2d(x.nchw().float(), k, 1, k // 2)
        out.tensor().copy_(y.permute(0, 2, 3, 1).to(out.t.dtype))
        return out
    _native.call("tca_maxpool_nhwc", _native.ptr(x.t), B, H, W, C, x.t.shape[-1], x.off, k, _native.ptr(out.t),
                 out.t.shape[-1], out.off, nhwc_dtype_code(x.t), _native.stream_ptr(stream))
    return out


def maxpool2d_nhwc(x: NHWC, out: NHWC, k: int = 3, s: int = 2, p: int = 1, stream=None) -> NHWC:
    """k x k max-pool with stride / padding (ResNet stem), slice → slice; out holds Ho x Wo."""
    B, H, W, C = x.shape
    Ho, Wo = out.shape[1], out.shape[2]
    if x.t.device.type != "cuda":
        y = F.max_pool2d(x.nchw().float(), k, s, p)
        out.tensor().copy_(y.permute(0, 2, 3, 1).to(out.t.dtype))
        return out
    _native.call("tca_maxpool2d_nhwc", _native.ptr(x.t), B, H, W, C, x.t.shape[-1], x.off, k, s, p,
                 _native.ptr(out.t), Ho, Wo, out.t.shape[-1], out.off, nhwc_dtype_code(x.t), _native.stream_ptr(stream))
    return out


def upsample2x_nhwc(x: NHWC, out: NHWC, stream=None) -> NHWC:
    """Nearest 2x upsample, slice → slice."""
    B, H, W, C = x.shape
    if x.t.device.type != "cuda":
        y = F.interpolate(x.nchw().float(), scale_factor=2.0, mode="nearest")
        out.tensor().copy_(y.permute(0, 2, 3, 1).to(out.t.dtype))
        return out
    _native.call("tca_upsample2x_nhwc", _native.ptr(x.t), B, H, W, C, x.t.shape[-1], x.off, _native.ptr(out.t),
                 out.t.shape[-1], out.off, nhwc_dtype_code(x.t), _native.stream_ptr(stream))
    return out
