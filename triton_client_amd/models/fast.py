"""Concat-free NHWC execution plans of the detectors on the fused MFMA conv.

Every activation is an NHWC buffer (fp32 in the ``precision="fp32"`` mode:
split-product MFMA convs, the reference's serving precision; bf16 in the
``"bf16"`` mode) allocated once per batch size (so a
whole forward is hipGraph-capturable with stable addresses); a layer whose
output feeds a concatenation writes straight into its channel slice of the
concat buffer (C3's two branches, SPPF's pyramid, PANet's skip joins, the BEV
neck's three up-sampled scales), so no concat kernel ever runs.

* :class:`FastYOLOv5`  — same math as :class:`~.yolov5.YOLOv5` (BN folded),
  input ``[B, H, W, 8]`` (3 RGB channels + 5 zero pad so Cin % 8 == 0),
  outputs the three Detect maps as NHWC slices (255 of 256 channels).
* :class:`FastBEV`     — BaseBEVBackbone + AnchorHeadSingle of
  :class:`~.pointpillars.PointPillars`; the three head 1x1 convs are merged
  into one 384→72 GEMM; outputs cls / box / dir as slices of it.
* :class:`FastCenterPoint` — det3d RPN + CenterHead of
  :class:`~.centerpoint.CenterPoint` (merged head GEMMs, see the class).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .. import _native
from ..ops.conv import NHWC, FusedConv, act_dtype, maxpool_nhwc, sppf_pools, to_pairs, upsample2x_nhwc
from .common import ACT_NONE, ACT_RELU, ACT_SILU, ConvBNAct

# fused K1 + YOLOv5 stem + b1 kernel for the frame-input camera step (FastYOLOv5.stem_fused_ok)
STEM_FUSED = True
# PointPillars first block: skip the tiles of the stride-1 convs whose receptive field is empty
# canvas (_BEVBackbonePlan.forward_blocks; False: dense, for A/B runs)
BEV_UNIFORM = True
# fp32-mode BEV blocks: a conv whose successor is an F(2,3) layer (ops/conv.py WINO) writes fp32
# storage instead of pairs (conv_wino.hip then skips the pair join); the last conv of a block
# writes pairs (the next block's stride-2 conv and the deblock read them)
WINO_F32_CHAIN = True
# YOLOv5 Detect convs fused with the decode + candidate filter (FastYOLOv5.detect_fused_ok)
DETECT_FUSED = True
# the c3_fused.hip C3 blocks (_C3Plan.fused2_ok); False: the unfused chain (tests compare the two)
C3_FUSED = True
FUSED_C3_WIDTHS = (16, 32, 64)  # c_ of the blocks c3_fused.hip takes


def _fc(m: ConvBNAct, device, precision: str = "bf16", **kw) -> FusedConv:
    assert m.fused, "call fuse_model() first"
    return FusedConv(m.conv, act=m.act, device=device, precision=precision, **kw)


class _Buffers:
    def __init__(self, device, precision: str = "bf16"):
        self.device = torch.device(device)
        self.precision = precision
        # the precision's activation dtype on the GPU; fp32 on the CPU reference path
        self.dtype = act_dtype(precision) if self.device.type == "cuda" else torch.float32
        self.bufs = []

    def new(self, B, H, W, C, pair: bool = False) -> NHWC:
        t = torch.zeros((B, H, W, C), dtype=self.dtype, device=self.device)
        self.bufs.append(t)
        return NHWC(t, pair=pair)

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self.bufs)


def _merged_1x1(a: ConvBNAct, b: ConvBNAct) -> Optional[nn.Conv2d]:
    """One 1x1 conv computing [a(x) | b(x)] (output channels concatenated) when a and b are
    fused 1x1 stride-1 convs of the same input with the same activation, else None."""
    ca, cb = a.conv, b.conv
    if not (a.fused and b.fused and a.act == b.act and ca.kernel_size == cb.kernel_size == (1, 1)
            and ca.stride == cb.stride == (1, 1) and ca.in_channels == cb.in_channels and ca.groups == cb.groups == 1):
        return None
    m = nn.Conv2d(ca.in_channels, ca.out_channels + cb.out_channels, 1, 1, 0, bias=True)
    with torch.no_grad():
        m.weight.copy_(torch.cat([ca.weight.detach().float(), cb.weight.detach().float()], 0))
        zb = lambda c: c.bias.detach().float() if c.bias is not None else torch.zeros(c.out_channels)  # noqa: E731
        m.bias.copy_(torch.cat([zb(ca), zb(cb)], 0))
    return m


class _C3Plan:
    """C3: cv3(cat(m(cv1(x)), cv2(x))) with the cat buffer written in place.  cv1 and cv2
    (two 1x1 convs of the same input) run as ONE conv writing [cv1 | cv2] straight into
    the cat buffer (x read once, one launch); the bottlenecks then start from its cv1 half
    and the last one writes its output back over that half (per-element residual in
    place: each output element's residual is read by the thread that writes it)."""

    def __init__(self, c3, B, H, W, bufs: _Buffers, device):
        pr = bufs.precision
        self.cv1, self.cv2, self.cv3 = _fc(c3.cv1, device, pr), _fc(c3.cv2, device, pr), _fc(c3.cv3, device, pr)
        self.m = [(_fc(b.cv1, device, pr), _fc(b.cv2, device, pr), b.add) for b in c3.m]
        c_ = self.cv1.N
        self.c_ = c_
        mc = _merged_1x1(c3.cv1, c3.cv2) if self.cv1.N == self.cv1.cout_real == self.cv2.N else None
        self.cv12 = FusedConv(mc, act=c3.cv1.act, device=device, precision=pr) if mc is not None else None
        self.cat = bufs.new(B, H, W, 2 * c_)
        self.a = [bufs.new(B, H, W, c_), bufs.new(B, H, W, c_)]
        self.tmp = bufs.new(B, H, W, c_)
        self.out_c = self.cv3.N
        # c3_fused.hip (c_ = 16 / 32 / 64): fragment-order split weights, built here (never in a capture).
        # The 20 x 20 c_ = 128 blocks stay on the chain (measured 118 vs 165-171 us at batch 32 for a
        # first version of the kernel that took them; profiles/r4/layers_camera_c3f_v2.json)
        self._fw = None
        convs = [self.cv12, self.cv3] + [c for b1, b2, _ in self.m for c in (b1, b2)] if self.cv12 is not None else []
        if (C3_FUSED and self.cv12 is not None and c_ in FUSED_C3_WIDTHS and torch.device(device).type == "cuda"
                and (len(self.m) == 1 or all(add for _, _, add in self.m)) and (c_ >= 32 or len(self.m) == 1)
                and all(c.precision == "fp32" and not c.transpose and c.act in (0, 1, 2, 3) for c in convs)
                and self.cv12.k == 1 and self.cv12.N == 2 * c_ and self.cv12.cin_p % 32 == 0
                and self.cv3.k == 1 and self.cv3.cin_p == 2 * c_ and self.cv3.N == 2 * c_
                and all(b1.k == 1 and b1.cin_p == c_ and b1.N == c_ and b2.k == 3 and b2.s == 1 and b2.p == 1
                        and b2.cin_p == c_ and b2.N == c_ for b1, b2, _ in self.m)):
            from ..ops.conv import frag_weights
            dev = torch.device(device)
            self._fw = (frag_weights(self.cv12.w_f32_gemm).to(dev), frag_weights(self.cv3.w_f32_gemm).to(dev),
                        [(frag_weights(b1.w_f32_gemm).to(dev), frag_weights(b2.w_f32_gemm).to(dev))
                         for b1, b2, _ in self.m])

    def fused2_ok(self, x: NHWC, out: NHWC) -> bool:
        """c3_fused.hip takes this block (c_ = 32 / 64 / 128, plain fp32 in and out)."""
        return (self._fw is not None and C3_FUSED and x.t.is_cuda and not x.pair and not out.pair
                and x.t.dtype == torch.float32 and out.t.dtype == torch.float32 and x.c == self.cv12.cin_p
                and out.c == self.cv3.N and x.off % 4 == 0 and out.off % 4 == 0
                and x.t.shape[-1] % 4 == 0 and out.t.shape[-1] % 4 == 0)

    def _fused2(self, x: NHWC, out: NHWC) -> NHWC:
        """The block as 1 (n = 1) or n (FIRST, MID..., LAST) c3_fused launches."""
        import ctypes
        B, H, W, _ = x.shape
        c_, n = self.c_, len(self.m)
        w12, w3, wm = self._fw
        cat_b = (self.cat.t, 2 * c_, c_)

        def launch(mode, i, xin=None, ain=None, bin_=None, y=None, aout=None, bout=None):
            b1, b2, add = self.m[i]
            t = lambda v: v[0] if v is not None else None  # noqa: E731
            ptrs = [t(xin), t(ain), t(bin_), t(y), t(aout), t(bout), w12, self.cv12.b_gemm, wm[i][0], b1.b_gemm,
                    wm[i][1], b2.b_gemm, w3, self.cv3.b_gemm]
            pa = (ctypes.c_void_p * 14)(*[_native.ptr(p) for p in ptrs])
            ld = lambda v: (v[1], v[2]) if v is not None else (0, 0)  # noqa: E731
            iv = [mode, c_, self.cv12.cin_p, self.cv3.N, int(bool(add)), B, H, W, *ld(xin), *ld(ain), *ld(bin_),
                  *ld(y), *ld(aout), *ld(bout), self.cv12.act, b1.act, b2.act, self.cv3.act]
            ia = (ctypes.c_int * 24)(*iv)
            _native.call("tca_c3_fused", ctypes.addressof(pa), ctypes.addressof(ia), _native.stream_ptr(None))

        xv, yv = (x.t, x.t.shape[-1], x.off), (out.t, out.t.shape[-1], out.off)
        if n == 1:
            launch(0, 0, xin=xv, y=yv)
            return out
        av = [(t.t, c_, 0) for t in self.a]
        launch(1, 0, xin=xv, aout=av[0], bout=cat_b)
        for i in range(1, n - 1):
            launch(2, i, ain=av[(i - 1) % 2], aout=av[i % 2])
        launch(3, n - 1, ain=av[(n - 2) % 2], bin_=cat_b, y=yv)
        return out

    def __call__(self, x: NHWC, out: NHWC) -> NHWC:
        c_ = self.c_
        if self.fused2_ok(x, out):
            return self._fused2(x, out)
        if self.cv12 is not None:
            self.cv12(x, out=NHWC(self.cat.t, 0, 2 * c_))
            cur = NHWC(self.cat.t, 0, c_)
        else:
            cur = self.cv1(x, out=self.a[0])
        for i, (b1, b2, add) in enumerate(self.m):
            last = i == len(self.m) - 1
            dst = NHWC(self.cat.t, 0, c_) if last else self.a[(i + 1) % 2]
            u = b1(cur, out=self.tmp)
            b2(u, out=dst, res=cur if add else None)
            cur = dst
        if self.cv12 is None:
            self.cv2(x, out=NHWC(self.cat.t, c_, c_))
        return self.cv3(self.cat, out=out)


class FastYOLOv5:
    """``s2d`` (default): the input is the 2x2 space-to-depth image
    [B, H/2, W/2, 16] that the preprocess kernel writes directly, and the k=6
    s=2 p=2 stem runs as the equivalent 3x3 s=1 conv over it
    (:func:`~..ops.image.s2d_stem_weight`): 12 of 16 input channels real
    instead of 3 of 8, half the input bytes, half the stem's MACs."""
    IN_CHANNELS = 8

    def __init__(self, model, batch: int, img_hw: Tuple[int, int] = (640, 640), device="cuda", s2d: bool = True,
                 precision: str = "bf16"):
        self.device = torch.device(device)
        self.precision = pr = precision
        H, W = img_hw
        self.H, self.W = H, W
        B = batch
        bufs = self.bufs = _Buffers(self.device, precision)
        m = model
        self.s2d = s2d and H % 2 == 0 and W % 2 == 0 and m.b0.conv.kernel_size == (6, 6) \
            and m.b0.conv.stride == (2, 2) and m.b0.conv.padding == (2, 2)
        if self.s2d:
            from ..ops.image import s2d_stem_weight

            assert m.b0.fused, "call fuse_model() first"
            c0 = m.b0.conv
            stem = nn.Conv2d(16, c0.out_channels, 3, 1, 1, bias=True)
            with torch.no_grad():
                stem.weight.copy_(s2d_stem_weight(c0.weight.detach().float()))
                stem.bias.copy_(c0.bias.detach().float() if c0.bias is not None else torch.zeros(c0.out_channels))
            self.x = bufs.new(B, H // 2, W // 2, 16)
            self.b0 = FusedConv(stem, act=m.b0.act, device=device, precision=pr)
        else:
            self.x = bufs.new(B, H, W, self.IN_CHANNELS)
            self.b0 = _fc(m.b0, device, pr, cin_pad=self.IN_CHANNELS)
        self.b1, self.b3, self.b5, self.b7 = (_fc(getattr(m, n), device, pr) for n in ("b1", "b3", "b5", "b7"))
        h2, w2 = H // 2, W // 2
        s4, s8, s16, s32 = (H // 4, W // 4), (H // 8, W // 8), (H // 16, W // 16), (H // 32, W // 32)
        self.t0 = bufs.new(B, h2, w2, self.b0.N)
        self.t1 = bufs.new(B, *s4, self.b1.N)
        self.c3_2 = _C3Plan(m.b2, B, *s4, bufs, device)
        self.t2 = bufs.new(B, *s4, self.c3_2.out_c)
        self.t3 = bufs.new(B, *s8, self.b3.N)
        self.c3_4 = _C3Plan(m.b4, B, *s8, bufs, device)
        c_p3 = self.c3_4.out_c
        self.h14 = _fc(m.h14, device, pr)
        self.cat17 = bufs.new(B, *s8, self.h14.N + c_p3)  # [up(h14) | p3]
        self.p3 = NHWC(self.cat17.t, self.h14.N, c_p3)
        self.t5 = bufs.new(B, *s16, self.b5.N)
        self.c3_6 = _C3Plan(m.b6, B, *s16, bufs, device)
        c_p4 = self.c3_6.out_c
        self.h10 = _fc(m.h10, device, pr)
        self.cat13 = bufs.new(B, *s16, self.h10.N + c_p4)  # [up(h10) | p4]
        self.p4 = NHWC(self.cat13.t, self.h10.N, c_p4)
        self.t7 = bufs.new(B, *s32, self.b7.N)
        self.c3_8 = _C3Plan(m.b8, B, *s32, bufs, device)
        self.t8 = bufs.new(B, *s32, self.c3_8.out_c)
        # SPPF
        self.sp1, self.sp2 = _fc(m.b9.cv1, device, pr), _fc(m.b9.cv2, device, pr)
        cs = self.sp1.N
        self.spcat = bufs.new(B, *s32, 4 * cs)
        self.t9 = bufs.new(B, *s32, self.sp2.N)
        self.k = m.b9.k
        # head
        self.h18, self.h21 = _fc(m.h18, device, pr), _fc(m.h21, device, pr)
        self.cat23 = bufs.new(B, *s32, self.h21.N + self.h10.N)  # [h21 | h10]
        self.h10_out = NHWC(self.cat23.t, self.h21.N, self.h10.N)
        self.c3_13 = _C3Plan(m.h13, B, *s16, bufs, device)
        self.t13 = bufs.new(B, *s16, self.c3_13.out_c)
        self.cat20 = bufs.new(B, *s16, self.h18.N + self.h14.N)  # [h18 | h14]
        self.h14_out = NHWC(self.cat20.t, self.h18.N, self.h14.N)
        self.c3_17 = _C3Plan(m.h17, B, *s8, bufs, device)
        self.o3 = bufs.new(B, *s8, self.c3_17.out_c)
        self.c3_20 = _C3Plan(m.h20, B, *s16, bufs, device)
        self.o4 = bufs.new(B, *s16, self.c3_20.out_c)
        self.c3_23 = _C3Plan(m.h23, B, *s32, bufs, device)
        self.o5 = bufs.new(B, *s32, self.c3_23.out_c)
        self.det = [FusedConv(c, act=ACT_NONE, device=device, precision=pr) for c in m.detect]
        self.dout = [bufs.new(B, *s, d.N) for s, d in zip((s8, s16, s32), self.det)]
        self.no_real = m.detect[0].out_channels

    def stem_fused_ok(self) -> bool:
        """The fused K1 + stem + b1 kernel (ops/image.py yolo_stem_fused) takes this plan:
        fp32, s2d stem 16 -> 16, b1 3x3 stride 2 16 -> 32, image sides divisible by 4.
        STEM_FUSED False keeps the three-kernel chain."""
        b0, b1 = self.b0, self.b1
        return (STEM_FUSED and self.s2d and self.precision == "fp32" and b0.N == 16 and b0.cin_p == 16
                and b0.Kp == 160 and b0.k == 3 and b0.s == 1 and b1.cin_p == 16 and b1.N == 32 and b1.Kp == 160
                and b1.k == 3 and b1.s == 2 and b1.p == 1 and not self.t1.pair
                and self.H % 4 == 0 and self.W % 4 == 0 and b0.act in (0, 1, 2, 3) and b1.act in (0, 1, 2, 3))

    def input_view(self) -> torch.Tensor:
        """[B, 3, H, W] channels_last view of the RGB part of the input buffer
        (what the preprocess kernel writes; channels 3..7 stay zero).  Not
        available in the space-to-depth layout: use :meth:`set_input`."""
        if self.s2d:
            raise RuntimeError("space-to-depth input: use set_input()")
        return self.x.t.permute(0, 3, 1, 2)

    def set_input(self, x: torch.Tensor) -> None:
        """x: [B, 3, H, W] normalised image -> the plan's input buffer."""
        if (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and self.x.t.is_contiguous()
                and self.x.t.shape[-1] in (8, 16)):
            from ..ops.image import planar_affine

            planar_affine(x, self.x.t)  # one kernel: layout change + channel pad (+ S2D)
            return
        if self.s2d:
            from ..ops.image import space_to_depth2

            self.x.t.copy_(space_to_depth2(x.permute(0, 2, 3, 1).to(self.x.t.device)).to(self.x.t.dtype))
        else:
            self.x.t.zero_()
            self.x.t[..., :3].copy_(x.permute(0, 2, 3, 1))

    def detect_fused_ok(self) -> bool:
        """The fused Detect convs + decode + filter kernel (ops/yolo.py YoloPostprocess.detect_fused,
        yolo_detect.hip) takes this plan's head: fp32, 1x1 stride-1 convs without activation over
        fp32 NHWC inputs with cin in {64, 128, 256}, 256 output rows.  DETECT_FUSED False keeps the
        convs + tca_yolo_decode_filter."""
        return (DETECT_FUSED and self.precision == "fp32" and self.device.type == "cuda"
                and all(d.k == 1 and d.s == 1 and d.p == 0 and not d.transpose and d.act == ACT_NONE
                        and d.cin_p in (64, 128, 256) and d.K == d.Kp and d.N == 256
                        and d.w_gemm.shape == (256, 2 * d.cin_p) and o.c == d.cin_p and not o.pair
                        for d, o in zip(self.det, (self.o3, self.o4, self.o5))))

    def forward(self, from_t1: bool = False, heads: bool = True) -> List[NHWC]:
        """from_t1: b1's output is already in ``t1`` (the fused K1 + stem + b1 kernel ran).
        heads False: stop before the Detect convs and return their inputs (o3, o4, o5)."""
        if from_t1:
            t = self.t1
        else:
            t = self.b0(self.x, out=self.t0)
            t = self.b1(t, out=self.t1)
        t = self.c3_2(t, out=self.t2)
        t = self.b3(t, out=self.t3)
        p3 = self.c3_4(t, out=self.p3)
        t = self.b5(p3, out=self.t5)
        p4 = self.c3_6(t, out=self.p4)
        t = self.b7(p4, out=self.t7)
        t = self.c3_8(t, out=self.t8)
        cs = self.sp1.N
        y0 = self.sp1(t, out=NHWC(self.spcat.t, 0, cs))
        sppf_pools(y0, self.spcat.t, cs, self.k)
        t9 = self.sp2(self.spcat, out=self.t9)
        h10 = self.h10(t9, out=self.h10_out)
        upsample2x_nhwc(h10, NHWC(self.cat13.t, 0, self.h10.N))
        t13 = self.c3_13(self.cat13, out=self.t13)
        h14 = self.h14(t13, out=self.h14_out)
        upsample2x_nhwc(h14, NHWC(self.cat17.t, 0, self.h14.N))
        o3 = self.c3_17(self.cat17, out=self.o3)
        self.h18(o3, out=NHWC(self.cat20.t, 0, self.h18.N))
        o4 = self.c3_20(self.cat20, out=self.o4)
        self.h21(o4, out=NHWC(self.cat23.t, 0, self.h21.N))
        o5 = self.c3_23(self.cat23, out=self.o5)
        if not heads:
            return [o3, o4, o5]
        outs = []
        for d, o, dst in zip(self.det, (o3, o4, o5), self.dout):
            d(o, out=dst)
            outs.append(NHWC(dst.t, 0, self.no_real))
        return outs


class _BEVBackbonePlan:
    """BaseBEVBackbone / det3d RPN: down blocks (ping-pong buffers) and deblocks
    writing straight into their channel slices of the concat buffer."""

    def __init__(self, bb, B: int, ny: int, nx: int, bufs: _Buffers, device, pair: bool = False):
        self.blocks = []
        H, W = ny, nx
        pr = bufs.precision
        convs_all = [[_fc(c, device, pr) for c in blk] for blk in bb.blocks]
        ups_all = [FusedConv(u.conv, act=ACT_RELU, device=device, precision=pr) for u in bb.deblocks]
        # pair storage (fp32 mode): every conv must take it (global_load_lds kernels)
        self.pair = pair and torch.device(device).type == "cuda" and all(
            c.pair_ok() for c in [cv for blk in convs_all for cv in blk] + ups_all)
        for convs in convs_all:
            s = convs[0].s
            H, W = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
            pp = [bufs.new(B, H, W, convs[0].N, self.pair), bufs.new(B, H, W, convs[0].N, self.pair)]
            self.blocks.append((convs, pp, H, W))
        self.ups = []
        up_c = [u.conv.out_channels for u in bb.deblocks]
        s0 = bb.deblocks[0].s
        if s0 < 1:
            k = int(round(1 / s0))
            H0, W0 = self.blocks[0][2] // k, self.blocks[0][3] // k
        else:
            H0, W0 = self.blocks[0][2] * int(round(s0)), self.blocks[0][3] * int(round(s0))
        self.out_hw = (H0, W0)
        self.cat = bufs.new(B, H0, W0, sum(up_c), self.pair)
        off = 0
        for u, fc, c in zip(bb.deblocks, ups_all, up_c):
            assert u.fused, "call fuse_model() first"
            self.ups.append((fc, off, c))
            off += c
        self.ny, self.nx = ny, nx
        self.uni_vals = self._uniform_values(device) if BEV_UNIFORM else None
        self.depth = None
        if self.uni_vals is not None:
            _, _, H1, W1 = self.blocks[0]
            self.depth = torch.zeros((B, H1, W1), dtype=torch.uint8, device=device)

    def out_pair(self, convs, i: int) -> bool:
        """Storage of conv i's output in its block: fp32 when the next conv is an F(2,3) layer and
        this conv can write fp32 (an F(2,3) layer, or the stride-2 hx3 kernel), else pairs."""
        from ..ops import conv as conv_mod
        if not (self.pair and WINO_F32_CHAIN and conv_mod.WINO) or i + 1 >= len(convs):
            return True
        cv, nxt = convs[i], convs[i + 1]
        return not (nxt.wino_ok() and (cv.wino_ok() or (cv.s == 2 and cv.hx3_ok() and conv_mod.HX3S2)))

    def _uniform_eligible(self) -> bool:
        convs = self.blocks[0][0]
        return (self.pair and len(convs) >= 2 and convs[0].s == 2 and convs[0].hx3_ok()
                and all(c.s == 1 and c.hx3_ok() for c in convs[1:]) and len(convs) <= 8)

    @torch.no_grad()
    def _uniform_values(self, device) -> Optional[List[torch.Tensor]]:
        """Pair storage of each first-block conv's output on a uniform pixel (see conv_hx3.hip
        tca_bev_uniform_depth): one image of the canvas shape with nothing occupied, run through
        the same kernels (same tile choice: the shapes match), and read at the centre.  Built
        here, outside any graph capture; the plan's weights are fixed from here on."""
        if not self._uniform_eligible() or torch.cuda.is_current_stream_capturing():
            return None
        convs = self.blocks[0][0]
        x = NHWC(torch.zeros((1, self.ny, self.nx, convs[0].cin_p), dtype=torch.float32, device=device), pair=True,
                 occ=torch.zeros((1, self.ny, self.nx), dtype=torch.uint8, device=device))
        vals = []
        for i, cv in enumerate(convs):
            Ho, Wo = cv.out_hw(x.t.shape[1], x.t.shape[2])
            x = cv(x, out=NHWC(torch.zeros((1, Ho, Wo, cv.N), dtype=torch.float32, device=device),
                               pair=self.out_pair(convs, i)))
            vals.append(x.t[0, Ho // 2, Wo // 2].clone())
        torch.cuda.synchronize(device)
        return vals

    def forward_blocks(self, canvas: NHWC, stop: Optional[int] = None, outs: Optional[List[NHWC]] = None,
                       mark: Optional[tuple] = None) -> List[NHWC]:
        """The down blocks only: each block's output (the deblocks' inputs).  With the canvas
        occupancy, the first block's stride-1 convs store their constant on the tiles whose
        receptive field holds no occupied cell (tca_bev_uniform_depth); bit-identical.
        stop: run blocks [0, stop) only; outs: the outputs of the blocks already run (continue
        from the last one -- bench.py --lidar-pipeline 4 runs the last block in the back half).
        mark = (n, event): record the event on the current stream after the first n convs."""
        outs = list(outs or [])
        x = outs[-1] if outs else canvas
        first = len(outs)
        stop = len(self.blocks) if stop is None else stop
        uni = (first == 0 and self.uni_vals is not None and canvas is not None and canvas.occ is not None
               and BEV_UNIFORM)
        if uni:
            B, ny, nx = canvas.occ.shape
            assert (ny, nx) == (self.ny, self.nx) and B == self.depth.shape[0], (canvas.occ.shape, self.depth.shape)
            _native.call("tca_bev_uniform_depth", _native.ptr(canvas.occ), B, ny, nx, len(self.blocks[0][0]),
                         _native.ptr(self.depth), _native.stream_ptr(None))
        issued = sum(len(c) for c, _, _, _ in self.blocks[:first])
        for bi, (convs, pp, H, W) in enumerate(self.blocks):
            if bi < first or bi >= stop:
                continue
            for i, cv in enumerate(convs):
                # the stride-2 conv skips tiles whose windows hold no occupied cell (depth >= 1)
                u = (self.depth, i + 1, self.uni_vals[i]) if uni and bi == 0 else None
                o = pp[i % 2] if self.out_pair(convs, i) else NHWC(pp[i % 2].t, pair=False)
                x = cv(x, out=o, uni=u)
                issued += 1
                if mark is not None and issued == mark[0]:
                    mark[1].record()
            outs.append(x)
        return outs

    def convs_before(self, n_blocks: int) -> int:
        """Convs in the first n_blocks down blocks."""
        return sum(len(c) for c, _, _, _ in self.blocks[:n_blocks])

    def up_strides(self, bb) -> List[float]:
        return [float(u.s) for u in bb.deblocks]

    def forward(self, canvas: NHWC) -> NHWC:
        for x, (up, off, c) in zip(self.forward_blocks(canvas), self.ups):
            up(x, out=self.cat.slice(off, c))
        return self.cat


class FastBEV:
    """PointPillars BEV backbone + anchor head on fused convs."""

    def __init__(self, model, batch: int, device="cuda", fused_neck: bool = True,
                 bev_hw: Optional[Tuple[int, int]] = None, precision: str = "bf16", pair: bool = True):
        """bev_hw: (ny, nx) of the backbone input when it is not the voxel grid
        (SECOND: the 8x-downsampled HeightCompression map)."""
        self.device = torch.device(device)
        self.precision = precision
        cfg = model.cfg
        if bev_hw is not None:
            ny, nx = bev_hw
        else:
            nx, ny, _ = cfg.voxel.grid_size
        B = batch
        bufs = self.bufs = _Buffers(self.device, precision)
        # fp32 mode keeps the BEV chain in pair storage (hi / lo bf16 halves as the
        # MFMA fragments read them): no split on any operand read
        self.bb = _BEVBackbonePlan(model.backbone, B, ny, nx, bufs, device, pair=pair and precision == "fp32")
        self.pair = self.bb.pair
        self.canvas_pairs = None  # conversion buffer for callers that hand in a plain fp32 canvas
        self.blocks, self.ups, self.cat, self.out_hw = self.bb.blocks, self.bb.ups, self.bb.cat, self.bb.out_hw
        H0, W0 = self.out_hw
        hd = model.head
        merged = nn.Conv2d(hd.conv_cls.in_channels,
                           hd.conv_cls.out_channels + hd.conv_box.out_channels + hd.conv_dir.out_channels, 1)
        with torch.no_grad():
            merged.weight.copy_(torch.cat([hd.conv_cls.weight, hd.conv_box.weight, hd.conv_dir.weight]).float())
            merged.bias.copy_(torch.cat([hd.conv_cls.bias, hd.conv_box.bias, hd.conv_dir.bias]).float())
        self.head = FusedConv(merged, act=ACT_NONE, device=device, precision=precision)
        self.n_cls, self.n_box, self.n_dir = (hd.conv_cls.out_channels, hd.conv_box.out_channels,
                                              hd.conv_dir.out_channels)
        self.hout = bufs.new(B, H0, W0, self.head.N)
        if self.pair and not self.head.pair_ok():
            raise ValueError("pair storage: the head conv must take the global_load_lds kernels")
        # deblocks + head as one kernel (K15) when the shapes fit its contract
        self.neck = None
        strides = self.bb.up_strides(model.backbone)
        if self.device.type == "cuda" and fused_neck and all(s >= 1 and float(s).is_integer() for s in strides):
            from ..ops.neck import FusedNeckHead, neck_head_supported

            ups = [u for u, _, _ in self.ups]
            si = [int(s) for s in strides]
            cins = [blk[0][-1].N for blk in self.blocks]
            if neck_head_supported(ups, si, cins, self.head, H0, W0):
                self.neck = FusedNeckHead(ups, si, self.head, self.device)

    def first_conv_gated(self) -> bool:
        """The plan's only reader of the pillar canvas is its first conv, and (pair storage with the
        occupancy bytes) that conv loads only occupied cells: a non-transposed conv of at most 32
        taps over pairs takes an occupancy-gated kernel (ops/conv.py: s2sp, hx3s2, x3p_occ)."""
        cv = self.blocks[0][0][0]
        return bool(self.pair and not cv.transpose and cv.k * cv.k <= 32)

    def forward(self, canvas: NHWC):
        if self.pair and not canvas.pair:
            if self.canvas_pairs is None or self.canvas_pairs.t.shape != canvas.tensor().shape:
                self.canvas_pairs = NHWC(torch.empty_like(canvas.tensor(), dtype=torch.float32), pair=True)
            self.canvas_pairs.t.copy_(to_pairs(canvas.tensor()))
            canvas = self.canvas_pairs
        elif canvas.pair and not self.pair:
            raise TypeError("pair canvas handed to a plan built without pair storage")
        if self.neck is not None:
            self.neck(self.bb.forward_blocks(canvas), self.hout)
        else:
            self.head(self.bb.forward(canvas), out=self.hout)
        return self.head_maps()

    def forward_blocks(self, canvas: NHWC, stop: Optional[int] = None, mark: Optional[tuple] = None) -> List[NHWC]:
        """The down blocks only (pair canvas), or the first ``stop`` of them; forward_neck finishes
        the batch from their outputs, which stay in this plan's buffers until its next
        forward_blocks.  mark = (n, event): the event is recorded after the first n convs."""
        assert self.neck is not None and canvas.pair == self.pair
        return self.bb.forward_blocks(canvas, stop, mark=mark)

    def forward_neck(self, blocks: List[NHWC]):
        if len(blocks) < len(self.bb.blocks):  # the remaining down blocks first
            blocks = self.bb.forward_blocks(None, outs=blocks)
        self.neck(blocks, self.hout)
        return self.head_maps()

    def head_maps(self):
        t = self.hout.t
        return (NHWC(t, 0, self.n_cls), NHWC(t, self.n_cls, self.n_box),
                NHWC(t, self.n_cls + self.n_box, self.n_dir))


class FastCenterPoint:
    """CenterPoint-PP RPN + CenterHead on fused convs (bf16 or fp32 split-product
    activations, like the other plans).

    * shared conv 3x3 384→64 (+BN+ReLU);
    * all tasks' first-level head convs (6 tasks × 6 heads × conv3x3 64→64
      +BN+ReLU) as ONE 64→2304 GEMM into a [B,H,W,2304] buffer;
    * per task, its heads' final 3x3 convs as one conv over the task's 384-channel
      slice with block-diagonal weights (out = reg2|height1|dim3|rot2|vel2|hm nc,
      padded to 16) writing channels [16t, 16t+16) of the merged head output —
      the layout :class:`~..ops.centerpoint.CenterPointPostprocess` decodes.
    """

    TASK_STRIDE = 16

    def __init__(self, model, batch: int, device="cuda", precision: str = "bf16"):
        from .centerpoint import HEAD_ORDER

        self.device = torch.device(device)
        self.precision = precision
        cfg = self.cfg = model.cfg
        nx, ny, _ = cfg.voxel.grid_size
        B = batch
        bufs = self.bufs = _Buffers(self.device, precision)
        self.bb = _BEVBackbonePlan(model.backbone, B, ny, nx, bufs, device)
        H0, W0 = self.bb.out_hw
        hd = model.head
        self.shared = _fc(hd.shared, device, precision)
        self.sh = bufs.new(B, H0, W0, self.shared.N)
        names = list(HEAD_ORDER) + ["hm"]
        pre = [t.pre[n] for t in hd.tasks for n in names]
        c_mid = pre[0].conv.out_channels
        big = nn.Conv2d(pre[0].conv.in_channels, c_mid * len(pre), 3, 1, 1)
        with torch.no_grad():
            big.weight.copy_(torch.cat([m.conv.weight for m in pre]).float())
            big.bias.copy_(torch.cat([m.conv.bias for m in pre]).float())
        self.pre = FusedConv(big, act=ACT_RELU, device=device, precision=precision)
        self.mid = bufs.new(B, H0, W0, self.pre.N)
        self.c_task_in = c_mid * len(names)
        self.finals = []
        for t, task in enumerate(hd.tasks):
            outs = [task.out[n] for n in names]
            n_out = sum(o.out_channels for o in outs)
            assert n_out <= self.TASK_STRIDE
            conv = nn.Conv2d(self.c_task_in, self.TASK_STRIDE, 3, 1, 1)
            with torch.no_grad():
                conv.weight.zero_()
                conv.bias.zero_()
                o0 = 0
                for h, o in enumerate(outs):
                    conv.weight[o0:o0 + o.out_channels, h * c_mid:(h + 1) * c_mid] = o.weight.float()
                    conv.bias[o0:o0 + o.out_channels] = o.bias.float()
                    o0 += o.out_channels
            self.finals.append(FusedConv(conv, act=ACT_NONE, device=device, precision=precision))
        self.task_offsets = [t * self.TASK_STRIDE for t in range(len(hd.tasks))]
        self.hout = bufs.new(B, H0, W0, self.TASK_STRIDE * len(hd.tasks))

    def forward(self, canvas: NHWC) -> NHWC:
        cat = self.bb.forward(canvas)
        self.shared(cat, out=self.sh)
        self.pre(self.sh, out=self.mid)
        for t, fc in enumerate(self.finals):
            fc(NHWC(self.mid.t, t * self.c_task_in, self.c_task_in),
               out=NHWC(self.hout.t, t * self.TASK_STRIDE, self.TASK_STRIDE))
        return self.hout


def _conv_out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


class FastDetectron:
    """Detectron2 RetinaNet / FCOS (ResNet-50-FPN) on fused convs.

    * input ``x`` [B, H, W, 8]: the K1 kernel writes normalised RGB + 5 zero pad
      channels (mean/std folded into K1's per-channel scale / bias);
    * bottleneck outputs relu(conv3 + shortcut) via the post-residual epilogue;
    * FPN top-down add fused as the lateral conv's residual (upsample2x → lateral);
    * RetinaNet: the cls and box towers' first convs share their input, so they
      run as one 256→512 GEMM; the head weights are shared over levels, each
      level has its own output buffers;
    * FCOS: GroupNorm(32)+ReLU kernels between the tower convs.
    """

    IN_CHANNELS = 8

    def __init__(self, model, batch: int, device="cuda", precision: str = "bf16"):
        """precision: "bf16", or "fp32" (the reference serves these networks at fp32:
        split-product convs, fp32 activations, fp32 GroupNorm / decode)."""
        from ..ops.conv import FusedConv

        self.device = torch.device(device)
        self.precision = precision
        cfg = self.cfg = model.cfg
        B = self.B = batch
        H, W = cfg.input_hw
        bufs = self.bufs = _Buffers(self.device, precision)
        self.x = bufs.new(B, H, W, self.IN_CHANNELS)
        bb = model.backbone
        P = precision
        self.stem = _fc(bb.stem, device, P, cin_pad=self.IN_CHANNELS)
        h, w = _conv_out(H, 7, 2, 3), _conv_out(W, 7, 2, 3)
        self.stem_out = bufs.new(B, h, w, 64)
        h, w = _conv_out(h, 3, 2, 1), _conv_out(w, 3, 2, 1)
        self.pool = bufs.new(B, h, w, 64)
        self.stages = []
        x_c = 64
        for st in bb.stages:
            blocks = []
            for blk in st:
                c1, c2, c3 = _fc(blk.conv1, device, P), _fc(blk.conv2, device, P), blk.conv3
                s = blk.conv1.s if blk.conv1.s > 1 else blk.conv2.s
                ho, wo = _conv_out(h, 1, s, 0), _conv_out(w, 1, s, 0)
                f3 = FusedConv(c3.conv, act=ACT_RELU, device=device, post_res=True, precision=P)
                sc = _fc(blk.shortcut, device, P) if blk.shortcut is not None else None
                t1, t2 = bufs.new(B, ho, wo, c1.N), bufs.new(B, ho, wo, c2.N)
                sbuf = bufs.new(B, ho, wo, sc.N) if sc is not None else None
                out = bufs.new(B, ho, wo, f3.N)
                blocks.append((c1, c2, f3, sc, t1, t2, sbuf, out))
                h, w, x_c = ho, wo, f3.N
            self.stages.append(blocks)
        fpn = model.fpn
        C = cfg.fpn_channels
        self.lv_hw = [blocks[-1][7].shape[1:3] for blocks in self.stages[1:]]  # res3..res5
        self.lat = [_fc(m, device, P) for m in fpn.lateral]
        self.outc = [_fc(m, device, P) for m in fpn.output]
        self.lat_buf = [bufs.new(B, hh, ww, C) for hh, ww in self.lv_hw]
        self.up_buf = [bufs.new(B, hh, ww, C) for hh, ww in self.lv_hw[:2]]
        self.p = [bufs.new(B, hh, ww, C) for hh, ww in self.lv_hw]
        self.p6p7_from_c5 = fpn.p6p7_from_c5
        p6 = fpn.p6.conv
        self.p6 = FusedConv(p6, act=ACT_NONE, device=device, precision=P)
        self.p6r = FusedConv(p6, act=ACT_RELU, device=device, precision=P)
        self.p7 = _fc(fpn.p7, device, P)
        h5, w5 = self.lv_hw[2]
        h6, w6 = _conv_out(h5, 3, 2, 1), _conv_out(w5, 3, 2, 1)
        h7, w7 = _conv_out(h6, 3, 2, 1), _conv_out(w6, 3, 2, 1)
        self.p.append(bufs.new(B, h6, w6, C))
        self.p6relu = bufs.new(B, h6, w6, C)
        self.p.append(bufs.new(B, h7, w7, C))
        self.level_hw = [tuple(t.shape[1:3]) for t in self.p]
        # ---- head
        hd = model.head
        self.fcos = cfg.arch == "fcos"
        if self.fcos:
            cls_convs = [m for m in hd.cls_subnet if isinstance(m, nn.Conv2d)]
            box_convs = [m for m in hd.bbox_subnet if isinstance(m, nn.Conv2d)]
            self.gn_cls = [m for m in hd.cls_subnet if isinstance(m, nn.GroupNorm)]
            self.gn_box = [m for m in hd.bbox_subnet if isinstance(m, nn.GroupNorm)]
            act = ACT_NONE
        else:
            cls_convs = [m.conv for m in hd.cls_subnet]
            box_convs = [m.conv for m in hd.bbox_subnet]
            act = ACT_RELU
        first = nn.Conv2d(C, 2 * C, 3, 1, 1)
        with torch.no_grad():
            first.weight.copy_(torch.cat([cls_convs[0].weight, box_convs[0].weight]).float())
            first.bias.copy_(torch.cat([cls_convs[0].bias, box_convs[0].bias]).float())
        self.t_first = FusedConv(first, act=act, device=device, precision=P)
        self.t_cls = [FusedConv(m, act=act, device=device, precision=P) for m in cls_convs[1:]]
        self.t_box = [FusedConv(m, act=act, device=device, precision=P) for m in box_convs[1:]]
        self.cls_score = FusedConv(hd.cls_score, act=ACT_NONE, device=device, precision=P)
        if self.fcos:
            merged = nn.Conv2d(C, 5, 3, 1, 1)
            with torch.no_grad():
                merged.weight.copy_(torch.cat([hd.bbox_pred.weight, hd.ctrness.weight]).float())
                merged.bias.copy_(torch.cat([hd.bbox_pred.bias, hd.ctrness.bias]).float())
            self.box_pred = FusedConv(merged, act=ACT_NONE, device=device, precision=P)
            dev = self.device
            f32 = lambda t: t.detach().float().contiguous().to(dev)  # noqa: E731
            self.gn_params = [(f32(torch.cat([gc.weight, gb.weight])), f32(torch.cat([gc.bias, gb.bias])))
                              for gc, gb in zip(self.gn_cls[:1], self.gn_box[:1])]
            self.gn_params += [((f32(gc.weight), f32(gc.bias)), (f32(gb.weight), f32(gb.bias)))
                               for gc, gb in zip(self.gn_cls[1:], self.gn_box[1:])]
            self.gn_groups = self.gn_cls[0].num_groups
            self.gn_eps = self.gn_cls[0].eps
        else:
            self.box_pred = FusedConv(hd.bbox_pred, act=ACT_NONE, device=device, precision=P)
        self.lvl = []
        for hh, ww in self.level_hw:
            self.lvl.append(dict(first=bufs.new(B, hh, ww, 2 * C), a=bufs.new(B, hh, ww, C), b=bufs.new(B, hh, ww, C),
                                 c=bufs.new(B, hh, ww, C), d=bufs.new(B, hh, ww, C),
                                 cls=bufs.new(B, hh, ww, self.cls_score.N), box=bufs.new(B, hh, ww, self.box_pred.N)))
        from ..ops._ws import Workspace
        self.ws = Workspace(self.device) if self.device.type == "cuda" else None

    def input_view(self) -> torch.Tensor:
        return self.x.t.permute(0, 3, 1, 2)

    def _gn(self, x: NHWC, gamma, beta, groups=None):
        from ..ops.detectron import group_norm_nhwc
        group_norm_nhwc(x, gamma, beta, groups or self.gn_groups, self.gn_eps, relu=True, ws=self.ws)

    def forward(self):
        from ..ops.conv import maxpool2d_nhwc, upsample2x_nhwc

        self.stem(self.x, out=self.stem_out)
        maxpool2d_nhwc(self.stem_out, self.pool, 3, 2, 1)
        x = self.pool
        feats = []
        for blocks in self.stages:
            for c1, c2, f3, sc, t1, t2, sbuf, out in blocks:
                c1(x, out=t1)
                c2(t1, out=t2)
                res = sc(x, out=sbuf) if sc is not None else x
                f3(t2, out=out, res=res)
                x = out
            feats.append(x)
        c3, c4, c5 = feats[1], feats[2], feats[3]
        cs = [c3, c4, c5]
        self.lat[2](c5, out=self.lat_buf[2])
        self.outc[2](self.lat_buf[2], out=self.p[2])
        for i in (1, 0):
            upsample2x_nhwc(self.lat_buf[i + 1], self.up_buf[i])
            self.lat[i](cs[i], out=self.lat_buf[i], res=self.up_buf[i])
            self.outc[i](self.lat_buf[i], out=self.p[i])
        src6 = c5 if self.p6p7_from_c5 else self.p[2]
        self.p6(src6, out=self.p[3])
        self.p6r(src6, out=self.p6relu)
        self.p7(self.p6relu, out=self.p[4])
        C = self.cfg.fpn_channels
        outs = []
        for lv, p in zip(self.lvl, self.p):
            f = self.t_first(p, out=lv["first"])
            if self.fcos:
                g, b = self.gn_params[0]
                self._gn(f, g, b, 2 * self.gn_groups)  # both towers at once: 512 channels, 64 groups of 8
            c_in, b_in = NHWC(f.t, 0, C), NHWC(f.t, C, C)
            cbuf, bbuf = (lv["a"], lv["b"]), (lv["c"], lv["d"])
            for k, (cc, cb) in enumerate(zip(self.t_cls, self.t_box)):
                c_in = cc(c_in, out=cbuf[k % 2])
                b_in = cb(b_in, out=bbuf[k % 2])
                if self.fcos:
                    (gc, bc), (gb, bb2) = self.gn_params[k + 1]
                    self._gn(c_in, gc, bc)
                    self._gn(b_in, gb, bb2)
            self.cls_score(c_in, out=lv["cls"])
            self.box_pred(b_in, out=lv["box"])
            if self.fcos:
                outs.append((NHWC(lv["cls"].t, 0, self.cfg.num_classes), NHWC(lv["box"].t, 0, 4),
                             NHWC(lv["box"].t, 4, 1)))
            else:
                outs.append((NHWC(lv["cls"].t, 0, self.cfg.num_anchors * self.cfg.num_classes),
                             NHWC(lv["box"].t, 0, self.cfg.num_anchors * 4)))
        return outs


class FastGraph:
    """A darknet-style layer graph (``model.spec``: conv / route / add / maxpool /
    upsample, e.g. :data:`~.yolov4.YOLOV4_SPEC`) on the fused NHWC convs.

    * route (concat) buffers are allocated once and each source writes straight
      into its channel slice (a source feeding a second route is copied);
    * ``add`` of a conv output that nothing else reads is fused into that conv's
      epilogue (residual), so residual blocks cost one launch per conv;
    * maxpool / upsample read and write channel slices.
    Input: ``x`` [B, H, W, 8] (RGB + zero pad, written by K1).
    """

    IN_CHANNELS = 8

    def __init__(self, model, batch: int, img_hw, device="cuda", outputs: Sequence[str] = (),
                 precision: str = "bf16"):
        from ..ops.conv import FusedConv

        self.device = torch.device(device)
        self.precision = precision
        B = self.B = batch
        H, W = img_hw
        spec, layers = model.spec, model.layers
        bufs = self.bufs = _Buffers(self.device, precision)
        shape = {"input": (H, W)}
        chan = {"input": self.IN_CHANNELS}
        consumers: dict = {}
        for name, op, a in spec:
            srcs = a["srcs"] if op == "route" else ([a["a"], a["b"]] if op == "add" else [a["src"]])
            for s in srcs:
                consumers.setdefault(s, []).append(name)
            if op == "conv":
                k, st = a["k"], a["s"]
                h, w = shape[a["src"]]
                shape[name] = ((h + 2 * (k // 2) - k) // st + 1, (w + 2 * (k // 2) - k) // st + 1)
                chan[name] = _ceil8(a["c"])
            elif op == "route":
                shape[name] = shape[a["srcs"][0]]
                chan[name] = sum(chan[s] for s in a["srcs"])
            elif op == "add":
                shape[name], chan[name] = shape[a["a"]], chan[a["a"]]
            elif op == "upsample":
                h, w = shape[a["src"]]
                shape[name], chan[name] = (2 * h, 2 * w), chan[a["src"]]
            else:
                shape[name], chan[name] = shape[a["src"]], chan[a["src"]]
        # fused adds: conv output read only by the add → the conv writes the add's value
        fused_add = {}
        for name, op, a in spec:
            if op == "add":
                c = next((x for x in spec if x[0] == a["a"]), None)
                if c is not None and c[1] == "conv" and consumers.get(a["a"]) == [name]:
                    fused_add[a["a"]] = (name, a["b"])
        # buffers: route slices first
        self.view = {"input": None}
        slot = {}
        for name, op, a in spec:
            if op == "route":
                h, w = shape[name]
                rb = bufs.new(B, h, w, chan[name])
                self.view[name] = rb
                off = 0
                for s in a["srcs"]:
                    src_name = s
                    if s not in slot:
                        slot[s] = NHWC(rb.t, off, chan[s])
                    else:
                        slot[(name, s)] = NHWC(rb.t, off, chan[s])  # needs a copy
                    off += chan[s]
        self.x = bufs.new(B, H, W, self.IN_CHANNELS)
        self.view["input"] = self.x
        self.ops = []
        for name, op, a in spec:
            if op == "route":
                for s in a["srcs"]:
                    if (name, s) in slot:
                        self.ops.append(("copy", (name, s), s))
                continue
            target = name
            if op == "conv" and name in fused_add:
                target = fused_add[name][0]
            if op == "add" and name in [v[0] for v in fused_add.values()]:
                continue  # produced by its conv
            if target not in self.view:
                h, w = shape[target]
                self.view[target] = slot.get(target) or bufs.new(B, h, w, chan[target])
            if op == "conv":
                m = layers[name]
                assert m.fused, "call fuse_model() first"
                fc = FusedConv(m.conv, act=m.act, device=device, precision=precision,
                               cin_pad=self.IN_CHANNELS if a["src"] == "input" else None)
                res = fused_add[name][1] if name in fused_add else None
                self.ops.append(("conv", fc, a["src"], target, res))
            elif op == "add":
                self.ops.append(("add", a["a"], a["b"], name))
            elif op == "maxpool":
                self.ops.append(("maxpool", a["src"], name, a["k"]))
            elif op == "upsample":
                self.ops.append(("upsample", a["src"], name))
        for k, v in list(slot.items()):
            if isinstance(k, tuple):
                self.view[k] = v
        self.outputs = list(outputs)

    def input_view(self) -> torch.Tensor:
        return self.x.t.permute(0, 3, 1, 2)

    def forward(self):
        from ..ops.conv import maxpool_nhwc, upsample2x_nhwc

        v = self.view
        for op in self.ops:
            kind = op[0]
            if kind == "conv":
                _, fc, src, dst, res = op
                fc(v[src], out=v[dst], res=v[res] if res is not None else None)
            elif kind == "maxpool":
                maxpool_nhwc(v[op[1]], v[op[2]], op[3])
            elif kind == "upsample":
                upsample2x_nhwc(v[op[1]], v[op[2]])
            elif kind == "add":
                v[op[3]].tensor().copy_(v[op[1]].tensor() + v[op[2]].tensor())
            elif kind == "copy":
                v[op[1]].tensor().copy_(v[op[2]].tensor())
        return [v[n] for n in self.outputs]


def _ceil8(c):
    return (c + 7) // 8 * 8
