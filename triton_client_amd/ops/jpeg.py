"""JPEG ingest: C++ Huffman decode into pinned staging, pixel reconstruction on
the GPU.

Reference: the camera node decodes each ``CompressedImage`` with
``cv2.imdecode`` + BGR→RGB on the subscriber thread, one message at a time
(``communicator/ros_inference.py:124-131``).  Here a batch of JPEGs is split:

* host (``csrc/runtime/jpeg_entropy.cpp``): marker parsing and Huffman
  decoding — the inherently serial part — on a pool of C++ threads (no GIL),
  writing quantised DCT coefficients straight into a pinned staging slot;
* GPU (``csrc/kernels/jpeg.hip``): dequantise + 8x8 IDCT (one wave64 per
  block), libjpeg-style fancy chroma upsampling and fixed-point YCbCr→RGB,
  written into the camera pipeline's uint8 NHWC frame buffer.

Frames the entropy decoder does not handle (progressive, arithmetic,
multi-scan) or whose geometry differs from the batch's are decoded by PIL on
the host and copied in, so any JPEG works; the fast path covers baseline
camera streams.  :func:`reconstruct_numpy` is the CPU reference of the GPU
stage (float64 IDCT, same upsampling / colour rules), used by the tests.
"""
from __future__ import annotations

import ctypes
import io
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native

GEOM_FIELDS = 16
ERRORS = {-1: "not a JPEG", -2: "unsupported JPEG (progressive / arithmetic / multi-scan / 12-bit)",
          -3: "corrupt JPEG", -4: "more blocks than the staging slot holds", -5: "truncated JPEG"}


@dataclass(frozen=True)
class JpegGeometry:
    width: int
    height: int
    nc: int
    hmax: int
    vmax: int
    mcux: int
    mcuy: int
    sampling: tuple  # ((h0, v0), (h1, v1), (h2, v2))
    nblocks: int

    @staticmethod
    def from_record(g: np.ndarray) -> "JpegGeometry":
        g = [int(v) for v in g]
        return JpegGeometry(g[0], g[1], g[2], g[3], g[4], g[5], g[6],
                            ((g[7], g[8]), (g[9], g[10]), (g[11], g[12])), g[13])

    def blocks(self, c: int):
        """(rows, cols) of component c's MCU-padded block grid."""
        h, v = self.sampling[c]
        return self.mcuy * v, self.mcux * h

    @property
    def plane_bytes(self) -> int:
        return sum(r * 8 * c * 8 for r, c in (self.blocks(c) for c in range(self.nc)))

    @property
    def gpu_ok(self) -> bool:
        if self.nc == 1:
            return True
        (h0, v0), (h1, v1), (h2, v2) = self.sampling
        if (h0, v0) != (self.hmax, self.vmax) or (h1, v1) != (h2, v2):
            return False
        return (self.hmax // h1, self.vmax // v1) in ((1, 1), (2, 1), (2, 2))


def _rt():
    return _native.runtime()


def probe(data: bytes) -> JpegGeometry:
    g = np.zeros(GEOM_FIELDS, np.int32)
    rc = _rt().tca_jpeg_probe(data, len(data), g.ctypes.data)
    if rc:
        raise ValueError(ERRORS.get(rc, f"JPEG error {rc}"))
    return JpegGeometry.from_record(g)


def decode_coefficients(data: bytes):
    """One JPEG -> (coef int16 [nblocks, 64] natural order, q float32 [3, 64],
    geometry)."""
    geo = probe(data)
    coef = np.empty((geo.nblocks, 64), np.int16)
    q = np.empty((3, 64), np.float32)
    g = np.zeros(GEOM_FIELDS, np.int32)
    rc = _rt().tca_jpeg_decode_coefs(data, len(data), coef.ctypes.data, geo.nblocks, q.ctypes.data, g.ctypes.data)
    if rc:
        raise ValueError(ERRORS.get(rc, f"JPEG error {rc}"))
    return coef, q, geo


def _idct_basis() -> np.ndarray:
    n = np.arange(8)[:, None]
    k = np.arange(8)[None, :]
    return 0.5 * np.where(k == 0, np.sqrt(0.5), 1.0) * np.cos((2 * n + 1) * k * np.pi / 16)  # [n, k]


def _upsample(p: np.ndarray, hs: int, vs: int, W: int, H: int) -> np.ndarray:
    """libjpeg fancy upsampling of a chroma plane cropped to its real size."""
    cw, ch = -(-W // hs), -(-H // vs)
    p = p[:ch, :cw].astype(np.int32)
    if hs == 1 and vs == 1:
        out = p
    elif vs == 1:
        left = np.concatenate([p[:, :1], p[:, :-1]], 1)
        right = np.concatenate([p[:, 1:], p[:, -1:]], 1)
        even = np.where(np.arange(cw)[None] == 0, p, (3 * p + left + 1) >> 2)
        odd = np.where(np.arange(cw)[None] == cw - 1, p, (3 * p + right + 2) >> 2)
        out = np.stack([even, odd], 2).reshape(ch, 2 * cw)
    else:
        up = np.concatenate([p[:1], p[:-1]], 0)
        down = np.concatenate([p[1:], p[-1:]], 0)
        rows = []
        for far in (up, down):
            s = 3 * p + far
            sl = np.concatenate([s[:, :1], s[:, :-1]], 1)
            sr = np.concatenate([s[:, 1:], s[:, -1:]], 1)
            first, last = np.arange(cw)[None] == 0, np.arange(cw)[None] == cw - 1
            even = np.where(first, (4 * s + 8) >> 4, (3 * s + sl + 8) >> 4)
            odd = np.where(last, (4 * s + 7) >> 4, (3 * s + sr + 7) >> 4)
            rows.append(np.stack([even, odd], 2).reshape(ch, 2 * cw))
        out = np.stack(rows, 1).reshape(2 * ch, 2 * cw)
    return out[:H, :W]


def reconstruct_numpy(coef: np.ndarray, q: np.ndarray, geo: JpegGeometry) -> np.ndarray:
    """CPU reference of the GPU stage: coefficients -> RGB uint8 [H, W, 3]."""
    C = _idct_basis()
    planes = []
    off = 0
    for c in range(geo.nc):
        bh, bw = geo.blocks(c)
        blk = coef[off:off + bh * bw].reshape(bh, bw, 8, 8).astype(np.float64) * q[c].reshape(8, 8)
        off += bh * bw
        pix = np.einsum("yv,abvu,xu->abyx", C, blk, C)  # column then row pass
        pix = np.clip(np.floor(pix + 128.5), 0, 255).astype(np.int32)
        planes.append(pix.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8))
    W, H = geo.width, geo.height
    Y = planes[0][:H, :W]
    if geo.nc == 1:
        return np.repeat(Y[..., None], 3, 2).astype(np.uint8)
    hs, vs = geo.hmax // geo.sampling[1][0], geo.vmax // geo.sampling[1][1]
    cb = _upsample(planes[1], hs, vs, W, H) - 128
    cr = _upsample(planes[2], hs, vs, W, H) - 128
    r = Y + ((91881 * cr + 32768) >> 16)
    g = Y + ((-22554 * cb + 32768 - 46802 * cr) >> 16)
    b = Y + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


def decode_pil(data: bytes) -> np.ndarray:
    from PIL import Image

    im = Image.open(io.BytesIO(data))
    if im.mode != "RGB":
        im = im.convert("RGB")
    return np.asarray(im)


class JpegBatchDecoder:
    """Batches of JPEG frames -> uint8 RGB NHWC frames on the GPU.

    ``stage(jpegs)`` runs the C++ entropy decoder on ``threads`` host threads
    (no GIL) into the next pinned slot — call it while the GPU works on the
    previous batch; ``upload(slot, stream)`` queues the slot's H2D copy (on a
    copy stream, so it overlaps compute); ``reconstruct(out)`` queues the two
    HIP kernels on the current stream behind that copy.  ``slots`` pinned
    slots rotate, and a slot is only rewritten after the copy that read it
    has completed; the device coefficient buffer is only overwritten after
    the kernels that read it.
    """

    def __init__(self, batch: int, device, threads: int = 8, slots: int = 2):
        self.B, self.device, self.threads, self.nslots = batch, torch.device(device), threads, slots
        self.geo: Optional[JpegGeometry] = None
        self.slot = 0
        self.stats = {"frames": 0, "host_s": 0.0, "fallback": 0}

    def _configure(self, geo: JpegGeometry) -> None:
        if not geo.gpu_ok:
            raise ValueError(f"JPEG sampling {geo.sampling} not handled on the GPU")
        B, S = self.B, self.nslots
        self.geo = geo
        self.coef = torch.empty((S, B, geo.nblocks, 64), dtype=torch.int16).pin_memory()
        self.q = torch.empty((S, B, 192), dtype=torch.float32).pin_memory()
        self.geoms = torch.zeros((S, B, GEOM_FIELDS), dtype=torch.int32)
        self.status = torch.zeros((S, B), dtype=torch.int32)
        self.fallback: List[dict] = [dict() for _ in range(S)]
        self.copied: List[Optional[torch.cuda.Event]] = [None] * S  # slot's H2D done
        self.coef_dev = torch.empty((B, geo.nblocks, 64), dtype=torch.int16, device=self.device)
        self.q_dev = torch.empty((B, 192), dtype=torch.float32, device=self.device)
        self.planes = torch.empty((B, geo.plane_bytes), dtype=torch.uint8, device=self.device)
        self.geom_rec = np.array([geo.width, geo.height, geo.nc, geo.hmax, geo.vmax, geo.mcux, geo.mcuy,
                                  *[v for hv in geo.sampling for v in hv], geo.nblocks, 0, 0], np.int32)
        self.rgb_host = torch.empty((B, geo.height, geo.width, 3), dtype=torch.uint8).pin_memory()
        self.uploaded = torch.cuda.Event()
        self.consumed = torch.cuda.Event()  # kernels done reading coef_dev / q_dev
        self.consumed.record()
        self.pending: Optional[int] = None  # slot whose upload reconstruct() consumes next

    def stage(self, jpegs: Sequence[bytes]) -> int:
        """Entropy-decode one batch into the next pinned slot; returns the slot."""
        if len(jpegs) != self.B:
            raise ValueError(f"expected {self.B} frames, got {len(jpegs)}")
        if self.geo is None:
            self._configure(probe(jpegs[0]))
        k = self.slot
        self.slot = (k + 1) % self.nslots
        if self.copied[k] is not None:
            self.copied[k].synchronize()  # the previous H2D out of this slot is done
        t0 = time.perf_counter()
        n = self.B
        ptrs = (ctypes.c_char_p * n)(*jpegs)
        lens = (ctypes.c_int64 * n)(*[len(j) for j in jpegs])
        failed = _rt().tca_jpeg_decode_batch(ptrs, lens, n, self.coef[k].data_ptr(), self.geo.nblocks,
                                             self.q[k].data_ptr(), self.geoms[k].data_ptr(), self.status[k].data_ptr(),
                                             self.threads)
        fb = {}
        ref = torch.from_numpy(self.geom_rec)
        for i in range(n):
            if (failed and int(self.status[k, i])) or not torch.equal(self.geoms[k, i], ref):
                rgb = decode_pil(jpegs[i])
                if rgb.shape != (self.geo.height, self.geo.width, 3):
                    raise ValueError(f"frame {i}: {rgb.shape[1]}x{rgb.shape[0]} differs from the batch's "
                                     f"{self.geo.width}x{self.geo.height}")
                fb[i] = rgb
        self.fallback[k] = fb
        self.stats["host_s"] += time.perf_counter() - t0
        self.stats["frames"] += n
        self.stats["fallback"] += len(fb)
        return k

    def upload(self, k: int, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Queue slot k's H2D on ``stream`` (default: current) behind the
        kernels that last read the device buffers."""
        s = stream or torch.cuda.current_stream()
        s.wait_event(self.consumed)
        with torch.cuda.stream(s):
            self.coef_dev.copy_(self.coef[k], non_blocking=True)
            self.q_dev.copy_(self.q[k], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s)
        self.copied[k] = ev
        self.uploaded = ev
        self.pending = k

    def reconstruct(self, out: torch.Tensor) -> torch.Tensor:
        """IDCT + colour kernels of the last uploaded slot into ``out``
        [B, H, W, 3] uint8 (device), on the current stream."""
        g, k = self.geo, self.pending
        if k is None:
            raise RuntimeError("reconstruct() without a staged + uploaded batch")
        if out.shape != (self.B, g.height, g.width, 3) or out.dtype != torch.uint8 or not out.is_contiguous():
            raise ValueError(f"out must be uint8 [{self.B}, {g.height}, {g.width}, 3], got {tuple(out.shape)}")
        cur = torch.cuda.current_stream()
        cur.wait_event(self.uploaded)
        st = _native.stream_ptr(cur)
        geom = self.geom_rec.ctypes.data
        _native.call("tca_jpeg_idct", self.coef_dev.data_ptr(), self.q_dev.data_ptr(), self.planes.data_ptr(), geom,
                     g.nblocks, g.plane_bytes, self.B, st)
        self.consumed = torch.cuda.Event()
        self.consumed.record(cur)
        _native.call("tca_jpeg_color", self.planes.data_ptr(), out.data_ptr(), geom, g.plane_bytes,
                     g.height * g.width * 3, self.B, st)
        fb = self.fallback[k]
        for i, rgb in fb.items():
            self.rgb_host[i].copy_(torch.from_numpy(rgb))
            out[i].copy_(self.rgb_host[i], non_blocking=True)
        if fb:
            torch.cuda.current_stream().synchronize()  # rgb_host is rewritten by the next batch
        self.pending = None
        return out

    def decode(self, jpegs: Sequence[bytes], out: torch.Tensor) -> torch.Tensor:
        """Synchronous convenience: stage + upload + reconstruct."""
        self.upload(self.stage(jpegs))
        return self.reconstruct(out)

    def host_us_per_frame(self) -> float:
        return 1e6 * self.stats["host_s"] / max(1, self.stats["frames"])
