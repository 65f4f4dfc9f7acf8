"""LiDAR per-frame ops: PointCloud2 unpack (K6), voxelisation (K7), fused
PillarVFE + BEV scatter (K8/K9), anchor decode (K11) + rotated-IoU NMS (K10).

GPU tensors run the HIP kernels (``csrc/kernels/{pointcloud,voxelize,pillars,
anchors,nms}.hip``); CPU tensors run vectorised NumPy with identical
semantics (tested against ``golden``).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from ..config.lidar import PointPillarsConfig, VoxelConfig, anchor_grid
from . import golden
from ._ws import Workspace, dtype_code, layout_of
from .nms import Candidates, NmsResult, SORT_CAP, sort_and_nms, sort_and_nms_cpu

INT_MAX = 0x7FFFFFFF

# sensor_msgs/PointField datatype codes
PF_INT8, PF_UINT8, PF_INT16, PF_UINT16, PF_INT32, PF_UINT32, PF_FLOAT32, PF_FLOAT64 = range(1, 9)
PF_NP = {1: np.int8, 2: np.uint8, 3: np.int16, 4: np.uint16, 5: np.int32, 6: np.uint32, 7: np.float32, 8: np.float64}


def _carr(ctype, vals):
    return (ctype * len(vals))(*vals)


# ----------------------------------------------------------------------------- K6
@dataclass
class PointLayout:
    point_step: int
    offsets: Tuple[int, int, int, int]  # x, y, z, intensity
    dtypes: Tuple[int, int, int, int]

    @staticmethod
    def xyzi_f32(point_step: int = 16) -> "PointLayout":
        return PointLayout(point_step, (0, 4, 8, 12), (PF_FLOAT32,) * 4)


def pc2_unpack(ws: Optional[Workspace], data: torch.Tensor, frame_off: torch.Tensor, frame_n: torch.Tensor,
               layout: PointLayout, max_points: int, normalize_intensity: bool = True, z_offset: float = 0.0,
               out_stride: int = 4, stream=None):
    """data: uint8 bytes of B PointCloud2 payloads; frame_off [B] int64 byte
    offsets, frame_n [B] int32 point counts.  Returns (points [B, max_points,
    out_stride] fp32, count [B] int32).  Semantics of
    ``read_points(skip_nans=True)`` + ``i /= max(i)`` + ``z += z_offset``
    (reference ros_inference3d.py:125-128)."""
    B = frame_n.shape[0]
    if data.device.type == "cuda":
        out = ws.get("pc2_points", (B, max_points, out_stride), torch.float32)
        cnt = ws.get("pc2_count", (B,), torch.int32)
        bpf = _native.kernels().tca_pc2_blocks_per_frame(max_points)
        blk = ws.get("pc2_blocks", (B, bpf), torch.int32)
        imax = ws.get("pc2_imax", (B,), torch.int32)
        _native.call("tca_pc2_unpack", _native.ptr(data), _native.ptr(frame_off), _native.ptr(frame_n), B, max_points,
                     layout.point_step, _carr(ctypes.c_int, layout.offsets), _carr(ctypes.c_int, layout.dtypes),
                     int(normalize_intensity), float(z_offset), _native.ptr(out), out_stride, _native.ptr(cnt),
                     _native.ptr(blk), _native.ptr(imax), _native.stream_ptr(stream))
        return out, cnt
    raw = data.numpy()
    offs, ns = frame_off.numpy(), frame_n.numpy()
    out = np.zeros((B, max_points, out_stride), np.float32)
    cnt = np.zeros((B,), np.int32)
    for b in range(B):
        n = min(int(ns[b]), max_points)
        rec = raw[int(offs[b]):int(offs[b]) + n * layout.point_step].reshape(n, layout.point_step)
        cols = []
        for off, dt in zip(layout.offsets, layout.dtypes):
            w = np.dtype(PF_NP[dt]).itemsize
            cols.append(rec[:, off:off + w].copy().view(PF_NP[dt]).reshape(-1).astype(np.float32))
        p = np.stack(cols, 1)
        p = p[~np.isnan(p).any(1)]
        if normalize_intensity and len(p):
            m = p[:, 3].max()
            if m > 0 and np.isfinite(m):
                p[:, 3] = p[:, 3] * np.float32(1.0 / m)
        p[:, 2] += np.float32(z_offset)
        out[b, :len(p), :4] = p
        cnt[b] = len(p)
    return torch.from_numpy(out), torch.from_numpy(cnt)


# ----------------------------------------------------------------------------- K7
def voxelize_np(points: np.ndarray, cfg: VoxelConfig, nfeat: Optional[int] = None):
    """Vectorised spconv-semantics voxeliser (one frame). Returns
    voxels [V, P, F], coords [V, 3] (z, y, x), num_points [V], plus per-voxel
    sorted point indices [V, P] (-1 padded)."""
    F = nfeat or points.shape[1]
    r = np.asarray(cfg.point_cloud_range, np.float32)
    vs = np.asarray(cfg.voxel_size, np.float32)
    nx, ny, nz = cfg.grid_size
    P, V = cfg.max_points_per_voxel, cfg.max_voxels
    c = np.floor((points[:, :3] - r[:3]) / vs).astype(np.int64)
    ok = (c >= 0).all(1) & (c[:, 0] < nx) & (c[:, 1] < ny) & (c[:, 2] < nz)
    pidx = np.nonzero(ok)[0]
    cell = (c[pidx, 2] * ny + c[pidx, 1]) * nx + c[pidx, 0]
    uniq, first, inv = np.unique(cell, return_index=True, return_inverse=True)
    rank_of_uniq = np.empty(len(uniq), np.int64)
    rank_of_uniq[np.argsort(first, kind="stable")] = np.arange(len(uniq))
    vid = rank_of_uniq[inv]
    nvox = min(len(uniq), V)
    keep = vid < nvox
    pidx, vid = pidx[keep], vid[keep]
    order = np.argsort(vid, kind="stable")  # stable → point order within voxel
    vid_s, pidx_s = vid[order], pidx[order]
    starts = np.searchsorted(vid_s, np.arange(nvox))
    rank = np.arange(len(vid_s)) - starts[vid_s]
    sel = rank < P
    voxels = np.zeros((nvox, P, F), np.float32)
    slots = np.full((nvox, P), -1, np.int64)
    voxels[vid_s[sel], rank[sel]] = points[pidx_s[sel], :F]
    slots[vid_s[sel], rank[sel]] = pidx_s[sel]
    num = np.bincount(vid_s, minlength=nvox)[:nvox]
    num = np.minimum(num, P).astype(np.int32)
    ucell = np.empty(nvox, np.int64)
    ucell[rank_of_uniq[rank_of_uniq < nvox]] = uniq[rank_of_uniq < nvox]
    coords = np.stack([ucell // (nx * ny), (ucell // nx) % ny, ucell % nx], 1).astype(np.int32)
    return voxels, coords, num, slots


# "1" / "0": force the voxeliser's hash-table cell rows on / off (tests); None: by grid size
VOX_HASH_FORCE = None


def voxel_hash_bits(cells: int, max_points: int) -> int:
    """log2 of the voxeliser's per-frame hash table (0: dense cell grid).  Hash when the grid has
    more than 16x as many cells as the table would (2 x max_points, rounded up to a power of 2)."""
    bits = max(10, int(2 * max(1, max_points) - 1).bit_length())
    force = VOX_HASH_FORCE
    if force == "0":
        return 0
    if force == "1" or cells > 16 * (1 << bits):
        return bits
    return 0


class Voxelizer:
    """Batched voxeliser with persistent, self-resetting GPU scratch."""

    def __init__(self, cfg: VoxelConfig, batch: int, max_points: int, device="cuda", nfeat: Optional[int] = None,
                 materialize: bool = True):
        self.cfg, self.B, self.max_points = cfg, batch, max_points
        self.device = torch.device(device)
        self.nfeat = nfeat or cfg.num_point_features
        self.materialize = materialize
        if self.device.type == "cuda":
            self.ws = Workspace(self.device)
            cells = cfg.num_cells
            V, P = cfg.max_voxels, cfg.max_points_per_voxel
            g = self.ws.get
            # cell rows: the dense grid, or (grids much larger than a frame's points: SECOND's 90 M
            # cells, 720 MB per frame dense) a per-frame hash table of >= 2 x max_points slots
            # (voxelize.hip hash_slot; VOX_HASH_FORCE forces it on / off)
            self.hash_bits = voxel_hash_bits(cells, max_points)
            rows = (1 << self.hash_bits) if self.hash_bits else cells
            self.cell_first = g("cell_first", (batch, rows), torch.int32, init=INT_MAX)
            self.cell_vid = g("cell_vid", (batch, rows), torch.int32, init=-1)
            self.keys = g("cell_keys", (batch, rows), torch.int32, init=-1) if self.hash_bits else None
            self.point_cell = g("point_cell", (batch, max_points), torch.int32)
            bpf = _native.kernels().tca_vox_blocks_per_frame(max_points)
            self.block_count = g("block_count", (batch, bpf), torch.int32)
            self.slots = g("slots", (batch, V, P), torch.int32, init=INT_MAX)
            self.vcount = g("vcount", (batch, V), torch.int32, init=0)
            self.voxels = g("voxels", (batch, V, P, self.nfeat), torch.float32, init=0) if materialize else None
            self.coords = g("coords", (batch, V, 4), torch.int32, init=0)
            self.num_points = g("num_points", (batch, V), torch.int32, init=0)
            self.voxel_count = g("voxel_count", (batch,), torch.int32, init=0)
            # stage c as a counting sort (tca_vox_slots_csr) when P <= 64
            self.csr_slots = P <= 64
            if self.csr_slots:
                self.offs = g("offs", (batch, V + 1), torch.int32)
                self.cursor = g("cursor", (batch, V), torch.int32)
                self.csr = g("csr", (batch, max_points), torch.int32)
                self.dense = g("dense", (batch, V), torch.int32)
                self.dense_count = g("dense_count", (batch,), torch.int32)
            self._range = _carr(ctypes.c_float, cfg.point_cloud_range)
            self._vsize = _carr(ctypes.c_float, cfg.voxel_size)
            self._grid = _carr(ctypes.c_int, cfg.grid_size)

    def _launch(self, points, npts, mode, gather, stream):
        if (mode & 1) and self.csr_slots:
            self._launch_raw(points, npts, 1 | 4, False, stream)  # a, b1, b2 only
            P = _native.ptr
            _native.call("tca_vox_slots_csr", P(self.point_cell), self.max_points, P(npts), points.shape[0],
                         self._grid, P(self.cell_vid), self.cfg.max_voxels, self.cfg.max_points_per_voxel,
                         P(self.voxel_count), P(self.vcount), P(self.offs), P(self.cursor), P(self.csr),
                         P(self.dense), P(self.dense_count), P(self.slots), self.hash_bits, _native.stream_ptr(stream))
            mode &= ~1
            if not mode:
                return
        self._launch_raw(points, npts, mode, gather, stream)

    def _launch_raw(self, points, npts, mode, gather, stream):
        cfg = self.cfg
        _native.call("tca_voxelize", _native.ptr(points), points.shape[-1], self.max_points, _native.ptr(npts),
                     points.shape[0], self._range, self._vsize, self._grid, cfg.max_points_per_voxel,
                     cfg.max_voxels, self.nfeat, _native.ptr(self.cell_first), _native.ptr(self.cell_vid),
                     _native.ptr(self.point_cell), _native.ptr(self.block_count), _native.ptr(self.slots),
                     _native.ptr(self.vcount), _native.ptr(self.voxels), _native.ptr(self.coords),
                     _native.ptr(self.num_points), _native.ptr(self.voxel_count), mode, int(gather),
                     _native.ptr(self.keys), self.hash_bits, _native.stream_ptr(stream))

    def assign(self, points: torch.Tensor, npts: torch.Tensor, stream=None) -> None:
        """Stage a-c: voxel ids, coords, sorted slot lists (GPU only)."""
        self._launch(points, npts, 1, False, stream)

    def finish(self, points: torch.Tensor, npts: torch.Tensor, gather: bool, stream=None) -> None:
        """Stage d: (optionally) gather voxels, write num_points, reset scratch."""
        self._launch(points, npts, 2, gather and self.materialize, stream)

    def __call__(self, points: torch.Tensor, npts: torch.Tensor, stream=None):
        """points [B, max_points, F], npts [B] → (voxels [B,V,P,F], coords [B,V,4]
        (b,z,y,x), num_points [B,V], voxel_count [B]).  Rows >= voxel_count are
        stale/padding."""
        if points.device.type == "cuda":
            self._launch(points, npts, 3, True, stream)
            return self.voxels, self.coords, self.num_points, self.voxel_count
        cfg = self.cfg
        B = points.shape[0]
        V, P = cfg.max_voxels, cfg.max_points_per_voxel
        vox = np.zeros((B, V, P, self.nfeat), np.float32)
        co = np.zeros((B, V, 4), np.int32)
        nump = np.zeros((B, V), np.int32)
        vc = np.zeros((B,), np.int32)
        pn = points.numpy()
        for b in range(B):
            v, c, n, _ = voxelize_np(pn[b, :int(npts[b])], cfg, self.nfeat)
            k = len(n)
            vox[b, :k], nump[b, :k], vc[b] = v, n, k
            co[b, :k, 0] = b
            co[b, :k, 1:] = c
        return torch.from_numpy(vox), torch.from_numpy(co), torch.from_numpy(nump), torch.from_numpy(vc)


# ----------------------------------------------------------------------------- K7s
IDENTITY_POSE = (1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0)


def merge_sweeps_np(cur: np.ndarray, history: Sequence[Tuple[np.ndarray, float, np.ndarray]], t_cur: float,
                    pose_cur: np.ndarray) -> np.ndarray:
    """Reference of the multi-sweep merge for one frame: ``cur`` [n, >=4] points of the
    current sweep; ``history`` newest first, (points [m, 4], timestamp, 3x4 pose) of
    earlier sweeps.  Returns [N, 5]: current sweep (lag 0), then each earlier sweep in
    the current sensor frame, inv(T_cur) * T_k, with lag t_cur - t_k (det3d order)."""
    Tc = np.asarray(pose_cur, np.float64).reshape(3, 4)
    out = [np.concatenate([cur[:, :4], np.zeros((len(cur), 1))], 1)]
    for pts, t, pose in history:
        Tk = np.asarray(pose, np.float64).reshape(3, 4)
        q = pts[:, :3].astype(np.float64) @ Tk[:, :3].T + Tk[:, 3] - Tc[:, 3]
        p = q @ Tc[:, :3]
        out.append(np.concatenate([p, pts[:, 3:4], np.full((len(pts), 1), t_cur - t)], 1))
    return np.concatenate(out).astype(np.float32)


class SweepAccumulator:
    """Device ring of the last ``nsweeps - 1`` sweeps per frame slot + the merge into
    one (x, y, z, intensity, time lag) point list per frame (sweeps.hip
    tca_sweep_step): det3d's multi-sweep input for CenterPoint
    (``data/nusc_centerpoint_pp_02voxel_two_pfn_10sweep.py`` ``nsweeps``).  ``clock``
    [B] (seconds) and ``pose`` [B, 12] (3x4 sensor-to-world) are the current sweep's,
    set by the caller before a step or auto-advanced by ``dt`` per step; the whole
    step is capture-safe (the ring position lives on the device)."""

    def __init__(self, nsweeps: int, batch: int, max_points: int, device="cuda", dt: float = 0.05):
        if not 2 <= nsweeps <= 32:
            raise ValueError(f"nsweeps {nsweeps}: 2..32")
        self.S, self.R, self.B, self.maxp, self.dt = nsweeps, nsweeps - 1, batch, max_points, float(dt)
        dev = torch.device(device)
        f = dict(dtype=torch.float32, device=dev)
        self.ring = torch.zeros((self.R, batch, max_points, 4), **f)
        self.ring_n = torch.zeros((self.R, batch), dtype=torch.int32, device=dev)
        # fp64 stamps: message times in epoch seconds (or hours of auto-clock) keep ms-exact lags
        self.ring_t = torch.zeros((self.R, batch), dtype=torch.float64, device=dev)
        self.ring_pose = torch.zeros((self.R, batch, 12), **f)
        self.head = torch.zeros((1,), dtype=torch.int32, device=dev)
        self.clock = torch.zeros((batch,), dtype=torch.float64, device=dev)
        self.pose = torch.tensor(IDENTITY_POSE, **f).repeat(batch, 1).contiguous()
        self.out = torch.zeros((batch, nsweeps * max_points, 5), **f)
        self.out_n = torch.zeros((batch,), dtype=torch.int32, device=dev)

    @property
    def out_points(self) -> int:
        return self.S * self.maxp

    def reset(self) -> None:
        self.ring_n.zero_()
        self.head.zero_()

    def __call__(self, points: torch.Tensor, npts: torch.Tensor, stream=None):
        """points [B, maxp, >=4], npts [B] -> (merged [B, S * maxp, 5], count [B])."""
        assert points.shape[:2] == (self.B, self.maxp) and points.is_contiguous(), points.shape
        P = _native.ptr
        _native.call("tca_sweep_step", P(points), points.shape[-1], P(npts), self.B, self.maxp, self.R, P(self.ring),
                     P(self.ring_n), P(self.ring_t), P(self.ring_pose), P(self.head), P(self.clock), P(self.pose),
                     self.dt, P(self.out), P(self.out_n), _native.stream_ptr(stream))
        return self.out, self.out_n


# ----------------------------------------------------------------------------- K8/K9
class PillarEncoder:
    """Fused PillarVFE (BN folded) + scatter into an NHWC BEV canvas (bf16, or
    fp32 for the fp32 precision mode)."""

    def __init__(self, cfg: VoxelConfig, weight: torch.Tensor, bias: torch.Tensor, batch: int, device="cuda",
                 channels: int = 64, dtype: torch.dtype = torch.bfloat16):
        self.cfg, self.B, self.C = cfg, batch, channels
        assert dtype in (torch.bfloat16, torch.float32), dtype
        self.dtype = dtype
        self._dt = 0 if dtype == torch.float32 else 2
        self.pair = False  # fp32 canvas written as pair storage (ops/conv.py to_pairs)
        self.device = torch.device(device)
        self.W = weight.detach().float().contiguous().to(self.device)  # [64, 10]
        self.b = bias.detach().float().contiguous().to(self.device)
        nx, ny, _ = cfg.grid_size
        self.nx, self.ny = nx, ny
        if self.device.type == "cuda":
            self.ws = Workspace(self.device)
            # NHWC canvas, zero-initialised once; cleared per frame by cell list
            self.canvas = self.ws.get("canvas", (batch, ny, nx, channels), dtype, init=0)
            # pair mode: per-cell occupancy bytes written by the scatter, cleared with the cells;
            # the first BEV conv skips the reads of unoccupied cells (most of the canvas)
            self.occ = None
            # occupancy-gated: every reader of the canvas features skips unoccupied cells (the
            # fast BEV plan's first conv gates its loads on occ), so a frame's clear resets only
            # the occupancy bytes of the previous frame's cells (set_occ_gated)
            self.occ_gated = False
            self._range = _carr(ctypes.c_float, cfg.point_cloud_range)
            self._vsize = _carr(ctypes.c_float, cfg.voxel_size)

    def set_pair(self, pair: bool) -> None:
        """fp32 canvas only: write the scatter in pair storage (what a pair-storage
        BEV plan reads).  Zero bytes are zero in both forms, so the per-frame
        clear-by-cell-list stays valid across a switch."""
        if pair and self.dtype != torch.float32:
            raise ValueError("pair storage needs the fp32 canvas")
        self.pair = bool(pair)
        self._dt = 5 if pair else (0 if self.dtype == torch.float32 else 2)
        if self.pair and self.occ is None and self.device.type == "cuda":
            self.occ = self.ws.get("occ", (self.B, self.ny, self.nx), torch.uint8, init=0)
            # the canvas was written without occupancy until now: mark nothing, the
            # first frame after the switch rewrites its cells (and the canvas was cleared by cells)

    def set_occ_gated(self, gated: bool) -> None:
        """The canvas's only feature reader gates on the occupancy bytes (pair storage with its
        occupancy): clear just those per frame, not the 256 B of features of every old pillar.
        Turning it off zeroes the canvas once (stale features outside the occupied cells)."""
        gated = bool(gated) and self.pair and self.occ is not None
        if self.occ_gated and not gated:
            self.canvas.zero_()
        self.occ_gated = gated

    def canvas_nhwc(self):
        from .conv import NHWC
        return NHWC(self.canvas, pair=self.pair, occ=self.occ if self.pair else None)

    def canvas_nchw(self) -> torch.Tensor:
        """Dense fp32 view for the PyTorch modules (calibration, the non-fused path); with an
        occupancy-gated canvas the unoccupied cells are masked to zero (a copy)."""
        if self.pair:
            from .conv import from_pairs
            c = from_pairs(self.canvas)
        else:
            c = self.canvas
        if self.occ_gated:
            c = c * self.occ[..., None].to(c.dtype)
        return c.permute(0, 3, 1, 2)  # channels_last view

    def clear(self, vox: Voxelizer, stream=None) -> None:
        """Zero the cells written for the voxels currently in ``vox`` (call
        before the voxeliser overwrites its coords with the next frame)."""
        self.clear_coords(vox.coords, vox.voxel_count, stream)

    def clear_coords(self, coords: torch.Tensor, voxel_count: torch.Tensor, stream=None) -> None:
        """coords [B, V, 4] (b, z, y, x), voxel_count [B]."""
        args = (_native.ptr(coords), _native.ptr(voxel_count), coords.shape[0], coords.shape[1], self.nx, self.ny,
                self.C, _native.ptr(self.canvas), self._dt)
        if self.occ is not None and self.occ_gated:
            _native.call("tca_pillar_occ_clear", _native.ptr(coords), _native.ptr(voxel_count), coords.shape[0],
                         coords.shape[1], self.nx, self.ny, _native.ptr(self.occ), _native.stream_ptr(stream))
        elif self.occ is not None:
            _native.call("tca_pillar_canvas_clear_occ", *args, _native.ptr(self.occ), _native.stream_ptr(stream))
        else:
            _native.call("tca_pillar_canvas_clear", *args, _native.stream_ptr(stream))

    def encode_from_slots(self, points: torch.Tensor, vox: Voxelizer, feat_out: Optional[torch.Tensor] = None,
                          stream=None) -> torch.Tensor:
        args = (_native.ptr(points), points.shape[-1], vox.max_points, _native.ptr(vox.slots), _native.ptr(vox.vcount),
                _native.ptr(vox.coords), _native.ptr(vox.voxel_count), self.B, self.cfg.max_voxels,
                self.cfg.max_points_per_voxel, _native.ptr(self.W), _native.ptr(self.b), self._range, self._vsize,
                self.nx, self.ny, _native.ptr(self.canvas), _native.ptr(feat_out), self._dt)
        if self.occ is not None:
            _native.call("tca_pillar_vfe_slots_occ", *args, _native.ptr(self.occ), _native.stream_ptr(stream))
        else:
            _native.call("tca_pillar_vfe_slots", *args, _native.stream_ptr(stream))
        # pair storage: the plan reads the raw buffer; decoding it here would cost a full pass
        return None if self.pair else self.canvas_nchw()

    def encode_from_voxels(self, voxels, num_points, coords, voxel_count, feat_out=None, stream=None):
        """voxels [B, V, P, 4], num_points [B, V], coords [B, V, 4], voxel_count [B]."""
        args = (_native.ptr(voxels), _native.ptr(num_points), _native.ptr(coords), _native.ptr(voxel_count),
                voxels.shape[0], voxels.shape[1], voxels.shape[2], _native.ptr(self.W), _native.ptr(self.b),
                self._range, self._vsize, self.nx, self.ny, _native.ptr(self.canvas), _native.ptr(feat_out), self._dt)
        if self.occ is not None:
            _native.call("tca_pillar_vfe_voxels_occ", *args, _native.ptr(self.occ), _native.stream_ptr(stream))
        else:
            _native.call("tca_pillar_vfe_voxels", *args, _native.stream_ptr(stream))
        # pair storage: the plan reads the raw buffer; decoding it here would cost a full pass
        return None if self.pair else self.canvas_nchw()


def pillar_features_reference(voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor,
                              cfg: VoxelConfig, W: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """fp32 PyTorch reference of the fused kernel's per-pillar output."""
    from ..models.pointpillars import pillar_point_features
    f = pillar_point_features(voxels.float(), num_points, coords, cfg)
    return torch.relu(f @ W.t().float() + b.float()).max(dim=1).values


# ----------------------------------------------------------------------------- K11 + K10
class AnchorPostprocess:
    """PointPillars head → boxes: decode + score filter + top-k + rotated NMS."""

    def __init__(self, cfg: PointPillarsConfig, batch: int, device="cuda"):
        self.cfg, self.B = cfg, batch
        self.device = torch.device(device)
        x0, xs, y0, ys, table = anchor_grid(cfg)
        self.x0, self.xs, self.y0, self.ys = x0, xs, y0, ys
        self.table = np.asarray(table, np.float32)  # [A, 6]
        self._table = _carr(ctypes.c_float, self.table.flatten().tolist())
        self.H, self.W = cfg.feature_map_size
        self.A = cfg.num_anchors_per_loc
        self.C = cfg.num_classes
        self.cap = min(self.H * self.W * self.A, 1 << 20)
        # exact top-k preselection (tca_anchor_topk_threshold) when every anchor would
        # pass the score filter and only pre_max of them reach the NMS
        self.topk_select = cfg.score_thresh <= 0.0 and cfg.nms_pre_max < self.H * self.W * self.A
        if self.device.type == "cuda":
            self.ws = Workspace(self.device)

    def __call__(self, cls, box, dir_, stream=None) -> NmsResult:
        """cls/box/dir: [B, C, H, W] tensors (NCHW or channels_last) or NHWC
        channel-slice views of one merged head output."""
        from .conv import NHWC
        if isinstance(cls, NHWC):
            if cls.t.device.type != "cuda":
                return self.cpu(cls.nchw(), box.nchw(), dir_.nchw())
            es = cls.t.element_size()
            pc, pb, pd = (_native.ptr(v.t) + v.off * es for v in (cls, box, dir_))
            lds = (cls.t.shape[-1], box.t.shape[-1], dir_.t.shape[-1])
            lay, dt, B = 1, dtype_code(cls.t), cls.t.shape[0]
        else:
            if cls.device.type != "cuda":
                return self.cpu(cls, box, dir_)
            lay, c = layout_of(cls)
            b_ = layout_of(box)[1]
            d_ = layout_of(dir_)[1]
            if layout_of(box)[0] != lay or layout_of(dir_)[0] != lay:
                c, b_, d_, lay = cls.contiguous(), box.contiguous(), dir_.contiguous(), 0
            pc, pb, pd = _native.ptr(c), _native.ptr(b_), _native.ptr(d_)
            lds = (0, 0, 0)
            dt, B = dtype_code(c), c.shape[0]
        cfg = self.cfg
        s = _native.stream_ptr(stream)
        if self.topk_select:
            # no score threshold and pre_max << anchors (SECONDHead proposals): find each
            # frame's exact top-k key threshold first, decode only those anchors
            hist = self.ws.get("anc_hist", (B, 4096), torch.int32, init=0)
            sel = self.ws.get("anc_sel", (B, 2), torch.int32)
            _native.call("tca_anchor_topk_threshold", pc, dt, lay, B, self.H, self.W, self.A, self.C, lds[0],
                         int(cfg.nms_pre_max), _native.ptr(hist), _native.ptr(sel), s)
            cand = Candidates.alloc(self.ws, "anc_", B, self.cap, 7)
            _native.call("tca_anchor_decode_filter_keyed", pc, pb, pd, dt, lay,
                         B, self.H, self.W, self.A, self.C, cfg.num_dir_bins, *lds, self._table, float(self.x0),
                         float(self.xs), float(self.y0), float(self.ys), float(cfg.dir_offset),
                         float(cfg.dir_limit_offset), _native.ptr(sel), _native.ptr(cand.box),
                         _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key),
                         _native.ptr(cand.count), self.cap, s)
            return sort_and_nms(self.ws, cand, 1, cfg.nms_thresh, cfg.nms_pre_max, cfg.nms_post_max, True, None,
                                prefix="anc_nms_", stream=stream)
        cand = Candidates.alloc(self.ws, "anc_", B, self.cap, 7)
        _native.call("tca_anchor_decode_filter", pc, pb, pd, dt, lay,
                     B, self.H, self.W, self.A, self.C, cfg.num_dir_bins, *lds, self._table, float(self.x0),
                     float(self.xs), float(self.y0), float(self.ys), float(cfg.dir_offset),
                     float(cfg.dir_limit_offset), float(cfg.score_thresh), _native.ptr(cand.box),
                     _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key), _native.ptr(cand.count),
                     self.cap, s)
        return sort_and_nms(self.ws, cand, 1, cfg.nms_thresh, cfg.nms_pre_max, cfg.nms_post_max, True, None,
                            prefix="anc_nms_", stream=stream)

    def decode_cpu(self, cls, box, dir_):
        """Reference decode (OpenPCDet semantics) → (boxes [B, N, 7], scores, labels)."""
        cfg = self.cfg
        B = cls.shape[0]
        H, W, A, C = self.H, self.W, self.A, self.C
        cl = cls.float().permute(0, 2, 3, 1).reshape(B, H * W * A, C)
        bx = box.float().permute(0, 2, 3, 1).reshape(B, H * W * A, 7)
        dr = dir_.float().permute(0, 2, 3, 1).reshape(B, H * W * A, cfg.num_dir_bins)
        t = torch.from_numpy(self.table)
        ys_, xs_ = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
        xa = (self.x0 + xs_.float() * self.xs).reshape(-1, 1).expand(-1, A).reshape(-1)
        ya = (self.y0 + ys_.float() * self.ys).reshape(-1, 1).expand(-1, A).reshape(-1)
        tt = t.repeat(H * W, 1)
        dxa, dya, dza, za, ra, diag = tt.unbind(1)
        out = torch.stack([bx[..., 0] * diag + xa, bx[..., 1] * diag + ya, bx[..., 2] * dza + za,
                           torch.exp(bx[..., 3]) * dxa, torch.exp(bx[..., 4]) * dya, torch.exp(bx[..., 5]) * dza,
                           bx[..., 6] + ra], -1)
        period = 2 * np.pi / cfg.num_dir_bins
        dl = dr.argmax(-1).float()
        val = out[..., 6] - cfg.dir_offset
        lim = val - torch.floor(val / period + cfg.dir_limit_offset) * period
        out[..., 6] = lim + cfg.dir_offset + period * dl
        score, lab = torch.sigmoid(cl).max(-1)
        return out, score, lab.int() + 1

    def cpu(self, cls, box, dir_) -> NmsResult:
        cfg = self.cfg
        boxes, scores, labels = self.decode_cpu(cls, box, dir_)
        B = boxes.shape[0]
        mo = cfg.nms_post_max
        ob = np.zeros((B, mo, 7), np.float32)
        os_ = np.zeros((B, mo), np.float32)
        oc = np.zeros((B, mo), np.int32)
        cnt = np.zeros((B,), np.int32)
        for b in range(B):
            s = scores[b].numpy()
            idx = np.nonzero(s >= cfg.score_thresh)[0]
            keep = sort_and_nms_cpu(boxes[b].numpy()[idx], s[idx], labels[b].numpy()[idx], idx, 1, cfg.nms_thresh,
                                    cfg.nms_pre_max, mo, True)
            k = idx[keep]
            n = len(k)
            ob[b, :n], os_[b, :n], oc[b, :n], cnt[b] = boxes[b].numpy()[k], s[k], labels[b].numpy()[k], n
        return NmsResult(torch.from_numpy(ob), torch.from_numpy(os_), torch.from_numpy(oc), torch.from_numpy(cnt))
