"""SECOND-IoU on MI355X: sparse 3D backbone (VoxelBackBone8x +
HeightCompression) and the SECONDHead RoI stage over ``csrc/kernels/spconv.hip``.

:class:`SparseBackbone` owns every level's static buffers (row features,
coords, dense site→row grid, neighbour tables, tap masks, device row counts)
sized for worst-case capacities — a stride-2 3x3x3 layer reaches at most 8
output sites per input site, and no level holds more sites than its grid — so
rows never drop and every launch has a static shape (hipGraph capturable).
Per step:

    reset    BEV map cleared / grids reset from the previous step's coord lists
    level 0  MeanVFE from the voxeliser's slot lists (or from received voxels)
             → feats [N0, 8] bf16, coords, grid
    layer    SparseConv3d: claim output sites → neighbour table; SubMConv3d:
             the level's shared neighbour table (built once) → gather-GEMM
    last     conv_out's epilogue scatters into the NHWC BEV map [B, ny, nx, 256]
             at channel z*128 + c (``models.second.bev_channel_permutation``)

:class:`RoIHead` pools 7x7 grids from the 512-channel BEV features for every
proposal (``tca_roi_grid_pool``), runs the BN-folded FC stack as plain
hipBLASLt GEMMs (bf16, fp32 accumulation) and turns sigmoid(IoU) into the
candidates of the final rotated NMS (``tca_roi_rescore`` → K10).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from .. import _native
from ..config.lidar import SecondIoUConfig, SparseConvSpec
from ._ws import Workspace
from .conv import split_pairs
from .nms import Candidates, NmsResult, sort_and_nms


def _iarr(vals) -> ctypes.Array:
    return (ctypes.c_int * len(vals))(*[int(v) for v in vals])


def _ceil(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class _Level:
    shape: tuple          # (Z, Y, X)
    cap: int
    coords: torch.Tensor  # [cap, 4] int32 (b, z, y, x)
    grid: torch.Tensor    # [B*Z*Y*X] int32, -1 = inactive
    count_idx: int
    dims: ctypes.Array
    subm_nbr: Optional[torch.Tensor] = None
    subm_mask: Optional[torch.Tensor] = None
    bufs: Optional[List[torch.Tensor]] = None


@dataclass
class _Layer:
    spec: SparseConvSpec
    level: int
    cin_p: int
    w: torch.Tensor       # [N, Kp] bf16
    b: torch.Tensor       # [N] fp32
    kp: int
    ksp: ctypes.Array
    nbr: Optional[torch.Tensor] = None   # down layers: own table
    mask: Optional[torch.Tensor] = None
    out: Optional[torch.Tensor] = None   # None → BEV scatter
    inp: Optional[torch.Tensor] = None


def _pow2_at_least(c: int, lo: int = 8) -> int:
    p = lo
    while p < c:
        p *= 2
    return p


class SparseBackbone:
    """GPU executor of MeanVFE + VoxelBackBone8x + HeightCompression."""

    def __init__(self, cfg: SecondIoUConfig, layers, batch: int, device="cuda", max_rows0: Optional[int] = None,
                 precision: str = "bf16"):
        """layers: the BN-folded :class:`~..models.second.SparseConv3d` modules.
        precision "fp32": fp32 rows / BEV map, weights as {hi | lo} bf16 pairs,
        split-product gather GEMMs (tca_sp_gemm_x3)."""
        self.cfg, self.B = cfg, batch
        self.f32 = precision == "fp32"
        fdt = torch.float32 if self.f32 else torch.bfloat16
        sfx = "_f32" if self.f32 else ""
        self._k_vfe_slots, self._k_vfe_voxels = "tca_sp_vfe_slots" + sfx, "tca_sp_vfe_voxels" + sfx
        self._k_bev_clear, self._k_gemm = "tca_sp_bev_clear" + sfx, "tca_sp_gemm_x3" if self.f32 else "tca_sp_gemm"
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("SparseBackbone runs on the GPU; models.second is the CPU path")
        self.ws = ws = Workspace(self.device)
        shapes = cfg.level_shapes()
        specs = list(cfg.sparse)
        nlev = 1 + sum(1 for s in specs if not s.subm)
        self.counts = ws.get("sp_counts", (nlev,), torch.int32, init=0)
        self.off = ws.get("sp_off", (batch,), torch.int32, init=0)
        cap0 = max_rows0 or batch * cfg.voxel.max_voxels
        self.levels: List[_Level] = []
        self.levels.append(self._new_level(0, shapes[0], cap0))
        self.feats0 = ws.get("sp_feats0", (cap0, 8), fdt, init=0)
        C, D = specs[-1].cout, shapes[-1][0]
        _, Hb, Wb = cfg.bev_shape
        self.bev_c = C * D
        self.bev = ws.get("sp_bev", (batch, Hb, Wb, self.bev_c), fdt, init=0)
        self.layers: List[_Layer] = []
        cur = 0
        x = self.feats0
        for i, (spec, mod) in enumerate(zip(specs, layers)):
            if not spec.subm:
                prev = self.levels[cur]
                mult = 1
                for d in range(3):
                    mult *= math.ceil(spec.kernel[d] / spec.stride[d])
                Z, Y, X = shapes[i + 1]
                cap = min(batch * Z * Y * X, prev.cap * mult)
                cur = len(self.levels)
                self.levels.append(self._new_level(cur, shapes[i + 1], cap))
            lev = self.levels[cur]
            cin_p = _pow2_at_least(spec.cin)
            w = mod.weight.detach().float()  # [Cout, KZ, KY, KX, Cin]
            T = spec.taps
            wk = torch.zeros(spec.cout, T, cin_p)
            wk[:, :, :spec.cin] = w.reshape(spec.cout, T, spec.cin)
            K = T * cin_p
            kp = _ceil(K, 32)
            W = torch.zeros(spec.cout, kp)
            W[:, :K] = wk.reshape(spec.cout, K)
            bias = mod.bias.detach().float() if mod.bias is not None else torch.zeros(spec.cout)
            ksp = _iarr(list(spec.kernel) + list(spec.stride) + list(spec.padding))
            Wd = split_pairs(W).to(self.device) if self.f32 else W.to(self.device, torch.bfloat16).contiguous()
            L = _Layer(spec, cur, cin_p, Wd,
                       bias.to(self.device).contiguous(), kp, ksp)
            if spec.subm:
                if lev.subm_nbr is None:
                    lev.subm_nbr = ws.get(f"sp_nbr_s{cur}", (_ceil(lev.cap, 64), 27), torch.int32)
                    lev.subm_mask = ws.get(f"sp_mask_s{cur}", ((lev.cap + 63) // 64,), torch.int32)
                L.nbr, L.mask = lev.subm_nbr, lev.subm_mask
            else:
                L.nbr = ws.get(f"sp_nbr_d{i}", (_ceil(lev.cap, 64), T), torch.int32)
                L.mask = ws.get(f"sp_mask_d{i}", ((lev.cap + 63) // 64,), torch.int32)
            assert x.shape[1] == cin_p, (i, x.shape, cin_p)
            L.inp = x
            if i == len(specs) - 1:
                L.out = None
            else:
                if lev.bufs is None or lev.bufs[0].shape[1] != spec.cout:
                    lev.bufs = [ws.get(f"sp_f{cur}_{spec.cout}_{k}", (lev.cap, spec.cout), fdt)
                                for k in range(2)]
                L.out = lev.bufs[0] if L.inp is not lev.bufs[0] else lev.bufs[1]
                x = L.out
            self.layers.append(L)
        self.subm_ksp = _iarr([3, 3, 3, 1, 1, 1, 1, 1, 1])
        self._bev_hw = (Hb, Wb)

    def _new_level(self, idx: int, shape, cap: int) -> _Level:
        Z, Y, X = shape
        g = self.ws.get(f"sp_grid{idx}", (self.B * Z * Y * X,), torch.int32, init=-1)
        co = self.ws.get(f"sp_coords{idx}", (cap, 4), torch.int32, init=0)
        return _Level(tuple(shape), cap, co, g, idx, _iarr(shape))

    # ------------------------------------------------------------------ helpers
    def _cnt(self, lev: _Level) -> int:
        return _native.ptr(self.counts) + 4 * lev.count_idx

    @property
    def nbytes(self) -> int:
        return self.ws.nbytes()

    def bev_nhwc(self) -> torch.Tensor:
        return self.bev

    def reset(self, stream=None) -> None:
        """Undo the previous step (its coord lists are still intact): clear the
        BEV cells conv_out wrote, reset every grid, zero the row counts."""
        s = _native.stream_ptr(stream)
        P = _native.ptr
        last = self.levels[-1]
        Hb, Wb = self._bev_hw
        _native.call(self._k_bev_clear, P(last.coords), self._cnt(last), last.cap, self.layers[-1].spec.cout,
                     P(self.bev), Hb, Wb, self.bev_c, s)
        for lev in self.levels:
            _native.call("tca_sp_grid_reset", P(lev.coords), self._cnt(lev), lev.cap, lev.dims, P(lev.grid), s)
        _native.call("tca_zero_i32", P(self.counts), self.counts.numel(), s)

    def encode_from_slots(self, points: torch.Tensor, vox, stream=None) -> None:
        """Level 0 from the voxeliser (after ``vox.assign``, before ``vox.finish``)."""
        s = _native.stream_ptr(stream)
        P = _native.ptr
        l0 = self.levels[0]
        v = self.cfg.voxel
        _native.call("tca_sp_offsets", P(vox.voxel_count), self.B, P(self.off), self._cnt(l0), s)
        _native.call(self._k_vfe_slots, P(points), points.shape[-1], vox.max_points, P(vox.slots), P(vox.vcount),
                     v.max_points_per_voxel, P(vox.coords), P(vox.voxel_count), self.B, v.max_voxels, P(self.off),
                     l0.dims, P(self.feats0), P(l0.coords), P(l0.grid), s)

    def encode_from_voxels(self, voxels: torch.Tensor, num_points: torch.Tensor, coords: torch.Tensor,
                           n: torch.Tensor, stream=None) -> None:
        """Level 0 from materialised voxels [cap, P, F], num_points [cap],
        coords [cap, 4] (b, z, y, x) and a device count n [1] (served path)."""
        s = _native.stream_ptr(stream)
        P = _native.ptr
        l0 = self.levels[0]
        self.counts[0:1].copy_(n)
        _native.call(self._k_vfe_voxels, P(voxels), voxels.shape[0], voxels.shape[1], voxels.shape[2],
                     P(num_points), P(coords), P(n), l0.dims, P(self.feats0), P(l0.coords), P(l0.grid), s)

    def forward(self, stream=None) -> torch.Tensor:
        """Run the sparse layers; returns the NHWC BEV map."""
        s = _native.stream_ptr(stream)
        P = _native.ptr
        built = set()
        Hb, Wb = self._bev_hw
        for i, L in enumerate(self.layers):
            lev = self.levels[L.level]
            if not L.spec.subm:
                prev = self.levels[L.level - 1]
                _native.call("tca_sp_claim", P(prev.coords), self._cnt(prev), prev.cap, L.ksp, lev.dims, P(lev.grid),
                             P(lev.coords), self._cnt(lev), lev.cap, s)
                _native.call("tca_sp_rulebook", P(lev.coords), self._cnt(lev), lev.cap, L.ksp, prev.dims, P(prev.grid),
                             P(L.nbr), P(L.mask), s)
            elif L.level not in built:
                _native.call("tca_sp_rulebook", P(lev.coords), self._cnt(lev), lev.cap, self.subm_ksp, lev.dims,
                             P(lev.grid), P(L.nbr), P(L.mask), s)
                built.add(L.level)
            last = L.out is None
            _native.call(self._k_gemm, P(L.inp), L.cin_p, P(L.nbr), L.spec.taps, P(L.mask), P(L.w), P(L.b),
                         L.spec.cout, L.kp, self._cnt(lev), lev.cap, P(L.out), P(lev.coords),
                         P(self.bev) if last else 0, Hb, Wb, self.bev_c, 1, s)
        return self.bev

    def level_rows(self) -> List[int]:
        """Host copy of the per-level row counts (diagnostics; syncs)."""
        return [int(v) for v in self.counts.cpu()]


class RoIHead:
    """SECONDHead on the GPU: RoI grid pool (HIP) → BN-folded FC stack
    (hipBLASLt) → sigmoid(IoU) rescoring (HIP) → rotated NMS (K10)."""

    def __init__(self, cfg: SecondIoUConfig, head, batch: int, feat_channels: int, device="cuda",
                 precision: str = "bf16"):
        self.cfg, self.B = cfg, batch
        self.f32 = precision == "fp32"
        adt = torch.float32 if self.f32 else torch.bfloat16
        self.device = torch.device(device)
        self.R, self.G, self.C = cfg.proposal_post_max, cfg.roi_grid, feat_channels
        lin = head.folded_linears()
        G, C = self.G, self.C
        w0, b0, r0 = lin[0]
        # OpenPCDet flattens pooled [N, C, G, G] as (c, gy, gx); the kernel writes (gy, gx, c)
        w0 = w0.view(w0.shape[0], C, G, G).permute(0, 2, 3, 1).reshape(w0.shape[0], -1)
        lin = [(w0, b0, r0)] + lin[1:]
        self.mid = [(w.t().contiguous().to(self.device, adt), b.to(self.device, adt), r)
                    for w, b, r in lin[:-1]]
        wl, bl, _ = lin[-1]
        self.w_last = wl.t().contiguous().to(self.device, torch.float32)  # [256, 1]
        self.b_last = bl.to(self.device, torch.float32)
        self.ws = Workspace(self.device)
        N = batch * self.R
        self.pooled = self.ws.get("roi_pooled", (N, G * G * C), adt, init=0)
        self.acts = [self.ws.get(f"roi_act{i}", (N, w.shape[1]), adt) for i, (w, _, _) in
                     enumerate(self.mid)]
        self.logit = self.ws.get("roi_logit", (N, 1), torch.float32)
        v = cfg.voxel
        ds = cfg.feature_map_stride
        self.geom = (float(v.point_cloud_range[0]), float(v.point_cloud_range[1]), float(v.voxel_size[0] * ds),
                     float(v.voxel_size[1] * ds))

    @torch.no_grad()
    def iou_logits(self, feat: torch.Tensor, props: NmsResult, coff: int = 0, stream=None) -> torch.Tensor:
        """feat: NHWC [B, H, W, ldc] bf16 (channels [coff, coff + C)); props:
        the proposal NMS result (box [B, R, 7], cls, count).  → [B*R, 1] fp32."""
        B, H, W, ldc = feat.shape
        assert props.box.shape[1] == self.R and B == self.B
        _native.call("tca_roi_grid_pool_f32" if self.f32 else "tca_roi_grid_pool", _native.ptr(feat), B, H, W, self.C, ldc, coff, _native.ptr(props.box),
                     props.box.shape[2], _native.ptr(props.count), self.R, *self.geom, self.G,
                     _native.ptr(self.pooled), _native.stream_ptr(stream))
        x = self.pooled
        for (w, b, relu), out in zip(self.mid, self.acts):
            torch.addmm(b, x, w, out=out)
            if relu:
                out.relu_()
            x = out
        torch.addmm(self.b_last, x.float(), self.w_last, out=self.logit)
        return self.logit

    @torch.no_grad()
    def __call__(self, feat: torch.Tensor, props: NmsResult, coff: int = 0, stream=None) -> NmsResult:
        logit = self.iou_logits(feat, props, coff, stream)
        cfg = self.cfg
        cand = Candidates.alloc(self.ws, "roi_cand_", self.B, self.R, props.box.shape[2])
        _native.call("tca_roi_rescore", _native.ptr(logit), _native.ptr(props.box), props.box.shape[2],
                     _native.ptr(props.cls), _native.ptr(props.count), self.B, self.R, float(cfg.score_thresh),
                     _native.ptr(cand.box), _native.ptr(cand.score), _native.ptr(cand.cls), _native.ptr(cand.key),
                     _native.ptr(cand.count), _native.stream_ptr(stream))
        return sort_and_nms(self.ws, cand, 1, cfg.nms_thresh, cfg.nms_pre_max, cfg.nms_post_max, True, None,
                            prefix="roi_nms_", stream=stream)
