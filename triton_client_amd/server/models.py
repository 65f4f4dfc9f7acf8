"""Servable detectors with the reference's Triton tensor contracts.

* :class:`YoloV5Model` — ``YOLOv5nCROP`` / ``weed_detector`` (512, 2 classes,
  ``examples/YOLOv5/config.pbtxt``) and ``YOLOv5nCOCO`` (640, 80 classes,
  ``.vscode/launch.json:12``): input ``images`` FP32 NCHW [3,H,W] (reshape
  [1,3,H,W]), output ``output`` FP32 [1, N, 5+nc] decoded rows — what the
  reference's ONNX export returns.  On MI355X: fp32 (split-product MFMA) captured
  batch plans + the HIP decode kernel writing the decoded tensor.
* :class:`SecondIoUModel` — ``second_iou`` (sparse 3D conv backbone + RoI IoU head).
* :class:`DetectronModel` — ``test_model`` (RetinaNet, ``examples/RetinaNet_detectron/config.pbtxt``)
  and the FCOS / RetinaNet Detectron2 names, fp32 like the reference's libtorch model.
* :class:`PointPillarsModel` — ``pointpillar_kitti``
  (``examples/pointpillar_kitti/config.pbtxt``): inputs ``voxels`` [-1,P,4],
  ``voxel_coords`` INT32 [-1,4] (b,z,y,x), ``voxel_num_points`` INT32 [-1];
  outputs ``pred_boxes`` [-1,7], ``pred_scores`` [-1], ``pred_labels`` INT64
  [-1] (1-based).  On MI355X: MFMA PillarVFE+scatter from the received
  voxels, fp32 pair-storage backbone, anchor decode + rotated NMS kernels.  The voxel
  geometry is published in ``ModelConfig.parameters`` so clients voxelise
  with the model's own parameters (fixes SURVEY Appendix A9).

Weights are random-init (He + LSUV on a synthetic sample, detection-head
prior calibrated) exactly like the bench; ``--weights`` loading of a
state_dict is supported for real checkpoints.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..config.lidar import PointPillarsConfig, VoxelConfig
from ..proto import model_config_pb2 as mc
from .model import PROFILE, InferError, ServedModel, tensor_spec
from ..utils.model_store import load_state_dict


_STAGE_POOL = None


def _stage_parallel(fn, n: int, inline: bool = False) -> None:
    """Run fn(0..n-1) on a small shared thread pool: the per-request copies of a
    dynamic batch into pinned staging (numpy releases the GIL inside copyto, so
    the host memcpys of several multi-MB requests overlap).  inline: no host
    copies to overlap (device or page-locked sources), run in this thread."""
    global _STAGE_POOL
    if n <= 1 or inline:
        for i in range(n):
            fn(i)
        return
    if _STAGE_POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _STAGE_POOL = ThreadPoolExecutor(8, thread_name_prefix="stage")
    list(_STAGE_POOL.map(fn, range(n)))


def _device(device) -> torch.device:
    if device in (None, "auto"):
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(device)


PLAN_SIZES = (1, 2, 4, 6, 8, 12, 16)  # captured batch sizes per served model; a dynamic batch runs on the smallest >= n


def _direct(a, dtype) -> Optional[torch.Tensor]:
    """The request tensor itself as a copy source: a view of a device shared-memory
    region (a device-to-device copy, any dtype: the copy converts), or a contiguous
    view of a page-locked system region with the model's dtype (a DMA, no staging copy)."""
    if isinstance(a, torch.Tensor):
        return a if a.is_cuda else None
    from .shm import pinned_host
    if a.dtype == np.dtype(dtype) and pinned_host(a):
        return torch.from_numpy(a)
    return None


def _direct_out(dst: Optional[Dict[str, np.ndarray]], name: str, staging: torch.Tensor) -> torch.Tensor:
    """Where one request's output goes from the device: its shared-memory output slice
    (``dst[name]``, raw bytes) viewed with the staging tensor's dtype and shape when that
    slice is large enough and page-locked, else the pinned staging."""
    from .shm import pinned_host
    d = dst.get(name) if dst else None
    nb = staging.numel() * staging.element_size()
    if isinstance(d, torch.Tensor):  # a device region: the output is copied on the device
        if d.is_cuda and d.numel() >= nb:
            return d[:nb].view(staging.dtype).view(tuple(staging.shape))
        return staging
    if d is not None and d.nbytes >= nb:
        v = d[:nb]
        if pinned_host(v):
            return torch.from_numpy(v.view(staging.numpy().dtype).reshape(tuple(staging.shape)))
    return staging


def _copy_all(dsts: Sequence[torch.Tensor], srcs: Sequence[torch.Tensor]) -> None:
    """dst[i] <- src[i] on the current stream: device-to-device pairs of one dtype and
    contiguous layout as ONE launch of the segment-copy kernel (csrc/kernels/copy.hip;
    an IPC-mapped slot would otherwise take the runtime's peer-copy path), the rest
    (host sources, dtype conversions, strided views) by one torch foreach call."""
    seg_d, seg_s, seg_n, rest_d, rest_s = [], [], [], [], []
    for d, s_ in zip(dsts, srcs):
        if (d.is_cuda and s_.is_cuda and d.dtype == s_.dtype and d.numel() == s_.numel()
                and d.is_contiguous() and s_.is_contiguous()):
            if d.numel():
                seg_d.append(d.data_ptr())
                seg_s.append(s_.data_ptr())
                seg_n.append(d.numel() * d.element_size())
        else:
            rest_d.append(d)
            rest_s.append(s_.view(d.shape) if s_.numel() == d.numel() and s_.shape != d.shape else s_)
    if seg_d:
        from .. import _native
        dp, sp, nb = (np.asarray(v, np.int64) for v in (seg_d, seg_s, seg_n))
        _native.call("tca_copy_segments", len(seg_d), dp.ctypes.data, sp.ctypes.data, nb.ctypes.data,
                     _native.stream_ptr(torch.cuda.current_stream()))
    if rest_d:
        torch._foreach_copy_(rest_d, rest_s, non_blocking=True)


class _Segs:
    """Device-to-device copy segments gathered from raw pointers and issued as ONE
    launch (csrc/kernels/copy.hip): the served plans' per-request copies cost no
    torch op each (every torch op drops and re-takes the GIL, which the server's
    request threads contend for)."""
    __slots__ = ("d", "s", "n")

    def __init__(self):
        self.d, self.s, self.n = [], [], []

    def add(self, dst: int, src: int, nbytes: int) -> None:
        if nbytes > 0:
            self.d.append(dst)
            self.s.append(src)
            self.n.append(nbytes)

    def launch(self) -> None:
        if self.d:
            from .. import _native
            dp, sp, nb = (np.asarray(v, np.int64) for v in (self.d, self.s, self.n))
            _native.call("tca_copy_segments", len(self.d), dp.ctypes.data, sp.ctypes.data, nb.ctypes.data,
                         _native.stream_ptr(torch.cuda.current_stream()))


def _dev_src(a, dtype: torch.dtype, nbytes: int) -> Optional[int]:
    """Pointer of a device-resident request tensor usable as a raw copy source
    (dtype, contiguity and size as the plan's slot), else None."""
    if (isinstance(a, torch.Tensor) and a.is_cuda and a.dtype == dtype and a.is_contiguous()
            and a.numel() * a.element_size() == nbytes):
        return a.data_ptr()
    return None


_OUT_VIEWS: Dict[tuple, torch.Tensor] = {}


def _typed_out(d: torch.Tensor, staging: torch.Tensor) -> torch.Tensor:
    """A device output slot (uint8 view of a device region) as staging's dtype / shape, cached."""
    key = (d.data_ptr(), d.numel(), staging.dtype, tuple(staging.shape))
    v = _OUT_VIEWS.get(key)
    if v is None:
        nb = staging.numel() * staging.element_size()
        v = d[:nb].view(staging.dtype).view(tuple(staging.shape))
        if len(_OUT_VIEWS) > 4096:
            _OUT_VIEWS.clear()
        _OUT_VIEWS[key] = v
    return v


class _PlanClock:
    """Served-plan phase clock for the server stage profile (TCA_SERVER_PROFILE):
    host time of each phase's issue and the device time between HIP events on the
    plan's stream (H2D, graph replay, D2H).  Inert when profiling is off."""

    def __init__(self, tag: str):
        from .model import PROFILE
        self.on, self.tag = PROFILE.on, tag
        if self.on:
            self.ev = [(None, torch.cuda.Event(enable_timing=True))]
            self.ev[0][1].record()
            self.t = time.perf_counter()

    def mark(self, name: str) -> None:
        if self.on:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.ev.append((name, e))
            from .model import PROFILE
            t = time.perf_counter()
            PROFILE.add(f"{self.tag}.host.{name}", t - self.t)
            self.t = t

    def done(self) -> None:
        if self.on:
            from .model import PROFILE
            self.ev[-1][1].synchronize()
            for (_, a), (name, b) in zip(self.ev[:-1], self.ev[1:]):
                PROFILE.add(f"{self.tag}.gpu.{name}", a.elapsed_time(b) * 1e-3)


def _instances(n: Optional[int]) -> int:
    """Model instances of the GPU models with captured batch plans (Triton instance_group count):
    the explicit value, else TCA_SERVE_INSTANCES, else 1.  Measured with 4 + 4 client processes
    (profiles/r3/served_instances.json): 2 instances split the arriving requests into batches of
    2-3 (vs 3-8 at one instance) and run slower on every wire, so one stays the default."""
    if n is None:
        n = int(os.environ.get("TCA_SERVE_INSTANCES", "1"))
    return max(1, int(n))


def _depth(d: Optional[int]) -> int:
    """Batches in flight per served GPU model (DynamicBatcher pipelining): the explicit value,
    else TCA_SERVE_PIPELINE, else 1.  At 2, batch k + 1 is staged, DMA'd and replayed on the
    other plan set's stream while batch k's D2H runs and its responses are encoded.  Measured
    with 4 + 4 client processes (profiles/r4/served/): 683 vs 741 pairs/s over shm, 266 vs 252
    raw -- the served path is bound by host work per request (gRPC + Python), not by the GPU,
    so one batch in flight (half the plan memory) stays the default."""
    if d is None:
        d = int(os.environ.get("TCA_SERVE_PIPELINE", "1"))
    return max(1, int(d))


def _pick(plans: Dict[int, object], n: int):
    return plans[min(b for b in plans if b >= n)]


class _YoloPlan:
    """A captured batch-B YOLOv5 pass over the calibrated module: the request
    images (straight from a pinned shm region, else one host copy into pinned
    staging) -> DMA -> fused-MFMA plan -> decode -> one D2H into pinned."""

    def __init__(self, pipe, B: int, img: int, device):
        from ..models.fast import FastYOLOv5
        from ..pipelines.graph import GraphRunner
        import copy

        from ..ops._ws import Workspace
        self.B, self.img = B, img
        self.fast = FastYOLOv5(pipe.model, B, (img, img), device, precision=pipe.precision)
        # a postprocess of its own: the workspace re-allocates its buffers when the batch
        # changes, which would free memory that another plan's captured graph writes
        post = copy.copy(pipe.post)
        post.ws = Workspace(device)
        self.x_dev = torch.zeros((B, 3, img, img), dtype=torch.float32, device=device)
        self.pin_in = torch.empty((B, 3, img, img), dtype=torch.float32).pin_memory()

        def step():
            self.fast.set_input(self.x_dev)
            return post.decode(self.fast.forward())
        self.runner = GraphRunner(step)
        self.runner.capture()  # under the repository's exclusive GPU phase, never lazily while serving
        self.pin_out = torch.empty(self.runner.out.shape, dtype=torch.float32).pin_memory()
        # static per-slot views and pointers: the run loop issues no torch op per request
        self.x_slots = [self.x_dev[i] for i in range(B)]
        self.pin_slots = [self.pin_out[i:i + 1] for i in range(B)]
        self.dec_slots = [self.runner.out[i:i + 1] for i in range(B)]
        self.x_bytes = 3 * img * img * 4
        self.o_bytes = self.pin_slots[0].numel() * 4
        self.dec_f32 = self.runner.out.dtype == torch.float32

    def run(self, images: Sequence[np.ndarray], dsts=None) -> List[Dict[str, torch.Tensor]]:
        """dsts: per request None or {output name: uint8 view of the request's output
        shared-memory slice}; a slice inside a page-locked region receives its output
        by DMA straight from the device, a device region (device shared memory) by the
        segment-copy kernel (the response encoder then has nothing to copy)."""
        return self.issue(images, dsts)()

    def issue(self, images: Sequence[np.ndarray], dsts=None):
        """Stage, DMA, replay and queue the D2H on the current stream without waiting:
        returns finish() -> the outputs (waits for this batch's work only).  The plan's
        buffers stay in use until finish() returns."""
        n, img = len(images), self.img
        clk = _PlanClock("YOLOv5")
        segs, host = _Segs(), []
        xb = self.x_dev.data_ptr()
        for i, a in enumerate(images):
            p = _dev_src(a, torch.float32, self.x_bytes)
            if p is None:
                host.append(i)
            else:
                segs.add(xb + i * self.x_bytes, p, self.x_bytes)
        srcs = {}

        def stage(i):
            a = images[i].reshape(3, img, img)
            src = _direct(a, np.float32)
            if src is None:
                np.copyto(self.pin_in[i].numpy(), a, casting="same_kind")
                src = self.pin_in[i]
            srcs[i] = src
        _stage_parallel(lambda k: stage(host[k]), len(host))
        clk.mark("host_stage")
        segs.launch()  # slots >= n: stale, outputs unused
        if host:
            _copy_all([self.x_slots[i] for i in host], [srcs[i] for i in host])
        clk.mark("h2d")
        self.runner()
        clk.mark("graph")
        outs, segs, rest = [None] * n, _Segs(), []
        ob = self.runner.out.data_ptr()
        for i in range(n):
            d = dsts[i].get("output") if dsts and dsts[i] else None
            if isinstance(d, torch.Tensor) and d.is_cuda and self.dec_f32 and d.numel() >= self.o_bytes:
                outs[i] = _typed_out(d, self.pin_slots[i])
                segs.add(outs[i].data_ptr(), ob + i * self.o_bytes, self.o_bytes)
            else:
                outs[i] = _direct_out(dsts[i] if dsts else None, "output", self.pin_slots[i])
                rest.append(i)
        segs.launch()
        if rest:
            _copy_all([outs[i] for i in rest], [self.dec_slots[i] for i in rest])
        clk.mark("d2h")
        done = torch.cuda.Event()
        done.record()

        def finish():
            done.synchronize()
            clk.mark("sync")
            clk.done()
            return [{"output": o} for o in outs]
        return finish


def check_voxel_shapes(inputs, P: int, max_voxels: int) -> int:
    """The shape part of :func:`check_voxel_inputs` (no value reads) → V."""
    vox, co, n = inputs["voxels"], inputs["voxel_coords"], inputs["voxel_num_points"]
    if vox.ndim != 3 or vox.shape[1] != P or vox.shape[2] < 4:
        raise InferError(f"voxels must be [-1, {P}, 4], got {list(vox.shape)}")
    V = vox.shape[0]
    if V > max_voxels:
        raise InferError(f"{V} voxels > max_voxels {max_voxels}")
    if co.ndim != 2 or co.shape[0] != V or co.shape[1] != 4:
        raise InferError(f"voxel_coords must be [{V}, 4], got {list(co.shape)}")
    if n.ndim != 1 or n.shape[0] != V:
        raise InferError(f"voxel_num_points must be [{V}], got {list(n.shape)}")
    return V


def check_voxel_inputs(inputs: Dict[str, np.ndarray], P: int, max_voxels: int, grid_size) -> int:
    """Validate one request's (voxels, voxel_coords, voxel_num_points) against the
    model's voxel grid before any byte reaches the device.  The GPU consumers index
    ``(b * ny + y) * nx + x`` (pillar scatter, canvas clear, sparse-conv rulebook)
    without a range check, so an out-of-range cell of one request would write into
    another request's canvas slot of a dynamic batch, or outside the allocation.
    Returns V.  Reference contract: ``examples/pointpillar_kitti/config.pbtxt:27-52``
    (voxels [-1, P, 4], voxel_coords [-1, 4] = (b, z, y, x), voxel_num_points [-1])."""
    vox, co, n = inputs["voxels"], inputs["voxel_coords"], inputs["voxel_num_points"]
    dev = isinstance(co, torch.Tensor)
    if vox.ndim != 3 or vox.shape[1] != P or vox.shape[2] < 4:
        raise InferError(f"voxels must be [-1, {P}, 4], got {list(vox.shape)}")
    V = vox.shape[0]
    if V > max_voxels:
        raise InferError(f"{V} voxels > max_voxels {max_voxels}")
    if co.ndim != 2 or co.shape[0] != V or co.shape[1] != 4:
        raise InferError(f"voxel_coords must be [{V}, 4], got {list(co.shape)}")
    if n.ndim != 1 or n.shape[0] != V:
        raise InferError(f"voxel_num_points must be [{V}], got {list(n.shape)}")
    if V:
        nx, ny, nz = (int(g) for g in grid_size)
        if dev:  # device shared memory: the reductions on the GPU, one small copy back
            lo, hi = torch.aminmax(co.to(torch.int64), dim=0)
            nlo, nhi = torch.aminmax(n.to(torch.int64))
            v = torch.cat([lo, hi, nlo.view(1), nhi.view(1)]).cpu().tolist()
            lo, hi, nmin, nmax = v[0:4], v[4:8], v[8], v[9]
        else:
            lo, hi = co.min(axis=0), co.max(axis=0)  # (b, z, y, x): two passes, not six
            nmin, nmax = n.min(), n.max()
        if (int(lo[1]) < 0 or int(hi[1]) >= nz or int(lo[2]) < 0 or int(hi[2]) >= ny
                or int(lo[3]) < 0 or int(hi[3]) >= nx):
            raise InferError(f"voxel_coords outside the {nz}x{ny}x{nx} (z, y, x) grid")
        if int(nmin) < 1 or int(nmax) > P:
            raise InferError(f"voxel_num_points must be in [1, {P}]")
    return V


class _PointPillarsPlan:
    """A captured batch-B PointPillars pass from received voxels: per-frame batch
    index -> pillar VFE + canvas scatter -> BEV plan -> anchor decode + rotated
    NMS, and the written canvas cells cleared at the end so the next replay
    starts from an empty canvas.  Outputs come back by one D2H per tensor."""

    def __init__(self, model, cfg: PointPillarsConfig, B: int, device):
        from ..pipelines.graph import GraphRunner
        from ..pipelines.lidar import LidarPipeline
        V, P = cfg.voxel.max_voxels, cfg.voxel.max_points_per_voxel
        self.B, self.V, self.P = B, V, P
        self.pipe = LidarPipeline(model, batch=B, max_points=1024, device=device)
        self.enc = self.pipe.enc
        self.voxels = torch.zeros((B, V, P, 4), dtype=torch.float32, device=device)
        self.coords = torch.zeros((B, V, 4), dtype=torch.int32, device=device)
        self.nump = torch.zeros((B, V), dtype=torch.int32, device=device)
        self.vcount = torch.zeros((B,), dtype=torch.int32, device=device)
        self.bidx = torch.arange(B, dtype=torch.int32, device=device).view(B, 1).expand(B, V).contiguous()
        self.pin_vcount = torch.zeros((B,), dtype=torch.int32).pin_memory()
        self.pin_vox = torch.empty((B, V, P, 4), dtype=torch.float32).pin_memory()
        self.pin_co = torch.empty((B, V, 4), dtype=torch.int32).pin_memory()
        self.pin_n = torch.empty((B, V), dtype=torch.int32).pin_memory()
        self.flags = torch.zeros((B,), dtype=torch.int32, device=device)  # per slot: coordinates out of range
        self.pin_flags = torch.zeros((B,), dtype=torch.int32).pin_memory()
        self.grid = tuple(int(g) for g in cfg.voxel.grid_size)  # nx, ny, nz
        self.enc.clear(self.pipe.vox)
        fast = self.pipe.fast or self.pipe.build_fast()  # sets the canvas storage first

        def step():
            self.coords[:, :, 0].copy_(self.bidx)
            self.enc.encode_from_voxels(self.voxels, self.nump, self.coords, self.vcount)
            res = self.pipe.post(*fast.forward(self.enc.canvas_nhwc()))
            self.enc.clear_coords(self.coords, self.vcount)
            return res
        self.runner = GraphRunner(step)
        self.runner.capture()
        r = self.runner.out
        self.outs = (r.count, r.box, r.score, r.cls)
        self.pin_out = [torch.empty(t.shape, dtype=t.dtype).pin_memory() for t in self.outs]
        # numpy views / raw slot strides: the run loop issues no torch op per request
        self.pin_np = [t.numpy() for t in self.pin_out]
        self.pin_vcount_np, self.pin_flags_np = self.pin_vcount.numpy(), self.pin_flags.numpy()
        self.d2h_src, self.d2h_dst = list(self.outs) + [self.flags], list(self.pin_out) + [self.pin_flags]
        self.vox_stride, self.co_stride, self.n_stride = V * P * 16, V * 16, V * 4

    def _device_slot(self, i: int, x, segs: "_Segs") -> bool:
        """Slot i's D2D copies when the request's tensors are device-resident (device shared
        memory) in the plan's dtypes and layouts."""
        vox, co, nn_ = x["voxels"], x["voxel_coords"], x["voxel_num_points"]
        if not (isinstance(vox, torch.Tensor) and vox.is_cuda and vox.dim() == 3 and vox.shape[2] == 4):
            return False
        V = vox.shape[0]
        pv = _dev_src(vox, torch.float32, V * self.P * 16)
        pc = _dev_src(co, torch.int32, V * 16)
        pn = _dev_src(nn_, torch.int32, V * 4)
        if pv is None or pc is None or pn is None:
            return False
        segs.add(self.voxels.data_ptr() + i * self.vox_stride, pv, V * self.P * 16)
        segs.add(self.coords.data_ptr() + i * self.co_stride, pc, V * 16)
        segs.add(self.nump.data_ptr() + i * self.n_stride, pn, V * 4)
        self.pin_vcount_np[i] = V
        return True

    def run(self, batch: Sequence[Dict[str, np.ndarray]]) -> List[Dict[str, np.ndarray]]:
        return self.issue(batch)()

    def issue(self, batch: Sequence[Dict[str, np.ndarray]]):
        """As _YoloPlan.issue: everything queued on the current stream, finish() waits
        for this batch and reads its results out of the pinned outputs."""
        n = len(batch)
        self.pin_vcount_np[:] = 0
        segs = _Segs()
        host = [i for i in range(n) if not self._device_slot(i, batch[i], segs)]
        srcs = [None] * n

        def stage(i):
            vox, co, nn_ = batch[i]["voxels"], batch[i]["voxel_coords"], batch[i]["voxel_num_points"]
            V = vox.shape[0]
            if isinstance(vox, torch.Tensor) and vox.is_cuda:  # device shared memory: device-to-device
                sv, sc, sn = vox[..., :4], co, nn_
            else:
                sv = _direct(vox, np.float32) if vox.shape[-1] == 4 else None
                sc, sn = _direct(co, np.int32), _direct(nn_, np.int32)
            if sv is None:
                np.copyto(self.pin_vox[i, :V].numpy(), vox[..., :4], casting="same_kind")
                sv = self.pin_vox[i, :V]
            if sc is None:
                np.copyto(self.pin_co[i, :V].numpy(), co, casting="unsafe")
                sc = self.pin_co[i, :V]
            if sn is None:
                np.copyto(self.pin_n[i, :V].numpy(), nn_, casting="unsafe")
                sn = self.pin_n[i, :V]
            srcs[i] = (V, sv, sc, sn)
            self.pin_vcount_np[i] = V
        clk = _PlanClock("PointPillars")
        _stage_parallel(lambda k: stage(host[k]), len(host))
        clk.mark("host_stage")
        segs.launch()
        dst, src = [self.vcount], [self.pin_vcount]  # slots >= n: no voxels
        for i in host:
            V, sv, sc, sn = srcs[i]
            if V:
                dst += [self.voxels[i, :V], self.coords[i, :V], self.nump[i, :V]]
                src += [sv, sc, sn]
        _copy_all(dst, src)
        # range check on the device (whatever the transport): a bad slot's voxel count is zeroed
        # before the graph reads it, and the request is answered with an error below
        from .. import _native
        nx, ny, nz = self.grid
        _native.call("tca_voxel_check", _native.ptr(self.coords), _native.ptr(self.nump), _native.ptr(self.vcount),
                     n, self.V, self.P, nz, ny, nx, _native.ptr(self.flags),
                     _native.stream_ptr(torch.cuda.current_stream()))
        clk.mark("h2d")
        self.runner()
        clk.mark("graph")
        torch._foreach_copy_(self.d2h_dst, self.d2h_src, non_blocking=True)  # all B slots: one call
        clk.mark("d2h")
        done = torch.cuda.Event()
        done.record()

        def finish():
            done.synchronize()
            clk.mark("sync")
            cnt, box, score, cls = self.pin_np
            bad = self.pin_flags_np
            res = [InferError(f"voxel_coords outside the {self.grid[2]}x{self.grid[1]}x{self.grid[0]} (z, y, x) "
                              f"grid or voxel_num_points outside [1, {self.P}]") if bad[i] else
                   {"pred_boxes": box[i, :k], "pred_scores": score[i, :k],
                    "pred_labels": cls[i, :k].astype(np.int64, copy=False)}
                   for i, k in enumerate(cnt[:n].tolist())]
            clk.mark("result")
            clk.done()
            return res
        return finish


class YoloV5Model(ServedModel):
    def __init__(self, name: str = "YOLOv5nCOCO", variant: str = "n", nc: int = 80, img: int = 640,
                 device="auto", weights: Optional[str] = None, seed: int = 0, calibrate_target: float = 100.0,
                 batch: int = 16, instances: Optional[int] = None, pipeline_depth: Optional[int] = None):
        super().__init__(name)
        self.batch = batch  # dynamic batching: concurrent requests run as one captured batch-`batch` graph
        self.instances = _instances(instances)
        self.pipeline_depth = _depth(pipeline_depth)
        self.variant, self.nc, self.img = variant, nc, img
        self.device = _device(device)
        self.weights, self.seed, self.calibrate_target = weights, seed, calibrate_target
        from ..models.yolov5 import YoloConfig
        self.N = YoloConfig(variant, nc, (img, img)).num_predictions()

    def inputs(self):
        return [tensor_spec("images", "FP32", [3, self.img, self.img], fmt="NCHW", reshape=[1, 3, self.img, self.img])]

    def outputs(self):
        return [tensor_spec("output", "FP32", [1, self.N, 5 + self.nc], output=True)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_GPU if self.device.type == "cuda" else mc.ModelInstanceGroup.KIND_CPU

    def load(self):
        from ..pipelines.camera import CameraPipeline
        from ..models.yolov5 import build_yolov5
        from ..utils.synthetic import camera_frame

        model = build_yolov5(self.variant, self.nc, self.img, self.seed)
        if self.weights:
            model.load_state_dict(load_state_dict(self.weights, getattr(self, "weights_sha256", None)))
        if self.device.type == "cuda":
            self.pipe = CameraPipeline(model, batch=1, src_hw=(self.img, self.img), img_hw=(self.img, self.img),
                                       mode="stretch", device=self.device)
            if not self.weights:
                self.pipe.frames[0].copy_(torch.from_numpy(camera_frame(self.img, self.img, self.seed)))
                self.pipe.calibrate_detection_density(self.calibrate_target)
            self.model = self.pipe.model
            # captured plans at PLAN_SIZES up to the dynamic batch (the same kernels as the local camera
            # pipeline), all over the calibrated module
            sizes = sorted({b for b in PLAN_SIZES if b <= max(1, self.batch)} | {max(1, self.batch)})
            self.plan_sets = [{b: _YoloPlan(self.pipe, b, self.img, self.device) for b in sizes}
                              for _ in range(self.plan_set_count())]
            self.plans = self.plan_sets[0]
            self.dynamic_batch = max(sizes)
        else:
            from ..models.common import fuse_model
            if not self.weights:  # same head prior as the GPU path (random init)
                pipe = CameraPipeline(model, batch=1, src_hw=(self.img, self.img), img_hw=(self.img, self.img),
                                      mode="stretch", device="cpu")
                pipe.frames[0].copy_(torch.from_numpy(camera_frame(self.img, self.img, self.seed)))
                pipe.calibrate_detection_density(self.calibrate_target)
                model = pipe.model
            self.model = fuse_model(model.eval())
        self.ready = True

    @torch.no_grad()
    def execute(self, inputs, requested):
        if self.device.type == "cuda":
            return self.plans[1].run([inputs["images"]])[0]  # the response encoder reads the pinned staging
        x = inputs["images"].reshape(1, 3, self.img, self.img)
        heads = self.model(torch.from_numpy(np.require(x, np.float32, ['C', 'W'])))
        from ..models.yolov5 import yolo_decode_reference
        out = yolo_decode_reference(heads, self.model.anchors).numpy()
        return {"output": out.astype(np.float32, copy=False)}

    accepts_out_dst = True
    device_inputs = True

    @torch.no_grad()
    def execute_batch(self, batch, requested, dsts=None, inst: int = 0):
        if self.device.type != "cuda":
            return [self.execute(x, requested) for x in batch]
        return _pick(self.plan_sets[inst], len(batch)).run([x["images"] for x in batch], dsts)

    @torch.no_grad()
    def execute_batch_async(self, batch, requested, dsts=None, inst: int = 0):
        """Plan set ``inst`` issues the batch on the current stream; returns finish()."""
        return _pick(self.plan_sets[inst], len(batch)).issue([x["images"] for x in batch], dsts)


class PointPillarsModel(ServedModel):
    def __init__(self, name: str = "pointpillar_kitti", cfg: Optional[PointPillarsConfig] = None, device="auto",
                 weights: Optional[str] = None, seed: int = 0, calibrate_target: float = 2000.0,
                 batch: int = 16, instances: Optional[int] = None, pipeline_depth: Optional[int] = None):
        super().__init__(name)
        self.batch = batch  # dynamic batching: concurrent requests share one batch-`batch` pass
        self.instances = _instances(instances)
        self.pipeline_depth = _depth(pipeline_depth)
        self.cfg = cfg or PointPillarsConfig()
        self.device = _device(device)
        self.weights, self.seed, self.calibrate_target = weights, seed, calibrate_target
        self.P = self.cfg.voxel.max_points_per_voxel

    def inputs(self):
        return [tensor_spec("voxels", "FP32", [-1, self.P, 4]), tensor_spec("voxel_coords", "INT32", [-1, 4]),
                tensor_spec("voxel_num_points", "INT32", [-1])]

    def outputs(self):
        return [tensor_spec("pred_boxes", "FP32", [-1, 7], output=True),
                tensor_spec("pred_scores", "FP32", [-1], output=True),
                tensor_spec("pred_labels", "INT64", [-1], output=True)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_GPU if self.device.type == "cuda" else mc.ModelInstanceGroup.KIND_CPU

    def config(self):
        c = super().config()
        v = self.cfg.voxel
        for k, val in (("point_cloud_range", list(v.point_cloud_range)), ("voxel_size", list(v.voxel_size)),
                       ("max_points_per_voxel", v.max_points_per_voxel), ("max_voxels", v.max_voxels),
                       ("class_names", list(self.cfg.class_names))):
            c.parameters[k].string_value = json.dumps(val)
        return c

    def load(self):
        from ..models.pointpillars import build_pointpillars
        model = build_pointpillars(self.cfg, self.seed)
        if self.weights:
            model.load_state_dict(load_state_dict(self.weights, getattr(self, "weights_sha256", None)))
        if self.device.type == "cuda":
            from ..pipelines.lidar import LidarPipeline
            from ..utils.synthetic import LidarSpec, lidar_sweep

            spec = LidarSpec(sensor_height=3.23)
            maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
            self.pipe = LidarPipeline(model, batch=1, max_points=maxp, device=self.device)
            if not self.weights:
                c = lidar_sweep(spec, self.seed)
                raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
                self.pipe.data[: raw.numel()].copy_(raw)
                self.pipe.frame_n.fill_(c.shape[0])
                self.pipe.calibrate_detection_density(self.calibrate_target)
            self.model = self.pipe.model
            sizes = sorted({b for b in PLAN_SIZES if b <= max(1, self.batch)} | {max(1, self.batch)})
            self.plan_sets = [{b: _PointPillarsPlan(self.model, self.cfg, b, self.device) for b in sizes}
                              for _ in range(self.plan_set_count())]
            self.plans = self.plan_sets[0]
            self.dynamic_batch = max(sizes)
        else:
            from ..models.common import fuse_model
            self.model = fuse_model(model.eval())
        self.ready = True

    def _check(self, inputs):
        return check_voxel_inputs(inputs, self.P, self.cfg.voxel.max_voxels, self.cfg.voxel.grid_size)

    device_inputs = True

    def validate(self, inputs):
        super().validate(inputs)
        if self.device.type == "cuda":
            # shapes here; the coordinate / point-count values of every slot are range-checked on the
            # device inside the batch plan (tca_voxel_check: a bad request is answered with its
            # InferError, its slot zeroed before the graph reads it).  The host reductions cost ~1.3 ms
            # of GIL per request (profiles/r4/served/*prof*: pointpillar_kitti.validate)
            check_voxel_shapes(inputs, self.P, self.cfg.voxel.max_voxels)
        else:
            self._check(inputs)

    @torch.no_grad()
    def execute_batch(self, batch, requested, inst: int = 0):
        """Host inputs validated by :meth:`validate` (every request reaches the batcher
        through it); every slot's coordinate / count ranges are checked again on the device
        inside the plan (csrc/kernels/copy.hip tca_voxel_check), which is the check for
        device shared-memory inputs."""
        if self.device.type != "cuda":
            return [self.execute(x, requested) for x in batch]
        return _pick(self.plan_sets[inst], len(batch)).run(batch)  # an out-of-range request's entry is its InferError

    @torch.no_grad()
    def execute_batch_async(self, batch, requested, dsts=None, inst: int = 0):
        return _pick(self.plan_sets[inst], len(batch)).issue(batch)

    @torch.no_grad()
    def execute(self, inputs, requested):
        vox = inputs["voxels"]
        co = inputs["voxel_coords"]
        n = inputs["voxel_num_points"]
        self._check(inputs)
        if self.device.type == "cuda":
            r = self.plans[1].run([inputs])[0]
            if isinstance(r, BaseException):
                raise r
            return r
        else:
            from ..models.pointpillars import pillar_point_features, scatter_to_bev
            from ..ops.lidar import AnchorPostprocess
            v = torch.from_numpy(np.require(vox[..., :4], np.float32, ['C', 'W']))
            c = torch.from_numpy(np.require(co, np.int32, ['C', 'W'])).clone()
            c[:, 0] = 0
            f = pillar_point_features(v, torch.from_numpy(n.astype(np.int64)), c, self.cfg.voxel)
            pf = self.model.vfe(f)
            nx, ny, _ = self.cfg.voxel.grid_size
            canvas = scatter_to_bev(pf, c, 1, ny, nx, channels_last=False)
            cls, box, dr = self.model.bev_forward(canvas)
            res = AnchorPostprocess(self.cfg, 1, device="cpu").cpu(cls, box, dr)
        k = int(res.count[0])
        return {"pred_boxes": res.box[0, :k].cpu().numpy().astype(np.float32),
                "pred_scores": res.score[0, :k].cpu().numpy().astype(np.float32),
                "pred_labels": res.cls[0, :k].cpu().numpy().astype(np.int64)}


class SecondIoUModel(ServedModel):
    """``second_iou`` — OpenPCDet SECONDNetIoU (``examples/second_iou/config.pbtxt``,
    KIND_GPU; ``examples/second_iou/1/model.py``): inputs ``voxels`` FP32
    [-1, 5, 4], ``voxel_coords`` INT32 [-1, 4] (b, z, y, x), ``voxel_num_points``
    INT32 [-1] — the client's KITTI voxels (``data/kitti_dataset.yaml``); outputs
    ``pred_boxes`` FP32 [-1, 7], ``pred_scores`` FP32 [-1] (sigmoid IoU),
    ``pred_labels`` INT64 [-1] (1-based).  GPU: MeanVFE + sparse 3D backbone
    (spconv.hip gather-GEMMs) from the received voxels, fused BEV convs,
    proposal top-k + rotated NMS, RoI grid pool + FC IoU head, final NMS."""

    def __init__(self, name: str = "second_iou", cfg=None, device="auto", weights: Optional[str] = None,
                 seed: int = 0, calibrate_target: float = 60.0):
        from ..config.lidar import SecondIoUConfig

        super().__init__(name)
        self.cfg = cfg or SecondIoUConfig()
        self.device = _device(device)
        self.weights, self.seed, self.calibrate_target = weights, seed, calibrate_target
        self.P = self.cfg.voxel.max_points_per_voxel

    def inputs(self):
        return [tensor_spec("voxels", "FP32", [-1, self.P, 4]), tensor_spec("voxel_coords", "INT32", [-1, 4]),
                tensor_spec("voxel_num_points", "INT32", [-1])]

    def outputs(self):
        return [tensor_spec("pred_boxes", "FP32", [-1, 7], output=True),
                tensor_spec("pred_scores", "FP32", [-1], output=True),
                tensor_spec("pred_labels", "INT64", [-1], output=True)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_GPU if self.device.type == "cuda" else mc.ModelInstanceGroup.KIND_CPU

    def config(self):
        c = super().config()
        v = self.cfg.voxel
        for k, val in (("point_cloud_range", list(v.point_cloud_range)), ("voxel_size", list(v.voxel_size)),
                       ("max_points_per_voxel", v.max_points_per_voxel), ("max_voxels", v.max_voxels),
                       ("class_names", list(self.cfg.class_names))):
            c.parameters[k].string_value = json.dumps(val)
        return c

    def load(self):
        from ..models.common import fuse_model
        from ..models.second import build_second_iou

        model = build_second_iou(self.cfg, self.seed)
        if self.weights:
            model.load_state_dict(load_state_dict(self.weights, getattr(self, "weights_sha256", None)))
        if self.device.type == "cuda":
            from ..pipelines.second import SecondPipeline
            from ..utils.synthetic import LidarSpec, lidar_sweep

            spec = LidarSpec(sensor_height=3.23)
            maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
            self.pipe = SecondPipeline(model, batch=1, max_points=maxp, device=self.device, z_offset=1.5)
            if not self.weights:
                c = lidar_sweep(spec, self.seed)
                raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
                self.pipe.data[: raw.numel()].copy_(raw)
                self.pipe.frame_n.fill_(c.shape[0])
                self.pipe.calibrate_detection_density(self.calibrate_target)
            V = self.cfg.voxel.max_voxels
            self.voxels = torch.zeros((V, self.P, 4), dtype=torch.float32, device=self.device)
            self.coords = torch.zeros((V, 4), dtype=torch.int32, device=self.device)
            self.nump = torch.zeros((V,), dtype=torch.int32, device=self.device)
            self.vcount = torch.zeros((1,), dtype=torch.int32, device=self.device)
            self.model = self.pipe.model
        else:
            self.model = fuse_model(model.eval())
        self.ready = True

    @torch.no_grad()
    def execute(self, inputs, requested):
        vox, co, n = inputs["voxels"], inputs["voxel_coords"], inputs["voxel_num_points"]
        V = check_voxel_inputs(inputs, self.P, self.cfg.voxel.max_voxels, self.cfg.voxel.grid_size)
        v = torch.from_numpy(np.require(vox[..., :4], np.float32, ['C', 'W']))
        c = torch.from_numpy(np.require(co, np.int32, ['C', 'W'])).clone()
        c[:, 0] = 0
        nn_ = torch.from_numpy(np.require(n, np.int32, ['C', 'W']))
        if self.device.type == "cuda":
            self.voxels[:V].copy_(v)
            self.coords[:V].copy_(c)
            self.nump[:V].copy_(nn_)
            self.vcount.fill_(V)
            res = self.pipe.run_voxels(self.voxels, self.nump, self.coords, self.vcount)
            k = int(res.count[0])
            return {"pred_boxes": res.box[0, :k].cpu().numpy().astype(np.float32),
                    "pred_scores": res.score[0, :k].cpu().numpy().astype(np.float32),
                    "pred_labels": res.cls[0, :k].cpu().numpy().astype(np.int64)}
        from ..models.second import postprocess_reference, proposal_config
        from ..ops.lidar import AnchorPostprocess
        m = self.model
        bev = m.sparse_forward(v, nn_.long(), c, 1)
        sf, cls, box, dr = m.bev_forward(bev)
        props = AnchorPostprocess(proposal_config(self.cfg), 1, device="cpu").cpu(cls, box, dr)
        logits = m.roi_iou(sf, props.box)
        bx, sc, lb = postprocess_reference(props.box, props.cls, props.count, logits, self.cfg)[0]
        return {"pred_boxes": bx.astype(np.float32), "pred_scores": sc.astype(np.float32),
                "pred_labels": lb.astype(np.int64)}


class CenterPointModel(ServedModel):
    """``centerpoint_pp`` — det3d CenterPoint-PointPillars (nuScenes, 10 classes):
    inputs ``voxels`` FP32 [-1, 20, 5] (x, y, z, r, time lag), ``voxel_coords``
    INT32 [-1, 4] (b, z, y, x), ``voxel_num_points`` INT32 [-1]; outputs
    ``pred_boxes`` FP32 [-1, 9] (x, y, z, w, l, h, vx, vy, yaw — yaw at index 8,
    as the reference's Detection3DArray branch reads it, ros_inference3d.py:189),
    ``pred_scores`` FP32 [-1], ``pred_labels`` INT64 [-1] (0-based nuScenes
    classes, data/nuScenes.names).  GPU: MFMA 2-layer PFN from the received
    voxels, fused RPN + CenterHead, K12 decode + per-task rotated NMS."""

    def __init__(self, name: str = "centerpoint_pp", cfg=None, device="auto", weights: Optional[str] = None,
                 seed: int = 0, calibrate_target: float = 1000.0, class_thresh=None):
        from ..config.lidar import CenterPointConfig

        super().__init__(name)
        self.cfg = cfg or CenterPointConfig()
        self.device = _device(device)
        self.weights, self.seed, self.calibrate_target = weights, seed, calibrate_target
        self.class_thresh = class_thresh
        self.P = self.cfg.voxel.max_points_per_voxel

    def inputs(self):
        return [tensor_spec("voxels", "FP32", [-1, self.P, 5]), tensor_spec("voxel_coords", "INT32", [-1, 4]),
                tensor_spec("voxel_num_points", "INT32", [-1])]

    def outputs(self):
        return [tensor_spec("pred_boxes", "FP32", [-1, 9], output=True),
                tensor_spec("pred_scores", "FP32", [-1], output=True),
                tensor_spec("pred_labels", "INT64", [-1], output=True)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_GPU if self.device.type == "cuda" else mc.ModelInstanceGroup.KIND_CPU

    def config(self):
        c = super().config()
        v = self.cfg.voxel
        for k, val in (("point_cloud_range", list(v.point_cloud_range)), ("voxel_size", list(v.voxel_size)),
                       ("max_points_per_voxel", v.max_points_per_voxel), ("max_voxels", v.max_voxels),
                       ("num_point_features", 5), ("class_names", list(self.cfg.class_names))):
            c.parameters[k].string_value = json.dumps(val)
        return c

    def load(self):
        from ..models.centerpoint import build_centerpoint
        from ..models.common import fuse_model

        model = build_centerpoint(self.cfg, self.seed)
        if self.weights:
            model.load_state_dict(load_state_dict(self.weights, getattr(self, "weights_sha256", None)))
        if self.device.type == "cuda":
            from ..pipelines.centerpoint import CenterPointPipeline
            from ..utils.synthetic import LidarSpec, lidar_sweep

            spec = LidarSpec(rings=32, azimuth_steps=1800, sensor_height=1.8)
            maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
            self.pipe = CenterPointPipeline(model, batch=1, max_points=maxp, device=self.device,
                                            class_thresh=self.class_thresh)
            if not self.weights:
                c = lidar_sweep(spec, self.seed)
                raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
                self.pipe.data[: raw.numel()].copy_(raw)
                self.pipe.frame_n.fill_(c.shape[0])
                self.pipe.calibrate_detection_density(self.calibrate_target)
            V = self.cfg.voxel.max_voxels
            self.voxels = torch.zeros((1, V, self.P, 5), dtype=torch.float32, device=self.device)
            self.coords = torch.zeros((1, V, 4), dtype=torch.int32, device=self.device)
            self.nump = torch.zeros((1, V), dtype=torch.int32, device=self.device)
            self.vcount = torch.zeros((1,), dtype=torch.int32, device=self.device)
            self.pipe.enc.clear(self.pipe.vox)
            self.model = self.pipe.model
        else:
            self.model = fuse_model(model.eval())
        self.ready = True

    @torch.no_grad()
    def execute(self, inputs, requested):
        vox, co, n = inputs["voxels"], inputs["voxel_coords"], inputs["voxel_num_points"]
        V = vox.shape[0]
        if vox.shape[1] != self.P or vox.shape[2] < 4:
            raise InferError(f"voxels must be [-1, {self.P}, 5], got {list(vox.shape)}")
        if V > self.cfg.voxel.max_voxels:
            raise InferError(f"{V} voxels > max_voxels {self.cfg.voxel.max_voxels}")
        F_ = min(vox.shape[2], 5)
        if self.device.type == "cuda":
            from ..ops.conv import NHWC

            p = self.pipe
            p.enc.clear_coords(self.coords, self.vcount)
            self.voxels[0, :V].zero_()
            self.voxels[0, :V, :, :F_].copy_(torch.from_numpy(np.require(vox[..., :F_], np.float32, ['C', 'W'])))
            self.coords[0, :V].copy_(torch.from_numpy(np.require(co, np.int32, ['C', 'W'])))
            self.coords[0, :V, 0] = 0
            self.nump[0, :V].copy_(torch.from_numpy(np.require(n, np.int32, ['C', 'W'])))
            self.vcount.fill_(V)
            p.enc.encode_from_voxels(self.voxels, self.nump, self.coords, self.vcount)
            fast = p.fast or p.build_fast()
            out = p.post(fast.forward(NHWC(p.enc.canvas))).per_image()[0]
        else:
            from ..models.centerpoint import merged_task_outputs, pfn_point_features
            from ..models.pointpillars import scatter_to_bev
            from ..ops.centerpoint import CenterPointPostprocess

            v = torch.zeros((V, self.P, 5))
            v[..., :F_] = torch.from_numpy(np.require(vox[..., :F_], np.float32, ['C', 'W']))
            c = torch.from_numpy(np.require(co, np.int32, ['C', 'W'])).clone()
            c[:, 0] = 0
            f = pfn_point_features(v, torch.from_numpy(n.astype(np.int64)), c, self.cfg.voxel)
            nx, ny, _ = self.cfg.voxel.grid_size
            canvas = scatter_to_bev(self.model.pfn(f), c, 1, ny, nx, channels_last=False)
            mo = merged_task_outputs(self.model.bev_forward(canvas))
            head = torch.cat([torch.nn.functional.pad(o, (0, 0, 0, 0, 0, 16 - o.shape[1])) for o in mo], 1)
            pp = CenterPointPostprocess(self.cfg, 1, [16 * t for t in range(len(mo))], "cpu", self.class_thresh)
            out = pp(head.permute(0, 2, 3, 1)).per_image()[0]
        return out


class _DetectronPlan:
    """A captured batch-B RetinaNet / FCOS pass from the served input tensor: request
    images (straight from a pinned shm region, else one host copy into pinned staging)
    -> DMA -> one kernel for (x - mean) / std + NCHW -> NHWC x 8 (image.hip
    tca_planar_affine) -> fused-MFMA ResNet-50-FPN + head -> decode / top-k / NMS
    -> one D2H per output into pinned staging."""

    def __init__(self, pipe, B: int, device):
        from ..models.fast import FastDetectron
        from ..ops.detectron import DetectronPostprocess
        from ..ops.image import planar_affine
        from ..pipelines.graph import GraphRunner

        H, W = pipe.cfg.input_hw
        self.B, self.H, self.W = B, H, W
        self.fast = FastDetectron(pipe.model, B, device, precision=pipe.precision)
        post = DetectronPostprocess(pipe.cfg, B, device)
        self.x_dev = torch.zeros((B, 3, H, W), dtype=torch.float32, device=device)
        self.pin_in = torch.empty((B, 3, H, W), dtype=torch.float32).pin_memory()
        sc, bi = pipe.scaling
        x_nhwc = self.fast.x.t

        def step():
            planar_affine(self.x_dev, x_nhwc, sc, bi)
            return post(self.fast.forward())
        self.runner = GraphRunner(step)
        self.runner.capture()  # under the repository's exclusive GPU phase
        r = self.runner.out
        self.outs = (r.count, r.box, r.score, r.cls)
        self.pin_out = [torch.empty(t.shape, dtype=t.dtype).pin_memory() for t in self.outs]

    def run(self, images: Sequence[np.ndarray]) -> List[Dict[str, np.ndarray]]:
        n, H, W = len(images), self.H, self.W
        srcs = [None] * n

        def stage(i):
            a = images[i].reshape(3, H, W)
            srcs[i] = _direct(a, np.float32)
            if srcs[i] is None:
                np.copyto(self.pin_in[i].numpy(), a, casting="same_kind")
                srcs[i] = self.pin_in[i]
        _stage_parallel(stage, n)
        _copy_all([self.x_dev[i] for i in range(n)], srcs)  # slots >= n: stale
        self.runner()
        for p, t in zip(self.pin_out, self.outs):
            p[:n].copy_(t[:n], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        cnt, box, score, cls = self.pin_out
        dims = np.array([[H, W]], np.int64)
        return [{"bboxex__0": box[i, :k].numpy(), "classes__1": cls[i, :k].numpy().astype(np.int64),
                 "scores__2": score[i, :k].numpy(), "dims__3": dims} for i, k in enumerate(cnt[:n].tolist())]


class DetectronModel(ServedModel):
    """Detectron2 RetinaNet / FCOS with the reference's served contract
    (``examples/RetinaNet_detectron/config.pbtxt``): input ``input__00`` FP32 NCHW
    [3, 640, 480] RGB 0..255 (the model normalises), outputs ``bboxex__0`` FP32
    [-1, 4] (xyxy, input pixels), ``classes__1`` INT64 [-1], ``scores__2`` FP32
    [-1], ``dims__3`` INT64 [1, 2] (input H, W).  GPU: fp32 like the reference's
    libtorch model (``config.pbtxt:7,16`` TYPE_FP32; split-product MFMA convs, fp32
    activations, GroupNorm and decode), as captured batch plans (1 / 4) with the
    normalisation folded into the input-layout kernel; ``precision="bf16"`` is the
    faster secondary mode."""

    platform = "pytorch_libtorch"

    def __init__(self, name: str = "test_model", arch: str = "retinanet", hw=(640, 480), nc: int = 80,
                 device="auto", weights: Optional[str] = None, seed: int = 0, calibrate_target: float = 300.0,
                 precision: str = "fp32", batch: int = 4):
        from ..config.detectron import DetectronConfig

        super().__init__(name)
        self.cfg = DetectronConfig(arch=arch, input_hw=tuple(hw), num_classes=nc)
        self.device = _device(device)
        self.weights, self.seed, self.calibrate_target = weights, seed, calibrate_target
        self.precision, self.batch = precision, batch

    def inputs(self):
        H, W = self.cfg.input_hw
        return [tensor_spec("input__00", "FP32", [3, H, W], fmt="NCHW")]

    def outputs(self):
        return [tensor_spec("bboxex__0", "FP32", [-1, 4], output=True),
                tensor_spec("classes__1", "INT64", [-1], output=True),
                tensor_spec("scores__2", "FP32", [-1], output=True),
                tensor_spec("dims__3", "INT64", [1, 2], output=True)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_GPU if self.device.type == "cuda" else mc.ModelInstanceGroup.KIND_CPU

    def load(self):
        from ..models.common import fuse_model
        from ..models.detectron import build_detectron

        model = build_detectron(self.cfg, self.seed)
        if self.weights:
            model.load_state_dict(load_state_dict(self.weights, getattr(self, "weights_sha256", None)))
        if self.device.type == "cuda":
            from ..pipelines.detectron import DetectronPipeline
            from ..utils.synthetic import camera_frame

            H, W = self.cfg.input_hw
            self.pipe = DetectronPipeline(model, batch=1, src_hw=(H, W), device=self.device, mode="stretch",
                                          precision=self.precision)
            if not self.weights:
                self.pipe.frames[0].copy_(torch.from_numpy(camera_frame(H, W, self.seed)))
                self.pipe.calibrate_detection_density(self.calibrate_target)
            self.model = self.pipe.model
            sizes = sorted({b for b in (1, 4) if b <= max(1, self.batch)} | {max(1, self.batch)})
            self.plans = {b: _DetectronPlan(self.pipe, b, self.device) for b in sizes}
            self.dynamic_batch = max(sizes)
        else:
            self.model = fuse_model(model.eval())
        self.ready = True

    @torch.no_grad()
    def execute(self, inputs, requested):
        H, W = self.cfg.input_hw
        if self.device.type == "cuda":
            return self.plans[1].run([inputs["input__00"]])[0]
        from ..models.detectron import decode_reference

        x = np.require(inputs["input__00"], np.float32, ["C", "W"]).reshape(1, 3, H, W)
        bx, sc, cl = decode_reference(self.model(torch.from_numpy(x)), self.cfg)[0]
        return {"bboxex__0": np.asarray(bx, np.float32).reshape(-1, 4),
                "classes__1": np.asarray(cl).astype(np.int64),
                "scores__2": np.asarray(sc, np.float32),
                "dims__3": np.array([[H, W]], np.int64)}

    @torch.no_grad()
    def execute_batch(self, batch, requested):
        if self.device.type != "cuda":
            return [self.execute(x, requested) for x in batch]
        return _pick(self.plans, len(batch)).run([x["input__00"] for x in batch])


class YoloV4Model(ServedModel):
    """``YOLOv4`` (examples/YOLOv4/config.pbtxt): input ``input`` FP32 NCHW
    [3, 512, 512] (reshape [1, 3, 512, 512], RGB / 255); outputs ``confs`` FP32
    [1, N, 80] and ``boxes`` FP32 [1, N, 1, 4] (normalised x1y1x2y2) with
    N = 16128 — what the reference's ONNX export (decode inside) returns.  GPU:
    CSPDarknet53-SPP-PANet on the fused convs + the K5 decode kernel."""

    platform = "onnxruntime_onnx"

    def __init__(self, name: str = "YOLOv4", nc: int = 80, img: int = 512, device="auto",
                 weights: Optional[str] = None, seed: int = 0, calibrate_target: float = 100.0):
        super().__init__(name)
        self.nc, self.img = nc, img
        self.device = _device(device)
        self.weights, self.seed, self.calibrate_target = weights, seed, calibrate_target
        from ..models.yolov4 import YoloV4Config
        self.N = YoloV4Config(nc=nc, img=(img, img)).num_predictions()

    def inputs(self):
        return [tensor_spec("input", "FP32", [3, self.img, self.img], fmt="NCHW", reshape=[1, 3, self.img, self.img])]

    def outputs(self):
        return [tensor_spec("confs", "FP32", [1, self.N, self.nc], output=True),
                tensor_spec("boxes", "FP32", [1, self.N, 1, 4], output=True)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_GPU if self.device.type == "cuda" else mc.ModelInstanceGroup.KIND_CPU

    def load(self):
        from ..models.common import fuse_model
        from ..models.yolov4 import build_yolov4

        model = build_yolov4(self.nc, self.img, self.seed)
        if self.weights:
            model.load_state_dict(load_state_dict(self.weights, getattr(self, "weights_sha256", None)))
        if self.device.type == "cuda":
            from ..pipelines.yolov4 import Yolov4Pipeline
            from ..utils.synthetic import camera_frame

            self.pipe = Yolov4Pipeline(model, batch=1, src_hw=(self.img, self.img), img=self.img, nc=self.nc,
                                       device=self.device)
            if not self.weights:
                self.pipe.frames[0].copy_(torch.from_numpy(camera_frame(self.img, self.img, self.seed)))
                self.pipe.calibrate_detection_density(self.calibrate_target)
            self.model = self.pipe.model
        else:
            self.model = fuse_model(model.eval())
        self.ready = True

    @torch.no_grad()
    def execute(self, inputs, requested):
        x = np.require(inputs["input"], np.float32, ["C", "W"]).reshape(1, 3, self.img, self.img)
        if self.device.type == "cuda":
            p = self.pipe
            f = p.fast or p.build_fast()
            f.x.t.zero_()
            f.x.t[..., :3].copy_(torch.from_numpy(x).to(self.device).permute(0, 2, 3, 1))
            _, boxes, confs = p.post(f.forward(), full=True)
            boxes, confs = boxes.cpu().numpy(), confs.cpu().numpy()
        else:
            from ..models.yolov4 import decode_reference

            b, c = decode_reference(self.model(torch.from_numpy(x)), self.nc)
            boxes, confs = b.numpy(), c.numpy()
        return {"confs": confs.astype(np.float32, copy=False), "boxes": boxes.astype(np.float32, copy=False)}
