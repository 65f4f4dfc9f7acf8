"""Frame-level data parallelism: one process per GPU, RCCL over xGMI.

The reference has no parallelism at all (one frame, one blocking RPC —
SURVEY §2.5).  Here sensor frames are batched and spread over the GPUs of a
node; detections are gathered back to the publishing rank.

Communication pattern (no reductions are needed, so no rings):

* ``scatter``: rank 0 → every peer, one grouped p2p send/recv per tensor set
  (``batch_isend_irecv`` → ``ncclGroupStart/End``): xGMI is point-to-point,
  7 links per MI355X, so a grouped scatter drives all links concurrently
  instead of serialising a ring.
* ``gather``: every peer → rank 0, fixed-size padded detection buffers
  (tens to hundreds of KB per rank: latency-bound), grouped the same way.

Two ingest modes (bench ``--ingest``):

* ``rccl``  — all sensor payloads enter through rank 0's host link (e.g. a
  single capture card / NIC), H2D once, then the grouped xGMI scatter.
* ``local`` — each rank pulls its own share of the node's sensor batch over
  its own PCIe link (host ring shared by the sensor process); only the
  detections travel over RCCL.  With 8 GPUs this removes rank 0's PCIe link
  as the bottleneck (8 × 64 GB/s instead of 1 ×).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int
    world: int
    local_rank: int
    device: torch.device

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> DistInfo:
    """One process per GPU.  ``TCA_DIST_BACKEND=gloo`` (rehearsal only) runs the
    GPU path with host-staged gloo transfers, so several ranks can share one
    GPU (RCCL refuses two ranks on one device): it exercises every DP code path
    of the bench and drivers except RCCL itself."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = backend or os.environ.get("TCA_DIST_BACKEND") or None
    if torch.cuda.is_available():
        if backend == "gloo":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if device.type == "cuda" else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistInfo(rank, world, local, device)


class FrameExchange:
    """Grouped p2p scatter/gather of fixed-shape tensor sets.

    ``native``: a :class:`~triton_client_amd.parallel.rccl.NativeComm`; the
    plan is then issued as one C++ RCCL group on the current stream instead of
    through ``batch_isend_irecv`` (GPU tensors only)."""

    def __init__(self, info: DistInfo, group=None, native=None):
        self.info = info
        self.group = group
        self.native = native

    def _run(self, ops, strict: bool = True) -> set:
        """ops: (0 send | 1 recv, tensor, peer).  Every op is waited for, even
        after one fails, so no operation of this call is left in flight.
        strict: raise on the first failed peer; else return the failed peers
        (the DP detectors' retry path)."""
        if not ops:
            return set()
        if self.native is not None:
            self.native.group_p2p(ops)
            return set()
        staged = []
        if dist.get_backend(self.group) == "gloo":  # gloo moves host tensors: stage device ones
            host = []
            for k, t, p in ops:
                if t.is_cuda:
                    h = t.cpu() if k == 0 else torch.empty(t.shape, dtype=t.dtype)
                    if k == 1:
                        staged.append((h, t, p))
                    t = h
                host.append((k, t, p))
            ops = host
        p2p = [dist.P2POp(dist.isend if k == 0 else dist.irecv, t, p, self.group) for k, t, p in ops]
        failed, err = set(), None
        for (k, t, p), w in zip(ops, dist.batch_isend_irecv(p2p)):
            try:
                w.wait()
            except RuntimeError as e:  # a dead / unreachable peer (gloo raises; RCCL would hang: see _DPBase)
                failed.add(p)
                err = err or e
        for h, t, p in staged:
            if p not in failed:
                t.copy_(h)
        if failed and strict:
            raise err
        return failed

    def scatter(self, src: Optional[Sequence[Sequence[torch.Tensor]]], dst: Sequence[torch.Tensor],
                peers: Optional[Sequence[int]] = None, strict: bool = True) -> set:
        """src (rank 0 only): src[i][k] is the k-th tensor for rank peers[i]
        (peers defaults to every rank; peers[0] is rank 0); dst[k] receives
        this rank's share.  Async w.r.t. the host; ordered on the current
        stream."""
        info = self.info
        if info.world == 1:
            for d, s in zip(dst, src[0]):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
            return set()
        peers = list(peers) if peers is not None else list(range(info.world))
        ops = []
        if info.rank == 0:
            for i, r in enumerate(peers[1:], 1):
                ops += [(0, s, r) for s in src[i]]
            for d, s in zip(dst, src[0]):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
        else:
            ops += [(1, d, 0) for d in dst]
        return self._run(ops, strict)

    def gather(self, src: Sequence[torch.Tensor], dst: Optional[Sequence[Sequence[torch.Tensor]]],
               peers: Optional[Sequence[int]] = None, strict: bool = True) -> set:
        """src: this rank's tensors; dst (rank 0 only): dst[i][k] receives rank
        peers[i]'s k-th tensor (peers defaults to every rank)."""
        info = self.info
        if info.world == 1:
            for d, s in zip(dst[0], src):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
            return set()
        peers = list(peers) if peers is not None else list(range(info.world))
        ops = []
        if info.rank == 0:
            for i, r in enumerate(peers[1:], 1):
                ops += [(1, d, r) for d in dst[i]]
            for d, s in zip(dst[0], src):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
        else:
            ops += [(0, s, 0) for s in src]
        return self._run(ops, strict)


def barrier(info: DistInfo) -> None:
    if info.world > 1:
        if info.device.type == "cuda" and dist.get_backend() != "gloo":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def allreduce_max(info: DistInfo, value: float) -> float:
    if info.world == 1:
        return value
    dev = "cpu" if dist.get_backend() == "gloo" else info.device
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- host-level DP detectors
_STOP = -1


class HealthMonitor:
    """Rank-failure detection for the host-level DP detectors.

    Every rank's background thread bumps a heartbeat counter in the c10d
    TCPStore (its own client connection, independent of the RCCL / gloo data
    plane, so a wedged communicator does not hide liveness).  Rank 0 declares a
    rank dead when its counter has not moved for ``timeout`` seconds of rank
    0's own monotonic clock (no cross-host clock comparison).  Detects crashed
    or killed processes; a rank whose process lives but whose serve loop hangs
    keeps beating (the per-step exception path below covers broken links)."""

    PREFIX = "tca_hb/"

    def __init__(self, info: DistInfo, interval: float = 0.25, timeout: float = 2.0, store=None):
        import threading
        import time

        self.info, self.interval, self.timeout = info, interval, timeout
        self._time = time
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        self.store = store or dist.TCPStore(host, port, info.world, is_master=False,
                                            timeout=datetime.timedelta(seconds=30), wait_for_workers=False)
        self.dead: set = set()
        self._seen = {}  # rank -> (counter, monotonic time it last changed)
        self._beats = 0
        self._stop = threading.Event()
        self.store.set(self._key(info.rank), "0")
        self._thread = threading.Thread(target=self._run, name="tca-heartbeat", daemon=True)
        self._thread.start()

    def _key(self, r: int) -> str:
        return f"{self.PREFIX}{r}"

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            self._beats += 1
            try:
                self.store.set(self._key(self.info.rank), str(self._beats))
            except Exception:  # store gone (rank 0 exited): stop beating
                return

    def alive(self) -> List[int]:
        """Rank 0: the ranks currently considered alive (always includes 0)."""
        now = self._time.monotonic()
        for r in range(1, self.info.world):
            if r in self.dead:
                continue
            try:
                v = int(self.store.get(self._key(r))) if self.store.check([self._key(r)]) else -1
            except Exception:
                v = -1
            last = self._seen.get(r)
            if last is None or v != last[0]:
                self._seen[r] = (v, now)
            elif now - last[1] > self.timeout:
                self.dead.add(r)
        return [0] + [r for r in range(1, self.info.world) if r not in self.dead]

    def wait_for_change(self, before: Sequence[int]) -> List[int]:
        """After a failed step: poll until some participant is declared dead
        (up to 2x timeout); returns the new live set (unchanged if none died)."""
        t_end = self._time.monotonic() + 2 * self.timeout + self.interval
        while self._time.monotonic() < t_end:
            now = self.alive()
            if len(now) < len(before):
                return now
            self._time.sleep(self.interval)
        return self.alive()

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=2 * self.interval + 1)


_HDR = 16  # header ints: [seq, payload fields..., participant bitmask]


class _DPBase:
    """Rank 0 calls ``detect(items)``; every other rank calls ``serve()``,
    which runs until rank 0 calls ``close()``.  Work is split into
    contiguous equal shards (padded) over the participating ranks, scattered
    with grouped p2p, run by each rank's local engine ON THE DEVICE (the
    shard the exchange landed in GPU memory goes straight into the engine's
    pipeline buffers: no host round trip on any rank), and gathered back as
    fixed-size padded device buffers.

    Failure handling (gloo transport; an RCCL peer that dies hangs the
    communicator instead of raising, so under RCCL a dead rank surfaces
    through :class:`HealthMonitor` / ``NativeComm.async_error`` and the job is
    restarted): every step carries a sequence number in its header, every
    peer echoes it in its gather payload and rank 0 checks it; rank 0 waits
    for EVERY scatter / gather operation of a step even after one peer has
    failed, so a failed step leaves no operation in flight and no stale
    payload queued (each survivor has consumed its shard and delivered its
    detections); then the shards are re-split over the survivors the
    :class:`HealthMonitor` reports and the step is retried with a new
    sequence number."""

    def __init__(self, local, info: DistInfo, monitor: Optional[HealthMonitor] = None):
        self.local, self.info = local, info
        self.ex = FrameExchange(info)
        self.names = getattr(local, "names", [])
        self.monitor = monitor
        self.retries = 0
        self.seq = 0
        import threading
        self._lock = threading.Lock()  # one step at a time on the p2p channel (live drivers may call from threads)

    def _participants(self) -> List[int]:
        return self.monitor.alive() if self.monitor is not None else list(range(self.info.world))

    def close(self) -> None:
        if self.info.world > 1 and self.info.is_main:
            self._send_header([_STOP], self._participants())

    def _hdr_dev(self):
        return "cpu" if dist.get_backend() == "gloo" else self.info.device

    def _send_header(self, vals, parts: Sequence[int]) -> List[int]:
        mask = 0
        for r in parts:
            mask |= 1 << r
        v = list(vals) + [0] * (_HDR - len(vals))
        v[_HDR - 1] = mask
        t = torch.tensor(v, dtype=torch.int64, device=self._hdr_dev())
        for r in parts:
            if r != 0:
                dist.send(t, r)
        return v

    def _recv_header(self) -> List[int]:
        t = torch.zeros(_HDR, dtype=torch.int64, device=self._hdr_dev())
        dist.recv(t, 0)
        return [int(x) for x in t.tolist()]

    @staticmethod
    def _workers(hdr) -> List[int]:
        mask = hdr[_HDR - 1]
        return [r for r in range(63) if (mask >> r) & 1]

    def serve(self) -> int:
        """Non-main ranks: process shards until rank 0 closes.  Returns shards done."""
        n = 0
        while True:
            hdr = self._recv_header()
            if hdr[0] == _STOP:
                return n
            self._step(hdr, None)
            n += 1

    def detect(self, items):
        if self.info.world == 1:
            return self.local.detect(items)
        if not items:
            return []
        with self._lock:
            return self._detect_locked(items)

    def _detect_locked(self, items):
        while True:
            parts = self._participants()
            if parts == [0]:
                return self.local.detect(items)  # every peer is gone: degrade to rank 0 alone
            self.seq += 1
            try:
                return self._step(self._send_header([self.seq] + self._make_header(items), parts), items)
            except RuntimeError:
                if self.monitor is None or len(self.monitor.wait_for_change(parts)) == len(parts):
                    raise
                self.retries += 1

    # shared step skeleton ---------------------------------------------------------------
    def _exchange(self, hdr, src, mine, run_local, out_like):
        """scatter ``src`` (rank 0) into ``mine``; ``run_local(valid)`` → this
        rank's padded device outputs (the last one an int32 count vector of
        length per + 1 whose last slot receives the step's sequence number);
        gather them.  Rank 0 returns (gathered, workers, per)."""
        info = self.info
        seq = hdr[0]
        wk = self._workers(hdr)
        nw, me = len(wk), wk.index(info.rank)
        n = hdr[1]
        per = (n + nw - 1) // nw
        strict = not info.is_main
        failed = self.ex.scatter(src, mine, wk, strict=strict)
        valid = max(0, min(per, n - me * per))
        outs = run_local(valid, per)
        outs[-1][per] = seq & 0x7FFFFFFF
        dst = [[torch.empty_like(t) for t in outs] for _ in range(nw)] if info.is_main else None
        failed |= self.ex.gather(outs, dst, wk, strict=strict)
        if not info.is_main:
            return None
        if failed:
            raise RuntimeError(f"DP step {seq}: ranks {sorted(failed)} failed")
        for r, d in zip(wk, dst):
            got = int(d[-1][per])
            if got != seq & 0x7FFFFFFF:
                raise RuntimeError(f"DP step {seq}: rank {r} answered for step {got}")
        return dst, wk, per


class DataParallelDetector2D(_DPBase):
    """Frames (HxWx3 uint8, one size per call) → per-frame [n, 6] detections.
    ``local`` must offer ``detect_device(frames [n, H, W, 3] uint8 GPU) ->
    (dets [n, max_det, 6], count [n])`` on device (LocalDetector2D does) or,
    for CPU engines, ``detect``."""

    def __init__(self, local, info: DistInfo, max_det: int = 300, monitor: Optional[HealthMonitor] = None):
        super().__init__(local, info, monitor)
        self.max_det = max_det

    def _make_header(self, frames):
        H, W = frames[0].shape[:2]
        return [len(frames), H, W]

    def detect(self, items):
        if self.info.world > 1 and items and any(f.shape[:2] != items[0].shape[:2] for f in items):
            groups = {}
            for i, f in enumerate(items):
                groups.setdefault(f.shape[:2], []).append(i)
            out = [None] * len(items)
            for idx in groups.values():  # one step per frame geometry
                for i, d in zip(idx, super().detect([items[i] for i in idx])):
                    out[i] = d
            return out
        return super().detect(items)

    def _local_padded(self, frames_dev: torch.Tensor, valid: int, per: int):
        dev = self.info.device
        pad = torch.zeros((per, self.max_det, 6), dtype=torch.float32, device=dev)
        cnt = torch.zeros((per + 1,), dtype=torch.int32, device=dev)
        if valid == 0:
            return [pad, cnt]
        if hasattr(self.local, "detect_device") and frames_dev.is_cuda:
            d, c = self.local.detect_device(frames_dev[:valid], self.max_det)
            pad[:valid] = d
            cnt[:valid] = c
            return [pad, cnt]
        dets = self.local.detect([frames_dev[i].cpu().numpy() for i in range(valid)])  # CPU engines
        for i, d in enumerate(dets):
            k = min(len(d), self.max_det)
            pad[i, :k] = torch.from_numpy(np.asarray(d[:k], np.float32)).to(dev)
            cnt[i] = k
        return [pad, cnt]

    def _step(self, hdr, frames):
        info = self.info
        n, H, W = hdr[1:4]
        wk = self._workers(hdr)
        nw = len(wk)
        per = (n + nw - 1) // nw
        dev = info.device
        src = None
        if info.is_main:
            buf = torch.zeros((nw, per, H, W, 3), dtype=torch.uint8, pin_memory=dev.type == "cuda")
            for i, f in enumerate(frames):
                buf[i // per, i % per].copy_(torch.from_numpy(np.ascontiguousarray(f[..., :3])))
            buf = buf.to(dev, non_blocking=True)
            src = [[buf[r]] for r in range(nw)]
            mine = [buf[0]]
        else:
            mine = [torch.empty((per, H, W, 3), dtype=torch.uint8, device=dev)]
        res = self._exchange(hdr, src, mine, lambda valid, per_: self._local_padded(mine[0], valid, per_), None)
        if res is None:
            return None
        dst, wk, per = res
        pads = torch.stack([d[0] for d in dst]).cpu().numpy()  # the one D2H of the step: detections only
        cnts = torch.stack([d[1] for d in dst]).cpu().numpy()
        out = []
        for i in range(n):
            r, j = divmod(i, per)
            out.append(pads[r, j, :int(cnts[r, j])])
        return out


class DataParallelDetector3D(_DPBase):
    """PointCloud2 messages (same field layout per call) → per-cloud dicts.
    ``local`` offers ``detect_device(data [n, maxb] uint8 GPU, npts [n],
    layout, max_out) -> (box [n, M, D], score [n, M], label [n, M], count [n])``
    (LocalDetector3D does) or, for CPU engines, ``detect``."""

    def __init__(self, local, info: DistInfo, max_out: int = 500, box_dim: int = 7,
                 monitor: Optional[HealthMonitor] = None):
        super().__init__(local, info, monitor)
        self.max_out, self.box_dim = max_out, box_dim

    def _make_header(self, clouds):
        c0 = clouds[0]
        by = {f.name: f for f in c0.fields}
        names = ("x", "y", "z", "intensity")
        offs = [by[k].offset for k in names]
        dts = [by[k].datatype for k in names]
        maxb = max(len(c.data) for c in clouds)
        return [len(clouds), c0.point_step, maxb] + offs + dts

    def _local_padded(self, data, npts, valid, per, step, offs, dts):
        from ..ros import msgs

        dev = self.info.device
        D, M = self.box_dim, self.max_out
        box = torch.zeros((per, M, D), dtype=torch.float32, device=dev)
        score = torch.zeros((per, M), dtype=torch.float32, device=dev)
        lab = torch.zeros((per, M), dtype=torch.int64, device=dev)
        cnt = torch.zeros((per + 1,), dtype=torch.int32, device=dev)
        if valid == 0:
            return [box, score, lab, cnt]
        fields = [msgs.PointField(k, o, d, 1) for k, o, d in zip(("x", "y", "z", "intensity"), offs, dts)]
        if hasattr(self.local, "detect_device") and data.is_cuda:
            b, s_, l_, c = self.local.detect_device(data[:valid], npts[:valid], fields, step, M)
            box[:valid, :, : b.shape[-1]] = b[..., :D]
            score[:valid], lab[:valid], cnt[:valid] = s_, l_, c
            return [box, score, lab, cnt]
        hb, hn = data.cpu().numpy(), npts.cpu().numpy()  # CPU engines
        local = [msgs.PointCloud2(height=1, width=int(hn[i]), fields=fields, point_step=step,
                                  row_step=step * int(hn[i]), data=hb[i, : int(hn[i]) * step].tobytes())
                 for i in range(valid)]
        for i, p in enumerate(self.local.detect(local)):
            k = min(len(p["pred_scores"]), M)
            box[i, :k] = torch.from_numpy(np.asarray(p["pred_boxes"][:k, :D], np.float32)).to(dev)
            score[i, :k] = torch.from_numpy(np.asarray(p["pred_scores"][:k], np.float32)).to(dev)
            lab[i, :k] = torch.from_numpy(np.asarray(p["pred_labels"][:k], np.int64)).to(dev)
            cnt[i] = k
        return [box, score, lab, cnt]

    def _step(self, hdr, clouds):
        info = self.info
        n, step, maxb = hdr[1:4]
        offs, dts = hdr[4:8], hdr[8:12]
        wk = self._workers(hdr)
        nw = len(wk)
        per = (n + nw - 1) // nw
        dev = info.device
        src = None
        if info.is_main:
            pin = dev.type == "cuda"
            buf = torch.zeros((nw, per, maxb), dtype=torch.uint8, pin_memory=pin)
            npts = torch.zeros((nw, per), dtype=torch.int64, pin_memory=pin)
            for i, c in enumerate(clouds):
                raw = np.frombuffer(c.data, np.uint8)
                buf[i // per, i % per, : raw.size].copy_(torch.from_numpy(raw))
                npts[i // per, i % per] = c.width * c.height
            buf, npts = buf.to(dev, non_blocking=True), npts.to(dev, non_blocking=True)
            src = [[buf[r], npts[r]] for r in range(nw)]
            mine = [buf[0], npts[0]]
        else:
            mine = [torch.empty((per, maxb), dtype=torch.uint8, device=dev),
                    torch.empty((per,), dtype=torch.int64, device=dev)]
        res = self._exchange(hdr, src, mine,
                             lambda valid, per_: self._local_padded(mine[0], mine[1], valid, per_, step, offs, dts),
                             None)
        if res is None:
            return None
        dst, wk, per = res
        hb = [torch.stack([d[k] for d in dst]).cpu().numpy() for k in range(4)]
        out = []
        for i in range(n):
            r, j = divmod(i, per)
            k = int(hb[3][r, j])
            out.append({"pred_boxes": hb[0][r, j, :k], "pred_scores": hb[1][r, j, :k], "pred_labels": hb[2][r, j, :k]})
        return out
