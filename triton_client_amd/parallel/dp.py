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
  its own PCIe link; only the detections travel over RCCL.  With 8 GPUs this
  removes rank 0's PCIe link as the bottleneck (8 × 64 GB/s instead of 1 ×).
  The live drivers' data-parallel detectors (:mod:`.ring_dp`) work this way:
  the sensor process (rank 0) writes each node batch into a POSIX shared-
  memory ring that every rank page-locks (:mod:`.host_ring`).
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
    if world > 1:
        # before the first GPU call: threads and pinned memory of this rank stay on its GPU's socket
        from .numa import bind_to_gpu
        bind_to_gpu(local)
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


# ----------------------------------------------------------------------------- rank failure detection


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


# the data-parallel live detectors: node batches through the shared host ring, detections over RCCL
from .ring_dp import DataParallelDetector2D, DataParallelDetector3D  # noqa: E402,F401
