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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if torch.cuda.is_available():
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
    """Grouped p2p scatter/gather of fixed-shape tensor sets."""

    def __init__(self, info: DistInfo, group=None):
        self.info = info
        self.group = group

    def scatter(self, src: Optional[Sequence[Sequence[torch.Tensor]]], dst: Sequence[torch.Tensor]) -> None:
        """src (rank 0 only): src[r][k] is the k-th tensor for rank r; dst[k]
        receives this rank's share.  Async w.r.t. the host; ordered on the
        current stream."""
        info = self.info
        if info.world == 1:
            for d, s in zip(dst, src[0]):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
            return
        ops = []
        if info.rank == 0:
            for r in range(1, info.world):
                for s in src[r]:
                    ops.append(dist.P2POp(dist.isend, s, r, self.group))
            for d, s in zip(dst, src[0]):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
        else:
            for d in dst:
                ops.append(dist.P2POp(dist.irecv, d, 0, self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()

    def gather(self, src: Sequence[torch.Tensor], dst: Optional[Sequence[Sequence[torch.Tensor]]]) -> None:
        """src: this rank's tensors; dst (rank 0 only): dst[r][k] receives rank r's k-th tensor."""
        info = self.info
        if info.world == 1:
            for d, s in zip(dst[0], src):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
            return
        ops = []
        if info.rank == 0:
            for r in range(1, info.world):
                for d in dst[r]:
                    ops.append(dist.P2POp(dist.irecv, d, r, self.group))
            for d, s in zip(dst[0], src):
                if d.data_ptr() != s.data_ptr():
                    d.copy_(s, non_blocking=True)
        else:
            for s in src:
                ops.append(dist.P2POp(dist.isend, s, 0, self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()


def barrier(info: DistInfo) -> None:
    if info.world > 1:
        if info.device.type == "cuda":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def allreduce_max(info: DistInfo, value: float) -> float:
    if info.world == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
