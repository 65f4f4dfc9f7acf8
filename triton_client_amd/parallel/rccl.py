"""Native RCCL communicator (``csrc/runtime/rccl_comm.cpp``) for the DP hot path.

``torch.distributed`` bootstraps the job (rendezvous, the c10d store, the
default RCCL process group).  The frame scatter / detection gather then go
through a second RCCL communicator owned by C++: a whole grouped p2p plan is
one ``ncclGroupStart .. ncclGroupEnd`` issued on the caller's HIP stream, with
no per-op Python objects or work handles ("a C++ RCCL
communicator built from the same unique id").  Being plain stream work, the
plan can be captured into a hipGraph.

Failure detection: :meth:`NativeComm.async_error` polls
``ncclCommGetAsyncError`` (SURVEY §5.3 "RCCL async error check plus a
heartbeat"); :meth:`abort` tears the communicator down without waiting for a
dead peer.

The reference has no multi-GPU code at all; parity is with the
design in SURVEY §5.8, not with a reference file.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _native

SEND, RECV = 0, 1
_IN_PROGRESS = 7  # ncclInProgress (non-blocking communicators only)


class RcclError(RuntimeError):
    pass


class NativeComm:
    """One RCCL communicator over every rank of the default process group."""

    def __init__(self, rank: int, world: int, group=None):
        lib = _native.runtime()
        self.lib, self.rank, self.world = lib, rank, world
        nb = lib.tca_rccl_unique_id_bytes()
        uid = ctypes.create_string_buffer(nb)
        if rank == 0:
            self._check(lib.tca_rccl_get_unique_id(uid), "ncclGetUniqueId")
        obj = [uid.raw if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(obj, src=0, group=group)
        raw = ctypes.create_string_buffer(obj[0], nb)
        self._comm = ctypes.c_void_p()
        self._check(lib.tca_rccl_comm_init(ctypes.byref(self._comm), world, raw, rank), "ncclCommInitRank")

    @classmethod
    def from_info(cls, info) -> "NativeComm":
        return cls(info.rank, info.world)

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self.lib.tca_rccl_error_string(rc)
            raise RcclError(f"{what}: {msg.decode() if msg else rc} ({rc})")

    @staticmethod
    def _stream(stream) -> int:
        return _native.stream_ptr(stream)

    def group_p2p(self, ops: Sequence[Tuple[int, torch.Tensor, int]], stream=None) -> None:
        """ops: (SEND | RECV, contiguous device tensor, peer rank); issued as one
        RCCL group on ``stream`` (default: the current stream)."""
        n = len(ops)
        if n == 0:
            return
        for _, t, p in ops:
            if not t.is_contiguous() or t.device.type != "cuda":
                raise ValueError("native p2p needs contiguous GPU tensors")
            if not 0 <= p < self.world:
                raise ValueError(f"peer {p} outside world {self.world}")
        kinds = (ctypes.c_int * n)(*[k for k, _, _ in ops])
        peers = (ctypes.c_int * n)(*[p for _, _, p in ops])
        bufs = (ctypes.c_void_p * n)(*[t.data_ptr() for _, t, _ in ops])
        nbytes = (ctypes.c_int64 * n)(*[t.numel() * t.element_size() for _, t, _ in ops])
        self._check(self.lib.tca_rccl_group_p2p(self._comm, n, kinds, peers, bufs, nbytes, self._stream(stream)),
                    "grouped send/recv")

    def allreduce_max_(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        """In-place MAX all-reduce of a float64 GPU tensor."""
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("allreduce_max_ needs a contiguous float64 GPU tensor")
        self._check(self.lib.tca_rccl_allreduce_max_f64(self._comm, t.data_ptr(), t.numel(), self._stream(stream)),
                    "ncclAllReduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("broadcast_ needs a contiguous GPU tensor")
        self._check(self.lib.tca_rccl_broadcast(self._comm, t.data_ptr(), t.numel() * t.element_size(), root,
                                                self._stream(stream)), "ncclBroadcast")
        return t

    def count(self) -> int:
        """Ranks RCCL built this communicator over (ncclCommCount)."""
        n = ctypes.c_int(0)
        self._check(self.lib.tca_rccl_comm_count(self._comm, ctypes.byref(n)), "ncclCommCount")
        return int(n.value)

    def async_error(self) -> Optional[str]:
        """None while healthy, else the RCCL error string (a peer died, a link broke)."""
        rc = self.lib.tca_rccl_async_error(self._comm)
        if rc in (0, _IN_PROGRESS):
            return None
        msg = self.lib.tca_rccl_error_string(rc)
        return msg.decode() if msg else str(rc)

    def abort(self) -> None:
        if self._comm:
            self.lib.tca_rccl_comm_abort(self._comm)
            self._comm = ctypes.c_void_p()

    def close(self) -> None:
        if self._comm:
            self._check(self.lib.tca_rccl_comm_destroy(self._comm), "ncclCommDestroy")
            self._comm = ctypes.c_void_p()


def native_selftest(comm: "NativeComm", rank: int, world: int, timeout_s: float = 60.0) -> Tuple[bool, str]:
    """Exercise the DP step's detection-gather pattern on ``comm`` before the real step uses it:
    every rank sends two small tensors to rank 0 as one grouped p2p plan, first eagerly, then
    captured into two hipGraphs (the double-buffered step's layout: one plan per graph over the
    one communicator) replayed alternately three times.  Rank 0 checks every received value.
    Each phase is waited for by polling an event; past ``timeout_s`` the communicator is aborted
    (its kernels leave their waits) and the test fails, so a caller can fall back to the process
    group's own p2p instead of hanging its first timed step.  Collective: every rank must call it.
    Returns (ok, detail)."""
    import time

    from ..pipelines.graph import GraphRunner

    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.Stream(device=dev)
    src = [torch.zeros(4, 3, device=dev), torch.zeros(4, dtype=torch.int32, device=dev)]
    dst = [[[torch.full_like(t, -1) for t in src] for _ in range(world)] for _ in range(2)] if rank == 0 else None
    vals = torch.zeros(2, device=dev)

    def plan(k):
        if rank == 0:
            ops = [(RECV, d, r) for r in range(world) for d in dst[k][r]]
        else:
            ops = []
        return ops + [(SEND, s, 0) for s in src]

    def wait(what: str) -> Optional[str]:
        ev = torch.cuda.Event()
        ev.record(stream)
        t0 = time.perf_counter()
        while not ev.query():
            if time.perf_counter() - t0 > timeout_s:
                comm.abort()
                return f"{what}: no completion within {timeout_s:.0f} s (communicator aborted)"
            time.sleep(0.001)
        return None

    def check(k: int, v: float) -> Optional[str]:
        if rank != 0:
            return None
        for r in range(world):
            want = v + r
            if float(dst[k][r][0].reshape(-1)[0]) != want or int(dst[k][r][1][0]) != int(want):
                return f"graph {k}: rank {r}'s tensors arrived wrong ({float(dst[k][r][0].reshape(-1)[0])} vs {want})"
        return None

    runs = []
    try:
        with torch.cuda.stream(stream):
            src[0].fill_(1.0 + rank)
            src[1].fill_(1 + rank)
            comm.group_p2p(plan(0))
        err = wait("eager grouped p2p")
        if err is None:
            err = check(0, 1.0)
        if err is not None:
            return False, err

        def step(k):
            def fn():
                src[0].copy_((vals[k] + rank).expand_as(src[0]))
                src[1].copy_((vals[k] + rank).to(torch.int32).expand_as(src[1]))
                comm.group_p2p(plan(k))
                return src
            return fn
        with torch.cuda.stream(stream):
            runs = [GraphRunner(step(0)), GraphRunner(step(1))]
            for run in runs:
                run.capture()
        for t, v in enumerate((2.0, 5.0, 9.0)):
            k = t % 2
            with torch.cuda.stream(stream):
                vals[k].fill_(v)
                runs[k]()
            err = wait(f"graph replay {t}") or check(k, v)
            if err is not None:
                return False, err
        return True, "eager and two-graph grouped p2p gather delivered"
    except Exception as e:  # noqa: BLE001 - reported to the caller, which falls back
        return False, f"{type(e).__name__}: {e}"
    finally:
        for r in runs:  # the graphs go before the communicator
            r.release()
