"""Data-parallel live detectors over the node's shared host ring.

Rank 0 runs the ROS driver (:class:`~triton_client_amd.inference.ros_inference.RosInference`
/ ``RosInference3D``) with one of these in place of the local engine; every
other rank runs :meth:`serve`.  A node step:

1. rank 0 writes the batch's raw message payloads (JPEG bytes, rgb8 rows,
   PointCloud2 records) and an item table into the next ring slot
   (:mod:`.host_ring`) and publishes the slot's sequence number;
2. every participant takes its contiguous shard out of the shared, page-locked
   slot over its own PCIe link and runs the same device path as a single GPU
   (:mod:`~triton_client_amd.inference.live`: its own JPEG entropy decode on
   its own cores, double-buffered graphs, GPU annotation) — annotated frames
   are DMA'd straight back into the slot's output area;
3. the detections — the engines' fixed-shape device result buffers — are
   gathered to rank 0 over RCCL (:class:`~triton_client_amd.parallel.rccl.NativeComm`
   grouped p2p, on a comm stream behind each rank's replay) or, in the
   one-GPU gloo rehearsal, host-staged gloo;
4. every participant acknowledges the slot; rank 0 assembles the per-message
   results (published ``Image`` messages wrap the slot's output area without a
   copy; a slot whose output is still viewed by held messages is not
   rewritten — rank 0 moves on to a fresh data generation instead, and the old
   mapping lives as long as those messages, so a consumer that holds messages
   can never stall the ring).

Nothing but sequence numbers and detections crosses process boundaries
outside the shared mapping: no per-step ``dist.send`` headers, no node batch
on rank 0's GPU, no per-step pinned allocations.  Engines without a device
path (CPU) run the same protocol with host results gathered over gloo.

Failure handling: each step carries its sequence number in the gather (a
stale payload is detected); with a :class:`~triton_client_amd.parallel.dp.HealthMonitor`
a failed step (gloo raises; RCCL peers are watched by the heartbeat) is
re-split over the surviving ranks and retried under a new sequence number.

Reference: none — the reference runs one blocking RPC per frame
(``communicator/ros_inference.py:147``); BASELINE.json configs 3 and 5 ask for
"batched DP scatter/gather over 8xMI355X".
"""
from __future__ import annotations

import logging
import os
import threading
import time
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..ros import msgs
from .dp import DistInfo, FrameExchange, HealthMonitor
from .host_ring import MAX_ITEMS, HostRing

KIND_STOP, KIND_JPEG, KIND_FRAMES, KIND_CLOUDS = -1, 1, 2, 3
# header ints
H_SEQ, H_KIND, H_N, H_GEN, H_SLOT, H_MASK, H_PER, H_DRAW, H_KEY = 0, 1, 2, 3, 4, 5, 6, 7, 8
H_CALIB = 60  # 1: rank 0 broadcasts its freshly calibrated weights in this step (every rank joins)
H_FILE = 61  # 1: file-sourced items read from the slot's path (sharded replay)
# item ints: in_off, in_size, out_off, out_size, meta0, meta1, in_src (0: the slot, 1: the ingest arena,
# 2: the step's source file -- in_off is then the payload's offset in that file)
I_IN, I_INSZ, I_OUT, I_OUTSZ, I_M0, I_M1, I_SRC = range(7)
SRC_SLOT, SRC_ARENA, SRC_FILE = 0, 1, 2
_ALIGN = 4096

log = logging.getLogger("triton_client_amd.ring_dp")


# rank 0's ring copy threads: 8 measured fastest on the 256-CPU box (147.5 GB/s vs 137.1 at 16 and 119.6
# at 32: one socket's memory bandwidth, profiles/r5/fanout/fanout_raw675.json)
COPY_THREADS = int(os.environ.get("TCA_RING_COPY_THREADS", "8"))
# rank 0's ingest arena (host_ring.IngestArena) in MiB when world > 1: deserialisers write payloads
# straight into it and the ring step copies nothing; 0 turns it off (every payload copied into the slot)
ARENA_MB = int(os.environ.get("TCA_RING_ARENA_MB", "512"))
# sharded replay: payloads that are views of a mapped file (a bag, host_ring.FileMaps) travel as file
# offsets and every rank reads its own shard from the file; 0 copies them into the slots like any payload
FILE_SHARD = os.environ.get("TCA_RING_FILE_SHARD", "1") != "0"

def _align(n: int) -> int:
    return (int(n) + _ALIGN - 1) // _ALIGN * _ALIGN


class RingStepError(RuntimeError):
    pass


class ReplicaMismatch(Exception):
    """The replicas' weights differ: a configuration error, never retried."""


class _Rechunk(Exception):
    """Fewer live ranks than the chunk was cut for: cut it again."""


class _RingDP:
    """Shared protocol; subclasses define the message kinds and the local run."""

    def __init__(self, local, info: DistInfo, monitor: Optional[HealthMonitor] = None, nslots: int = 4,
                 comm=None, ack_timeout_s: float = 120.0, arena_mb: Optional[int] = None):
        self.local, self.info, self.monitor = local, info, monitor
        self.names = list(getattr(local, "names", []) or [])
        self.ex = FrameExchange(info, native=comm)
        self.nslots = nslots
        self.retries = 0
        self.seq = 0
        self.steps = 0
        self.arena_items = self.copied_items = 0  # rank 0: payloads read from the arena / copied into slots
        self.ack_timeout_s = ack_timeout_s
        self._lock = threading.Lock()
        self.gpu = (getattr(getattr(local, "device", None), "type", "cpu") == "cuda"
                    and callable(getattr(local, "live", None)))
        self._comm_stream = torch.cuda.Stream(info.device) if self.gpu else None
        name = [f"tca_ring_{os.getpid()}_{id(self) & 0xffffff:x}" if info.is_main else None]
        if info.world > 1:
            dist.broadcast_object_list(name, src=0)
        if info.is_main:
            arena = (ARENA_MB if arena_mb is None else int(arena_mb)) << 20 if info.world > 1 else 0
            self.ring = HostRing(name[0], nslots, info.world, create=True, arena_bytes=arena)
        if info.world > 1:
            dist.barrier()
        if not info.is_main:
            self.ring = HostRing(name[0])
        # rank 0: per slot, (seq, every live rank) of its last use -- every peer reads every
        # slot's header in sequence and acks it, participant or not, so a slot is rewritten
        # only once all of them have; open output leases per (data generation, slot):
        # published Image messages still viewing the slot's output area
        self._slot_use: List[Optional[Tuple[int, List[int]]]] = [None] * nslots
        self._leases: Dict[Tuple[int, int], int] = {}
        self._lease_lock = threading.Lock()
        self._path: Optional[str] = None  # the current step's source file (file-sourced items)
        self.file_items = 0  # rank 0: payloads every rank read from the source file itself

    @property
    def file_sharding(self) -> bool:
        """Bag replays should hand this engine messages whose payloads stay in the mapped
        file (``Bag.read_messages(mapped=True)``): every rank then reads its own shard."""
        return FILE_SHARD and self.info.world > 1

    # ------------------------------------------------------------------ rank 0
    def ingest_buffer(self, nbytes: int) -> Optional[np.ndarray]:
        """Rank 0's deserialisers: a writable ``nbytes`` buffer in the ring's ingest
        arena for a message payload (``rosmsg.deserialize(..., alloc=)``,
        ``Bag.read_messages(..., alloc=)``).  A payload there reaches every rank
        without rank 0 copying it into a slot.  None: no arena (one rank, or
        ``TCA_RING_ARENA_MB=0``) or full -- keep a ``bytes`` payload."""
        arena = self.ring.arena if self.info.is_main else None
        return arena.alloc(nbytes) if arena is not None else None

    def _raw(self, items, i: int, view: np.ndarray) -> np.ndarray:
        """Item i's input bytes: in the slot (``view``) or in the ingest arena."""
        off, n = int(items[i, I_IN]), int(items[i, I_INSZ])
        src = int(items[i, I_SRC])
        if src == SRC_ARENA:
            return self.ring.arena.buf[off:off + n]
        if src == SRC_FILE:  # this rank's own mapping of the source file: read by its own staging copy
            from .host_ring import FileMaps
            return FileMaps.view(self._path)[off:off + n]
        return view[off:off + n]

    def _participants(self) -> List[int]:
        return self.monitor.alive() if self.monitor is not None else list(range(self.info.world))

    def _drain(self, s: int) -> bool:
        """Wait until every rank live at slot s's last step has acked it (peers that
        did not take part still read its header: rewriting it earlier could hand a slow
        peer a newer or half-written header).  Returns False
        if published messages still view the slot's output area in the current
        data generation (the caller then moves to a fresh generation; the old
        mapping lives on under those messages)."""
        use = self._slot_use[s]
        if use is not None:
            seq, parts = use
            self._wait_acks(s, [r for r in parts if r != 0], seq)
            self._slot_use[s] = None
        with self._lease_lock:
            return self._leases.get((self.ring.gen, s), 0) == 0

    def _wait_acks(self, s: int, ranks: List[int], seq: int) -> None:
        end = time.monotonic() + self.ack_timeout_s
        while ranks:
            missing = self.ring.wait_acks(s, ranks, seq, 100)
            if self.monitor is not None:
                dead = self.monitor.dead
                missing = [r for r in missing if r not in dead]
            if not missing:
                return
            if time.monotonic() > end:
                raise RingStepError(f"ranks {missing} did not acknowledge step {seq}")
            ranks = missing

    def _lease(self, s: int, view: np.ndarray) -> None:
        """Slot s of this generation stays reserved until every published view of
        ``view`` is gone."""
        key = (self.ring.gen, s)
        with self._lease_lock:
            self._leases[key] = self._leases.get(key, 0) + 1

        def release(lock=self._lease_lock, leases=self._leases, key=key):
            with lock:
                leases[key] -= 1
                if leases[key] == 0:
                    del leases[key]
        weakref.finalize(view, release)

    def _write_step(self, kind: int, payloads: Sequence, metas: Sequence[Tuple[int, int]], out_sizes: Sequence[int],
                    key: Sequence[int], draw: bool, parts: List[int], per: int,
                    calib: bool = False) -> Tuple[int, int, np.ndarray]:
        """Payloads + item table into the next slot, then publish. -> (seq, slot, items)."""
        from ..inference.live import gather_copy

        n = len(payloads)
        if n > MAX_ITEMS:
            raise ValueError(f"{n} items in one step (max {MAX_ITEMS})")
        self.seq += 1
        seq, s = self.seq, self.seq % self.nslots
        free = self._drain(s)
        sizes = [len(p) if not isinstance(p, np.ndarray) else p.nbytes for p in payloads]
        arena = self.ring.arena
        at = [arena.offset_of(p, z) if arena is not None else None for p, z in zip(payloads, sizes)]
        at = [(SRC_ARENA, a) if a is not None else None for a in at]
        path = None
        if FILE_SHARD:
            from .host_ring import FileMaps
            for i, (p, z) in enumerate(zip(payloads, sizes)):
                if at[i] is None:
                    loc = FileMaps.locate(p, z)
                    if loc is not None and (path is None or loc[0] == path):  # one source file per step
                        path = loc[0]
                        at[i] = (SRC_FILE, loc[1])
        need = sum(_align(z) for z, a in zip(sizes, at) if a is None) + sum(_align(z) for z in out_sizes)
        ring = self.ring
        if ring.data is None or need > ring.data.slot_bytes or not free:
            if ring.data is not None:
                why = "leased" if need <= ring.data.slot_bytes else "grow"
                ring.generation_switches[why] += 1
                if why == "leased":  # a consumer holds published Images of this slot
                    log.warning("host ring %s: slot %d still viewed by published messages: new data generation "
                                "(%d so far; re-pins the ring on every rank)", ring.name, s,
                                ring.generation_switches["leased"])
            for t in range(self.nslots):  # every slot acked before the data area is replaced
                self._drain(t)
            size = max(need + need // 4, 1 << 20, ring.data.slot_bytes if ring.data is not None else 0)
            ring.new_generation(size)
        data = ring.data
        base = s * data.slot_bytes
        items = ring.items(s)
        items[:n] = 0
        off = 0
        copy = []
        for i, (z, (m0, m1), a) in enumerate(zip(sizes, metas, at)):
            items[i, I_INSZ], items[i, I_M0], items[i, I_M1] = z, m0, m1
            if a is not None:  # in the ingest arena / the source file: every rank reads it there
                items[i, I_SRC], items[i, I_IN] = a
            else:
                items[i, I_IN] = off
                copy.append(i)
                off += _align(z)
        for i, z in enumerate(out_sizes):
            items[i, I_OUT], items[i, I_OUTSZ] = off, z
            off += _align(z)
        if copy:
            gather_copy([data.base + base + int(items[i, I_IN]) for i in copy], [payloads[i] for i in copy],
                        [sizes[i] for i in copy], COPY_THREADS)
        nfile = sum(1 for a in at if a is not None and a[0] == SRC_FILE)
        self.file_items += nfile
        self.arena_items += n - len(copy) - nfile
        self.copied_items += len(copy)
        self._path = path
        if path is not None:
            ring.set_path(s, path)
        hdr = ring.header(s)
        hdr[:] = 0
        mask = 0
        for r in parts:
            mask |= 1 << r
        hdr[H_SEQ], hdr[H_KIND], hdr[H_N], hdr[H_GEN], hdr[H_SLOT] = seq, kind, n, ring.gen, data.slot_bytes
        hdr[H_MASK], hdr[H_PER], hdr[H_DRAW] = mask, per, int(draw)
        hdr[H_KEY:H_KEY + len(key)] = key
        hdr[H_CALIB] = int(calib)
        hdr[H_FILE] = int(path is not None)
        ring.publish(s, seq)
        self._slot_use[s] = (seq, self._participants())
        return seq, s, items[:n].copy()

    def close(self) -> None:
        """Rank 0: end every peer's serve() loop (a STOP step), then release the ring."""
        if self.info.is_main:
            with self._lock:
                if self.info.world > 1:
                    parts = self._participants()
                    self.seq += 1
                    s = self.seq % self.nslots
                    self._drain(s)
                    hdr = self.ring.header(s)
                    hdr[:] = 0
                    hdr[H_SEQ], hdr[H_KIND] = self.seq, KIND_STOP
                    self.ring.publish(s, self.seq)
                    try:
                        self._wait_acks(s, [r for r in parts if r != 0], self.seq)
                    except RingStepError:
                        pass
        self.ring.close()

    # ------------------------------------------------------------------ every rank
    def _tag(self, seq: int) -> torch.Tensor:
        """[seq, rank, weights signature (2 x int32)]: rank 0 checks every peer answered this
        step and runs the same weights."""
        dev = self.info.device if self.gpu else "cpu"
        sig = np.array([self._signature()], np.float64).view(np.int32)
        return torch.tensor([seq & 0x7FFFFFFF, self.info.rank, int(sig[0]), int(sig[1])], dtype=torch.int32,
                            device=dev)

    def _signature(self) -> float:
        if getattr(self, "_sig", None) is None:
            model = getattr(self.local, "model", None)
            if model is None or getattr(self.local, "calibrate_target", None) is not None:
                return 0.0  # not built / not calibrated yet
            with torch.no_grad():
                self._sig = float(sum(float(t.double().sum()) for t in model.parameters()))
        return self._sig

    def _calibration_sample(self, hdr, items, view):
        """The node batch's first message (rebuilt from the slot) while the local
        engine still has to set its random-init head prior: every rank calibrates
        on the frame one GPU would have used."""
        if getattr(self.local, "calibrate_target", None) is None:
            return None
        return self._shard_items(hdr, items, view, 0, 1)[0]

    def _gather(self, src: List[torch.Tensor], wk: List[int], like: Optional[List[torch.Tensor]], strict: bool,
                after: Optional[torch.cuda.Event] = None) -> Tuple[Optional[list], set, Optional[torch.cuda.Event]]:
        """Gather src (this rank's tensors) to rank 0 over the workers wk; on a GPU
        engine the collective runs on the comm stream behind ``after``."""
        dst = None
        if self.info.is_main:
            dst = [[torch.empty_like(t) for t in like] for _ in wk]
        if self._comm_stream is None:
            return dst, self.ex.gather(src, dst, wk, strict=strict), None
        cs = self._comm_stream
        if after is not None:
            cs.wait_event(after)
        with torch.cuda.stream(cs):
            failed = self.ex.gather(src, dst, wk, strict=strict)
            ev = torch.cuda.Event()
            ev.record(cs)
        return dst, failed, ev

    def serve(self, max_steps: Optional[int] = None) -> int:
        """Non-main ranks: run every step rank 0 publishes until it closes.
        Returns the steps this rank took part in."""
        done = 0
        ring = self.ring
        seq = 0
        while max_steps is None or done < max_steps:
            seq += 1
            s = seq % self.nslots
            while not ring.wait_ready(s, seq, 1000):
                pass
            hdr = ring.header(s).copy()
            if hdr[H_SEQ] != seq:
                raise RingStepError(f"slot {s}: step {int(hdr[H_SEQ])}, expected {seq}")
            if hdr[H_KIND] == KIND_STOP:
                ring.ack(s, self.info.rank, seq)
                return done
            if hdr[H_CALIB]:  # rank 0 calibrated its random-init weights: take them (every rank)
                self._adopt_weights(hdr)
            mask = int(hdr[H_MASK])
            self._path = ring.path(s) if hdr[H_FILE] else None
            if (mask >> self.info.rank) & 1:
                data = ring.use_generation(int(hdr[H_GEN]), int(hdr[H_SLOT]))
                items = ring.items(s)[:int(hdr[H_N])].copy()
                self._serve_step(hdr, items, data.slot(s))
                done += 1
            ring.ack(s, self.info.rank, seq)
        return done

    @staticmethod
    def _workers(mask: int) -> List[int]:
        return [r for r in range(64) if (mask >> r) & 1]

    def _shard(self, hdr, wk: List[int]) -> Tuple[int, int]:
        n, per = int(hdr[H_N]), int(hdr[H_PER])
        me = wk.index(self.info.rank)
        return min(n, me * per), min(n, (me + 1) * per)

    def _needs_calibration(self) -> bool:
        """A device engine whose random-init head prior is still to be set.  The GPU
        calibration (LSUV statistics through the PyTorch modules) is not bit-reproducible
        across processes, so on the device path only rank 0 calibrates — on the node
        batch's first frame, as one GPU does — and broadcasts the resulting weights."""
        return self.gpu and self.info.world > 1 and getattr(self.local, "calibrate_target", None) is not None

    def _broadcast_weights(self) -> None:
        from ..models.common import broadcast_parameters
        broadcast_parameters(self.local.model)
        self._sig = None

    def _adopt_weights(self, hdr) -> None:
        """Peers: fold the model the way rank 0's pipeline did (without calibrating), then
        receive rank 0's weights; engines are built only after this."""
        self.local.calibrate_target = None
        self._model_like_rank0(hdr)
        self._broadcast_weights()

    def _run_step(self, kind, payloads, metas, out_sizes, key, draw, assemble, prebuild=None):
        """Rank 0: one node step with retries; ``assemble(dst, wk, per, items,
        slot_view, own)`` builds the results.  ``prebuild()``: builds (and so calibrates)
        rank 0's engine for this step before it is published."""
        calib = self._needs_calibration()
        if calib:
            prebuild()
        while True:
            parts = self._participants()
            n = len(payloads)
            per = -(-n // len(parts))
            if self._cap_per(per) < per:
                raise _Rechunk()
            wk = parts[:-(-n // per)]
            seq, s, items = self._write_step(kind, payloads, metas, out_sizes, key, draw, wk, per, calib)
            if calib:  # every rank joins this collective as soon as it reads the header
                self._broadcast_weights()
                calib = False
            slot_view = self.ring.data.slot(s)
            try:
                hdr = self.ring.header(s).copy()
                own, src, like, ran = self._local_step(hdr, items, slot_view, wk)
                dst, failed, ev = self._gather(src, wk, like, strict=False, after=ran)
                if failed:
                    raise RingStepError(f"step {seq}: ranks {sorted(failed)} failed")
                self._after_gather(own, ev)
                if ev is not None:
                    ev.synchronize()
                for r, d in zip(wk, dst):
                    tag = d[-1].cpu()
                    if int(tag[0]) != seq & 0x7FFFFFFF or int(tag[1]) != r:
                        raise RingStepError(f"step {seq}: rank {r} answered for step {int(tag[0])}")
                    if (int(tag[2]), int(tag[3])) != (int(dst[0][-1][2]), int(dst[0][-1][3])):
                        raise ReplicaMismatch(f"rank {r} runs different weights than rank 0")
                self._wait_acks(s, [r for r in wk if r != 0], seq)  # their outputs are in the slot
                self.steps += 1
                return assemble(dst, wk, per, items, slot_view, own, s)
            except (RuntimeError, RingStepError):
                if self.monitor is None or len(self.monitor.wait_for_change(parts)) == len(parts):
                    raise
                self.retries += 1

    def _cap_per(self, per: int) -> int:
        """Items a rank takes per step: a device engine runs one batch of B."""
        B = int(getattr(self, "B", 0) or 0)
        return min(per, B) if (self.gpu and B) else per

    def _chunk(self, n: int) -> int:
        """Items of the next step: one engine batch per live rank."""
        B = int(getattr(self, "B", 0) or 0)
        return min(n, B * len(self._participants())) if (self.gpu and B) else n

    def _after_gather(self, own, ev) -> None:
        pass


# ============================================================================ camera
class DataParallelDetector2D(_RingDP):
    """Camera frames over the node's GPUs.  ``live().process(messages, draw,
    names)`` is the drivers' interface (same as :class:`~triton_client_amd.inference.live.LiveCamera`);
    ``detect(frames)`` takes HxWx3 uint8 arrays.  ``local`` is a
    :class:`~triton_client_amd.inference.engines.LocalDetector2D` (device path) or
    any engine with ``detect(frames)`` (host path, e.g. CPU)."""

    def __init__(self, local, info: DistInfo, max_det: int = 300, monitor: Optional[HealthMonitor] = None,
                 nslots: int = 4, comm=None, arena_mb: Optional[int] = None):
        super().__init__(local, info, monitor, nslots, comm, arena_mb=arena_mb)
        self.max_det = max_det
        self.B = int(getattr(local, "B", 0) or 0)

    def live(self):
        return self

    # ------------------------------------------------------------------ rank 0
    def detect(self, frames: Sequence[np.ndarray]) -> List[np.ndarray]:
        from ..ros import compat

        ims = [compat.numpy_to_imgmsg(np.ascontiguousarray(f[..., :3]), "rgb8") for f in frames]
        return [d for _, d in self.process(ims, draw=False)]

    def process(self, messages: Sequence, draw: bool = True, names: Optional[Sequence[str]] = None) -> List[tuple]:
        """Messages -> [(Image, dets [n, 6])] in message order (rank 0)."""
        if not messages:
            return []
        if self.info.world == 1:
            if self.gpu:
                return self.local.live().process(messages, draw, names)
            return self._host_only(messages, draw)
        with self._lock:
            groups: Dict[tuple, List[int]] = {}
            prepared = [self._prepare(m) for m in messages]
            for i, (key, _, _) in enumerate(prepared):
                groups.setdefault(key, []).append(i)
            out: List[Optional[tuple]] = [None] * len(messages)
            for key, idx in groups.items():
                while idx:
                    chunk = idx[:self._chunk(len(idx))]
                    try:
                        res = self._step_camera(key, [prepared[i][1] for i in chunk], [messages[i] for i in chunk],
                                                draw)
                    except _Rechunk:
                        continue
                    for i, r in zip(chunk, res):
                        out[i] = r
                    idx = idx[len(chunk):]
            return out

    def _prepare(self, m):
        """(key, payload) for the ring: (KIND_JPEG, H, W) with the JPEG bytes when the
        device path decodes it, else (KIND_FRAMES, H, W) with rgb8 rows."""
        from ..inference.live import LiveCamera, _is_compressed

        if self.gpu and _is_compressed(m):
            key = self.local.live()._key(m)
            if key[0] == "jpeg":
                return (KIND_JPEG, key[1][0], key[1][1]), m.data, m
        if not _is_compressed(m) and m.encoding == "rgb8" and m.step == 3 * m.width:
            return (KIND_FRAMES, int(m.height), int(m.width)), memoryview(m.data)[:m.height * m.step], m
        rgb = LiveCamera.host_rgb(m)
        return (KIND_FRAMES, rgb.shape[0], rgb.shape[1]), np.ascontiguousarray(rgb), m

    def _host_only(self, messages, draw):
        from ..inference.live import LiveCamera
        from ..ros import compat
        from ..utils.draw import draw_detections

        rgb = [LiveCamera.host_rgb(m) for m in messages]
        dets = self.local.detect(rgb)
        out = []
        for m, f, d in zip(messages, rgb, dets):
            img = draw_detections(f.copy(), d, self.names) if draw else f
            out.append((compat.numpy_to_imgmsg(img, "rgb8", header=m.header), np.asarray(d, np.float32)))
        return out

    def _step_camera(self, key, payloads, messages, draw):
        kind, H, W = key
        frame = H * W * 3
        out_sizes = [frame] * len(payloads) if draw else []
        metas = [(0, 0)] * len(payloads)

        def prebuild():
            live = self.local.live()
            live._engine(live._key(messages[0]), draw, tuple(self.names), messages[0])
        return self._run_step(kind, payloads, metas, out_sizes, (H, W), draw,
                              lambda dst, wk, per, items, view, own, s: self._assemble(
                                  dst, wk, per, items, view, own, s, messages, H, W, draw), prebuild)

    def _model_like_rank0(self, hdr) -> None:
        p = self.local._calibrated_pipeline((int(hdr[H_KEY]), int(hdr[H_KEY + 1])), None)
        del p  # only its BN folding / device placement of the shared model is wanted

    # ------------------------------------------------------------------ every rank
    def _shard_items(self, hdr, items, view, lo, hi):
        return self._shard_messages(hdr, items, view, lo, hi)

    def _shard_messages(self, hdr, items, view, lo, hi):
        kind, H, W = int(hdr[H_KIND]), int(hdr[H_KEY]), int(hdr[H_KEY + 1])
        out = []
        for i in range(lo, hi):
            raw = self._raw(items, i, view)
            if kind == KIND_JPEG:
                out.append(msgs.CompressedImage(format="jpeg", data=memoryview(raw)))
            else:
                out.append(msgs.Image(height=H, width=W, encoding="rgb8", step=3 * W, data=memoryview(raw)))
        return out

    def _local_step(self, hdr, items, view, wk):
        """This rank's shard -> (own pending, gather tensors, rank-0 receive shapes, ran event)."""
        lo, hi = self._shard(hdr, wk)
        seq, draw, per = int(hdr[H_SEQ]), bool(hdr[H_DRAW]), int(hdr[H_PER])
        H, W = int(hdr[H_KEY]), int(hdr[H_KEY + 1])
        batch = self._shard_messages(hdr, items, view, lo, hi)
        if self.gpu:
            live = self.local.live()
            key = live._key(batch[0]) if batch else (("jpeg" if int(hdr[H_KIND]) == KIND_JPEG else "frames"),
                                                     (H, W), None)
            if not batch and key[0] == "jpeg":
                raise RingStepError("empty JPEG shard without a geometry")
            eng = live._engine(key, draw, tuple(self.names), self._calibration_sample(hdr, items, view))
            pend, ran, src = None, None, None
            if batch:
                outs = None
                if draw:
                    outs = [torch.from_numpy(view[int(items[i, I_OUT]):int(items[i, I_OUT]) + H * W * 3]
                                             .reshape(H, W, 3)) for i in range(lo, hi)]
                pend = eng.submit(batch, out_frames=outs)
                ran, src = pend.ticket.ran, list(pend.ticket.stage)
            else:
                src = eng.zero_stage()
            like = eng.zero_stage()
            return (eng, pend), src + [self._tag(seq)], like + [self._tag(0)], ran
        # host engine: padded host results
        from ..inference.live import LiveCamera
        sample = self._calibration_sample(hdr, items, view)
        if sample is not None:
            self.local.detect([LiveCamera.host_rgb(sample)])  # calibrates on the node batch's first frame
        rgb = [LiveCamera.host_rgb(m) for m in batch]
        dets = self.local.detect(rgb) if rgb else []
        pad = torch.zeros((per, self.max_det, 6), dtype=torch.float32)
        cnt = torch.zeros((per,), dtype=torch.int32)
        for j, d in enumerate(dets):
            k = min(len(d), self.max_det)
            pad[j, :k] = torch.from_numpy(np.asarray(d[:k], np.float32).reshape(-1, 6))
            cnt[j] = k
        if draw:
            from ..utils.draw import draw_detections
            for j, (i, f, d) in enumerate(zip(range(lo, hi), rgb, dets)):
                o = view[int(items[i, I_OUT]):int(items[i, I_OUT]) + H * W * 3].reshape(H, W, 3)
                o[...] = f
                draw_detections(o, d, self.names)
        src = [pad, cnt, self._tag(seq)]
        return (None, None), src, [pad, cnt, self._tag(0)], None

    def _after_gather(self, own, ev) -> None:
        eng, pend = own
        if eng is not None and pend is not None and ev is not None:
            eng.ex.hold(pend.ticket.k, ev)  # the stage is read by the gather

    def _serve_step(self, hdr, items, view) -> None:
        wk = self._workers(int(hdr[H_MASK]))
        own, src, _, ran = self._local_step(hdr, items, view, wk)
        _, failed, ev = self._gather(src, wk, None, strict=True, after=ran)
        self._after_gather(own, ev)
        eng, pend = own
        if ev is not None:
            ev.synchronize()
        if pend is not None:
            pend.ticket.wait()  # the annotated frames are in the slot before the ack

    def _assemble(self, dst, wk, per, items, view, own, s, messages, H, W, draw):
        from ..pipelines.stream import rebuild

        eng, pend = own
        n = len(messages)
        if pend is not None:
            pend.ticket.wait()
        if draw:  # the published Images view the slot's output area: this step's own array is the lease
            slot_out = np.frombuffer(self.ring.data.mm, np.uint8, self.ring.data.slot_bytes,
                                     s * self.ring.data.slot_bytes)
            self._lease(s, slot_out)
        out = []
        for r_i, (r, d) in enumerate(zip(wk, dst)):
            lo, hi = min(n, r_i * per), min(n, (r_i + 1) * per)
            if hi <= lo:
                continue
            if self.gpu:
                host = [t.cpu() for t in d[:-1]] if r != 0 else pend.ticket.host
                res = rebuild(eng.ex.template, host)
                cnt, box, score, cls = (res.count.numpy(), res.box.numpy(), res.score.numpy(), res.cls.numpy())
                rows = []
                for j in range(hi - lo):
                    c = int(min(cnt[j], box.shape[1]))
                    dd = np.empty((c, 6), np.float32)
                    dd[:, :4], dd[:, 4], dd[:, 5] = box[j, :c, :4], score[j, :c], cls[j, :c]
                    rows.append(dd)
            else:
                pad, cnt = d[0].numpy(), d[1].numpy()
                rows = [pad[j, :int(cnt[j])].copy() for j in range(hi - lo)]
            for j, dd in enumerate(rows):
                i = lo + j
                m = messages[i]
                if draw:
                    o0, sz = int(items[i, I_OUT]), int(items[i, I_OUTSZ])
                    data = memoryview(slot_out[o0:o0 + sz])
                else:
                    data = b""
                im = msgs.Image(header=m.header, height=H if draw else 0, width=W if draw else 0, encoding="rgb8",
                                step=3 * W if draw else 0, data=data)
                out.append((im, dd))
        return out


# ============================================================================ LiDAR
class DataParallelDetector3D(_RingDP):
    """PointCloud2 messages over the node's GPUs: ``live().process(clouds)`` /
    ``detect(clouds)`` -> per-cloud {pred_boxes, pred_scores, pred_labels}."""

    FIELDS = ("x", "y", "z", "intensity")

    def __init__(self, local, info: DistInfo, max_out: int = 500, box_dim: int = 7,
                 monitor: Optional[HealthMonitor] = None, nslots: int = 4, comm=None,
                 arena_mb: Optional[int] = None):
        super().__init__(local, info, monitor, nslots, comm, arena_mb=arena_mb)
        self.max_out, self.box_dim = max_out, box_dim
        self.B = int(getattr(local, "B", 0) or 0)

    def live(self):
        return self

    def detect(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        return self.process(clouds)

    def process(self, clouds: Sequence[msgs.PointCloud2]) -> List[dict]:
        if not clouds:
            return []
        if self.info.world == 1:
            return self.local.live().process(clouds) if self.gpu else self.local.detect(clouds)
        from ..ros.compat import cloud_layout

        with self._lock:
            groups: Dict[tuple, List[int]] = {}
            lays = {}
            for i, c in enumerate(clouds):
                lay = cloud_layout(c, self.FIELDS)
                k = (lay.point_step, *lay.offsets, *lay.dtypes)
                lays[k] = lay
                groups.setdefault(k, []).append(i)
            out: List[Optional[dict]] = [None] * len(clouds)
            for key, idx in groups.items():
                while idx:
                    chunk = idx[:self._chunk(len(idx))]
                    cs = [clouds[i] for i in chunk]
                    npts = [int(x.width * x.height) for x in cs]
                    payloads = [memoryview(x.data)[:k * key[0]] for x, k in zip(cs, npts)]
                    maxp = max(npts)

                    def prebuild(lay=lays[key], maxp=maxp, c0=cs[0]):
                        self.local.live()._engine(lay, maxp, c0)
                    try:
                        res = self._run_step(KIND_CLOUDS, payloads, [(k, 0) for k in npts], [], (*key, maxp), False,
                                             self._assemble, prebuild)
                    except _Rechunk:
                        continue
                    for i, r in zip(chunk, res):
                        out[i] = r
                    idx = idx[len(chunk):]
            return out

    def _shard_items(self, hdr, items, view, lo, hi):
        return self._shard_clouds(hdr, items, view, lo, hi)

    def _shard_clouds(self, hdr, items, view, lo, hi):
        step = int(hdr[H_KEY])
        offs, dts = [int(v) for v in hdr[H_KEY + 1:H_KEY + 5]], [int(v) for v in hdr[H_KEY + 5:H_KEY + 9]]
        fields = [msgs.PointField(k, o, d, 1) for k, o, d in zip(self.FIELDS, offs, dts)]
        out = []
        for i in range(lo, hi):
            raw = self._raw(items, i, view)
            k = int(items[i, I_M0])
            out.append(msgs.PointCloud2(height=1, width=k, fields=fields, point_step=step, row_step=k * step,
                                        data=memoryview(raw), is_dense=False))
        return out

    def _local_step(self, hdr, items, view, wk):
        lo, hi = self._shard(hdr, wk)
        seq, per = int(hdr[H_SEQ]), int(hdr[H_PER])
        clouds = self._shard_clouds(hdr, items, view, lo, hi)
        if self.gpu:
            from ..ops.lidar import PointLayout
            live = self.local.live()
            step = int(hdr[H_KEY])
            layout = PointLayout(step, tuple(int(v) for v in hdr[H_KEY + 1:H_KEY + 5]),
                                 tuple(int(v) for v in hdr[H_KEY + 5:H_KEY + 9]))
            # the node batch's max point count: the same engine on every rank
            eng = live._engine(layout, int(hdr[H_KEY + 9]), self._calibration_sample(hdr, items, view))
            pend, ran = None, None
            if clouds:
                pend = eng.submit(clouds)
                ran, src = pend.ticket.ran, list(pend.ticket.stage)
            else:
                src = eng.zero_stage()
            return (eng, pend), src + [self._tag(seq)], eng.zero_stage() + [self._tag(0)], ran
        sample = self._calibration_sample(hdr, items, view)
        if sample is not None:
            self.local.detect([sample])  # calibrates on the node batch's first cloud
        D, M = self.box_dim, self.max_out
        box = torch.zeros((per, M, D), dtype=torch.float32)
        score = torch.zeros((per, M), dtype=torch.float32)
        lab = torch.zeros((per, M), dtype=torch.int64)
        cnt = torch.zeros((per,), dtype=torch.int32)
        for j, p in enumerate(self.local.detect(clouds) if clouds else []):
            k = min(len(p["pred_scores"]), M)
            box[j, :k] = torch.from_numpy(np.asarray(p["pred_boxes"][:k, :D], np.float32))
            score[j, :k] = torch.from_numpy(np.asarray(p["pred_scores"][:k], np.float32))
            lab[j, :k] = torch.from_numpy(np.asarray(p["pred_labels"][:k], np.int64))
            cnt[j] = k
        src = [box, score, lab, cnt, self._tag(seq)]
        return (None, None), src, [box, score, lab, cnt, self._tag(0)], None

    _after_gather = DataParallelDetector2D._after_gather

    def _model_like_rank0(self, hdr) -> None:
        from ..ops.lidar import PointLayout
        layout = PointLayout(int(hdr[H_KEY]), tuple(int(v) for v in hdr[H_KEY + 1:H_KEY + 5]),
                             tuple(int(v) for v in hdr[H_KEY + 5:H_KEY + 9]))
        maxp = self.local.max_points
        while maxp < int(hdr[H_KEY + 9]):
            maxp *= 2
        p = self.local._calibrated_pipeline(layout, maxp, None)
        del p

    def _serve_step(self, hdr, items, view) -> None:
        wk = self._workers(int(hdr[H_MASK]))
        own, src, _, ran = self._local_step(hdr, items, view, wk)
        _, failed, ev = self._gather(src, wk, None, strict=True, after=ran)
        self._after_gather(own, ev)
        if ev is not None:
            ev.synchronize()

    def _assemble(self, dst, wk, per, items, view, own, s):
        from ..pipelines.stream import rebuild

        eng, pend = own
        n = len(items)
        if pend is not None:
            pend.ticket.wait()
        out = []
        for r_i, (r, d) in enumerate(zip(wk, dst)):
            lo, hi = min(n, r_i * per), min(n, (r_i + 1) * per)
            if hi <= lo:
                continue
            if self.gpu:
                host = [t.cpu() for t in d[:-1]] if r != 0 else pend.ticket.host
                out += self.local._frames_out(rebuild(eng.ex.template, host))[:hi - lo]
            else:
                box, score, lab, cnt = (t.numpy() for t in d[:4])
                for j in range(hi - lo):
                    k = int(cnt[j])
                    out.append({"pred_boxes": box[j, :k].copy(), "pred_scores": score[j, :k].copy(),
                                "pred_labels": lab[j, :k].copy()})
        return out
