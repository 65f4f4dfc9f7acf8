"""Double-buffered graph execution of a pipeline step for streaming callers.

The live drivers (``inference/live.py``) and the bench run the same device
step: static input buffers -> captured hipGraph -> static result buffers.  A
streaming caller also needs the *next* batch's host staging and H2D copy, and
the *previous* batch's D2H copy, to overlap the current replay.  This
executor keeps ``sets`` (2) copies of the step's input buffers and captures
one graph per set; batch t uses set t % 2:

    h2d stream:      H2D(inputs[k])  ───────────────► (waits for set k's last D2H)
    compute stream:             pre(k) ─ replay k ─ stage results[k] ─►
    d2h stream:                                                   D2H(results[k], extras) ─► set_free[k]

Each stage waits only on the events it needs, so with two host threads
submitting, batch t+1's H2D and batch t-1's D2H run beside batch t's
replay.  ``submit`` only enqueues (it takes a short lock); the returned
:class:`Ticket` is waited on with the GIL released.

Reference: the reference runs every stage of a frame serially inside one ROS
callback (``communicator/ros_inference.py:117-175``); this is the MI355X
replacement for that loop's device half.
"""
from __future__ import annotations

import dataclasses
import threading
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native
from .graph import GraphRunner, capture_gate


def flatten_tensors(obj) -> List[torch.Tensor]:
    """Tensors of a (nested dataclass) pipeline result, in field order."""
    if isinstance(obj, torch.Tensor):
        return [obj]
    if dataclasses.is_dataclass(obj):
        out = []
        for f in dataclasses.fields(obj):
            if f.init:
                out += flatten_tensors(getattr(obj, f.name))
        return out
    if isinstance(obj, (list, tuple)):
        out = []
        for v in obj:
            out += flatten_tensors(v)
        return out
    return []


def rebuild(obj, tensors: Sequence[torch.Tensor]):
    """The same result structure with its tensors replaced, in flatten order."""
    it = iter(tensors)

    def go(o):
        if isinstance(o, torch.Tensor):
            return next(it)
        if dataclasses.is_dataclass(o):
            return dataclasses.replace(o, **{f.name: go(getattr(o, f.name)) for f in dataclasses.fields(o)
                                             if f.init})
        if isinstance(o, (list, tuple)):
            return type(o)(go(v) for v in o)
        return o
    return go(obj)


def copy_segments(dst: Sequence[torch.Tensor], src: Sequence[torch.Tensor], stream=None) -> None:
    """Every (dst, src) pair with ONE batched copy kernel (csrc/kernels/copy.hip);
    a graph node per tensor costs ~11 us each at the end of a step."""
    pairs = [(d, s) for d, s in zip(dst, src) if s.numel()]
    if not pairs:
        return
    if not all(d.is_contiguous() and s.is_contiguous() and d.is_cuda for d, s in pairs):
        for d, s in pairs:
            d.copy_(s, non_blocking=True)
        return
    dp, sp, nb = (np.asarray(v, np.int64) for v in (
        [d.data_ptr() for d, _ in pairs], [s.data_ptr() for _, s in pairs],
        [s.numel() * s.element_size() for _, s in pairs]))
    _native.call("tca_copy_segments", len(pairs), dp.ctypes.data, sp.ctypes.data, nb.ctypes.data,
                 _native.stream_ptr(stream))


class Ticket:
    """One submitted batch: ``wait()`` blocks (GIL released) until its results
    and extras are in the pinned host tensors.  ``stage`` / ``ran``: the
    device copies of the results and the event after which they are complete
    (for device consumers such as the data-parallel gather, which then
    :meth:`StreamExecutor.hold` the set until they are done reading)."""

    def __init__(self, k: int, done: torch.cuda.Event, host: List[torch.Tensor], extras: List[torch.Tensor],
                 uploaded: torch.cuda.Event, template, ran: torch.cuda.Event, stage: List[torch.Tensor]):
        self.k, self.done, self.host, self.extras, self.uploaded = k, done, host, extras, uploaded
        self.template, self.ran, self.stage = template, ran, stage

    def wait(self):
        self.done.synchronize()
        return self

    def result(self):
        """The step's result structure over the host copies (after wait())."""
        return rebuild(self.template, self.host)


class StreamExecutor:
    """``sets`` captured replays of ``step`` over ``sets`` copies of its inputs.

    step:       capture-safe callable reading ``getattr(owner, attr)`` for each
                of ``inputs`` and returning a result structure (dataclasses of
                tensors, see :func:`flatten_tensors`);
    inputs:     (owner, attr) pairs; set 0 is the owner's own tensors, the
                others are allocated alike; while set k is captured the
                attributes point at set k's tensors.
    """

    def __init__(self, step: Callable[[], object], inputs: Sequence[Tuple[object, str]], device,
                 sets: int = 2, graph: bool = True):
        self.step, self.owners = step, list(inputs)
        self.device = torch.device(device)
        base = [getattr(o, a) for o, a in self.owners]
        self.inputs: List[List[torch.Tensor]] = [base] + [[torch.empty_like(t) for t in base]
                                                          for _ in range(sets - 1)]
        self.stage: List[Optional[List[torch.Tensor]]] = [None] * sets
        self.template = None
        self.runners = [GraphRunner(self._bound(k), enabled=graph, capture_error_mode="thread_local")
                        for k in range(sets)]
        self.compute = torch.cuda.Stream(self.device)
        self.h2d = torch.cuda.Stream(self.device)
        self.d2h = torch.cuda.Stream(self.device)
        self.set_free: List[List[torch.cuda.Event]] = [[] for _ in range(sets)]
        self.next = 0
        self.lock = threading.Lock()
        self.batches = 0
        # capture every set now, over whatever the inputs hold: the eager warm-up
        # runs of a capture must not see (and, for an in-place annotator, modify)
        # a real batch
        self.gate = capture_gate(self.device)
        with torch.cuda.stream(self.compute):
            for k, r in enumerate(self.runners):
                if r.enabled:
                    r.capture()
                else:
                    r()  # eager: one run allocates the stage buffers
            self.compute.synchronize()

    @property
    def sets(self) -> int:
        return len(self.inputs)

    def _bound(self, k: int):
        def fn():
            for (o, a), t in zip(self.owners, self.inputs[k]):
                setattr(o, a, t)
            try:
                res = self.step()
            finally:
                for (o, a), t in zip(self.owners, self.inputs[0]):
                    setattr(o, a, t)
            outs = flatten_tensors(res)
            if self.stage[k] is None:  # allocated in the eager warm-up, before capture
                self.stage[k] = [torch.empty_like(t) for t in outs]
                self.template = res
            copy_segments(self.stage[k], outs)
            return res
        return fn

    def hold(self, k: int, event: torch.cuda.Event) -> None:
        """Set k is not rewritten (inputs or stage) before ``event`` — e.g. a
        device-side gather still reading its stage."""
        with self.lock:
            self.set_free[k].append(event)

    def submit(self, copies: Callable[[int], Sequence[Tuple[torch.Tensor, torch.Tensor]]],
               pre: Optional[Callable[[int], None]] = None,
               extras: Optional[Callable[[int], Sequence[torch.Tensor]]] = None,
               extras_dst: Optional[Sequence[Optional[torch.Tensor]]] = None) -> Ticket:
        """Enqueue one batch.  ``copies(k)``: (device, pinned host) pairs to
        upload into set k (a host tensor may be shorter than its device
        buffer: its leading elements are written); ``pre(k)``: extra work on
        the compute stream before the replay (e.g. JPEG reconstruction into
        set k); ``extras(k)``: device tensors copied back after the replay
        (e.g. the annotated frames of set k) into fresh pinned tensors, or
        into ``extras_dst[i]`` (page-locked host tensors, e.g. slots of the
        data-parallel host ring) where given."""
        # executor lock first, then the gate's shared side: a thread waiting for the lock holds
        # no shared hold, so a first-use capture below (shared -> exclusive while holding the
        # lock) only waits for other executors' submissions, which never need this lock
        with self.lock, self.gate.shared():  # (no submission inside another thread's capture window)
            k = self.next
            self.next = (k + 1) % self.sets
            for ev in self.set_free[k]:  # set k's inputs / stage are still being read back
                self.h2d.wait_event(ev)
            self.set_free[k] = []
            with torch.cuda.stream(self.h2d):
                for d, h in copies(k):
                    d.view(-1)[:h.numel()].copy_(h.view(-1), non_blocking=True)
                up = torch.cuda.Event()
                up.record(self.h2d)
            self.compute.wait_event(up)
            with torch.cuda.stream(self.compute):
                if pre is not None:
                    pre(k)
                self.runners[k]()  # first use: warm-up + capture
                ran = torch.cuda.Event()
                ran.record(self.compute)
            self.d2h.wait_event(ran)
            with torch.cuda.stream(self.d2h):
                host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in self.stage[k]]
                for h, d in zip(host, self.stage[k]):
                    h.copy_(d, non_blocking=True)
                ex = []
                for i, d in enumerate(extras(k) if extras is not None else ()):
                    h = extras_dst[i] if extras_dst is not None and i < len(extras_dst) else None
                    if h is None:
                        h = torch.empty(d.shape, dtype=d.dtype, pin_memory=True)
                    h.copy_(d, non_blocking=True)
                    ex.append(h)
                done = torch.cuda.Event()
                done.record(self.d2h)
            self.set_free[k].append(done)
            self.batches += 1
            return Ticket(k, done, host, ex, up, self.template, ran, self.stage[k])

    def synchronize(self) -> None:
        for s in (self.h2d, self.compute, self.d2h):
            s.synchronize()


class PinnedSlots:
    """A pool of host staging slots (pinned buffers built by ``make()``) for
    concurrent producers: ``acquire()`` blocks until a slot is free;
    ``release(slot, event)`` frees it once ``event`` (the last device read of
    the slot) has completed."""

    def __init__(self, n: int, make: Callable[[], object]):
        self.free = [(make(), None) for _ in range(n)]
        self.cv = threading.Condition()

    def acquire(self):
        with self.cv:
            while not self.free:
                self.cv.wait()
            slot, ev = self.free.pop()
        if ev is not None:
            ev.synchronize()
        return slot

    def release(self, slot, event: Optional[torch.cuda.Event] = None) -> None:
        with self.cv:
            self.free.append((slot, event))
            self.cv.notify()
