"""hipGraph capture of a whole pipeline step.

The per-frame work is dozens of short kernels (preprocess, ~60 convs,
decode, sort, NMS...).  Eager launch costs ≈3-4 µs of host time per kernel
(MI355X_MICROARCH.md price list, row graph-replay-floor), so a step is
captured once and replayed: static input buffers are written (H2D copy or
RCCL receive) before ``replay()``, outputs are read from static buffers
after it.  Every op in this package is capture-safe by construction (no
allocation, no host sync, device-side counts).

Capture hygiene is checked, not assumed.  A step that forks work onto a side
stream and does not join it back before the capture ends leaves HIP with an
unjoined capture; on this ROCm ``hipStreamEndCapture`` then crashed the
process inside ``torch.cuda.graphs.capture_end`` (round 3, a three-stream
variant of the pipelined LiDAR step).  :meth:`GraphRunner.capture` therefore
records every stream the step enters (``torch.cuda.stream`` contexts) and,
before the capture ends, asks HIP for each stream's capture tips
(``hipStreamGetCaptureInfo_v2``): a side stream whose last captured work is
not an ancestor of the capturing stream's tips (``hipGraphNodeGetDependencies``)
was never joined.  Such streams are joined back (so the capture ends
cleanly), the graph is discarded and :class:`GraphCaptureError` names them.  A native launch (``_native.call``)
onto a stream that is *not* part of the capture while one is active on the
thread — work that would silently run once, eagerly, instead of on every
replay — raises the same error.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading
from typing import Callable, Dict, Optional, Set

import torch


class GraphCaptureError(RuntimeError):
    pass


_TL = threading.local()

class CaptureGate:
    """Reader/writer gate of one device between graph captures and stream work.

    ``shared()``: stream work that must not interleave with a capture window --
    executor submissions (pinned result allocation, H2D / D2H enqueue, replays) and
    capture warm-ups.  Any number of threads hold it together: two engines' submissions
    no longer serialise against each other.
    ``exclusive()``: the capture window itself (``torch.cuda.graph`` begin..end); it waits
    for the current shared holders and blocks new ones (writer preference, so a steady
    stream of submissions cannot starve an engine build).

    Why a capture window is exclusive -- the mechanism, from the code on these paths: a
    thread_local-mode capture restricts only the capturing thread, and the calls other
    threads make here are legal on their own streams; the two that are device- or
    process-wide are (a) ``hipHostMalloc`` / ``hipHostFree`` behind ``torch.empty(...,
    pin_memory=True)`` in :meth:`~triton_client_amd.pipelines.stream.StreamExecutor.submit`
    (the caching host allocator calls them with the GIL held), and (b) the old warm-up's
    ``torch.cuda.synchronize()`` (hipDeviceSynchronize over every stream of the device).
    A capture also needs the GIL to run the Python step it records.  A thread blocked in a
    device-wide call with the GIL held while another thread sits inside a capture window
    therefore stalls both -- the intermittent stall of two live drivers building engines
    at once (round 4).  The warm-up now waits on its own stream only, runs under the
    shared side, and only the capture window is exclusive.

    Reentrant per thread; a thread holding the shared side that asks for the exclusive
    side gives its shared holds up while it waits (a first-use capture inside a
    submission), and gets them back after."""

    def __init__(self):
        self._cv = threading.Condition(threading.Lock())
        self._readers = 0
        self._writer: Optional[int] = None
        self._writer_depth = 0
        self._writers_waiting = 0
        self._tl = threading.local()
        self.captures = 0

    def _shared_depth(self) -> int:
        return getattr(self._tl, "shared", 0)

    @contextlib.contextmanager
    def shared(self):
        me = threading.get_ident()
        with self._cv:
            if self._writer != me and self._shared_depth() == 0:
                while self._writer is not None or self._writers_waiting:
                    self._cv.wait()
            self._readers += 1
            self._tl.shared = self._shared_depth() + 1
        try:
            yield
        finally:
            with self._cv:
                self._readers -= 1
                self._tl.shared -= 1
                self._cv.notify_all()

    @contextlib.contextmanager
    def exclusive(self):
        me = threading.get_ident()
        with self._cv:
            if self._writer == me:
                self._writer_depth += 1
            else:
                held = self._shared_depth()
                self._readers -= held  # give up this thread's shared holds while waiting
                self._writers_waiting += 1
                self._cv.notify_all()
                while self._writer is not None or self._readers > 0:
                    self._cv.wait()
                self._writers_waiting -= 1
                self._writer, self._writer_depth = me, 1
                self._readers += held
                self.captures += 1
        try:
            yield
        finally:
            with self._cv:
                self._writer_depth -= 1
                if self._writer_depth == 0:
                    self._writer = None
                self._cv.notify_all()


_GATES: Dict[int, CaptureGate] = {}
_GATES_LOCK = threading.Lock()


def capture_gate(device=None) -> CaptureGate:
    """The :class:`CaptureGate` of ``device`` (default: the current device)."""
    idx = torch.device(device).index if device is not None else None
    if idx is None:
        idx = torch.cuda.current_device() if torch.cuda.is_available() else -1
    with _GATES_LOCK:
        g = _GATES.get(idx)
        if g is None:
            g = _GATES[idx] = CaptureGate()
        return g


_SPY_LOCK = threading.Lock()
_SPY = {"installed": False}


def _install_stream_spy() -> None:
    """Wrap ``torch.cuda.set_stream`` once: while this thread captures, the
    streams it makes current are recorded (``torch.cuda.stream(s)`` goes
    through ``set_stream``)."""
    with _SPY_LOCK:
        if _SPY["installed"]:
            return
        real = torch.cuda.set_stream

        def set_stream(stream):
            rec = getattr(_TL, "streams", None)
            if rec is not None and stream is not None:
                rec[int(stream.cuda_stream)] = stream
            return real(stream)
        torch.cuda.set_stream = set_stream
        _SPY["installed"] = True


def capturing_thread() -> bool:
    """True while this thread is inside :meth:`GraphRunner.capture`."""
    return getattr(_TL, "streams", None) is not None


_HIPF: Dict[str, object] = {}


def _hip_fn(name: str, argtypes):
    """A HIP runtime entry point with its argtypes (None if unavailable)."""
    if name not in _HIPF:
        from .. import _native

        hip = _native._load_hip()
        fn = getattr(hip, name, None) if hip is not None else None
        if fn is not None:
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _HIPF[name] = fn
    return _HIPF[name]


def stream_is_capturing(handle: int) -> bool:
    """hipStreamIsCapturing on a raw stream handle (0: the null stream)."""
    fn = _hip_fn("hipStreamIsCapturing", [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)])
    if fn is None:
        return False
    st = ctypes.c_int(0)
    rc = fn(ctypes.c_void_p(int(handle)), ctypes.byref(st))
    return rc == 0 and st.value == 1  # hipStreamCaptureStatusActive


def _capture_tips(handle: int) -> Optional[Set[int]]:
    """Graph nodes the next captured op on this stream would depend on (its capture
    "tips"); None if the stream is not capturing or the query is unavailable."""
    fn = _hip_fn("hipStreamGetCaptureInfo_v2",
                 [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulonglong),
                  ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.POINTER(ctypes.c_void_p)),
                  ctypes.POINTER(ctypes.c_size_t)])
    if fn is None:
        return None
    st, cid, graph = ctypes.c_int(0), ctypes.c_ulonglong(0), ctypes.c_void_p()
    deps, n = ctypes.POINTER(ctypes.c_void_p)(), ctypes.c_size_t(0)
    if fn(ctypes.c_void_p(int(handle)), ctypes.byref(st), ctypes.byref(cid), ctypes.byref(graph), ctypes.byref(deps),
          ctypes.byref(n)) != 0 or st.value != 1:
        return None
    return {int(deps[i] or 0) for i in range(n.value)}


def _ancestors(nodes: Set[int]) -> Set[int]:
    """``nodes`` and every node they (transitively) depend on."""
    fn = _hip_fn("hipGraphNodeGetDependencies",
                 [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)])
    seen, todo = set(nodes), list(nodes)
    while todo and fn is not None:
        node = ctypes.c_void_p(todo.pop())
        n = ctypes.c_size_t(0)
        if fn(node, None, ctypes.byref(n)) != 0 or n.value == 0:
            continue
        arr = (ctypes.c_void_p * n.value)()
        if fn(node, arr, ctypes.byref(n)) != 0:
            continue
        for d in arr[:n.value]:
            d = int(d or 0)
            if d not in seen:
                seen.add(d)
                todo.append(d)
    return seen


def unjoined_streams(origin, streams: Dict[int, object]) -> Dict[int, object]:
    """Streams forked into the capture on ``origin`` whose last captured work is
    not (yet) a dependency of the origin stream's tips."""
    otips = _capture_tips(int(origin.cuda_stream))
    if otips is None:
        return {}
    anc = None
    out = {}
    for h, st in streams.items():
        if h == int(origin.cuda_stream):
            continue
        tips = _capture_tips(h)
        if not tips:
            continue  # not part of this capture, or nothing captured on it
        if anc is None:
            anc = _ancestors(otips)
        if not tips <= anc:
            out[h] = st
    return out


class GraphRunner:
    def __init__(self, fn: Callable[[], object], warmup: int = 3, enabled: bool = True,
                 pool=None, capture_error_mode: str = "global"):
        self.fn = fn
        self.enabled = enabled and torch.cuda.is_available()
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.warmup = warmup
        self.pool = pool
        # "thread_local": other host threads may keep issuing HIP calls (event
        # waits, pinned allocations) while this thread captures (live drivers)
        self.capture_error_mode = capture_error_mode

    def capture(self) -> None:
        if not self.enabled:
            return
        gate = capture_gate()
        with gate.shared():  # warm-up: ordinary stream work beside other threads' submissions
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    self.out = self.fn()
            torch.cuda.current_stream().wait_stream(s)
            s.synchronize()  # this stream only: no device-wide sync (see CaptureGate)
        with gate.exclusive():
            self._capture()

    def _capture(self) -> None:
        _install_stream_spy()
        g = torch.cuda.CUDAGraph()
        unjoined: Dict[int, object] = {}
        _TL.streams = {}
        try:
            with torch.cuda.graph(g, pool=self.pool, capture_error_mode=self.capture_error_mode):
                origin = torch.cuda.current_stream()
                try:
                    self.out = self.fn()
                finally:
                    # before capture_end: every forked stream must be joined back
                    unjoined.update(unjoined_streams(origin, _TL.streams))
                    for st in unjoined.values():
                        origin.wait_stream(st)  # join it, so the capture ends cleanly
        finally:
            _TL.streams = None
        if unjoined:
            self.graph = None
            raise GraphCaptureError(f"the captured step left {len(unjoined)} forked stream(s) unjoined "
                                    f"(handles {[hex(h) for h in unjoined]}): join every side stream back into "
                                    "the capturing stream (current_stream().wait_stream(side)) before it returns")
        self.graph = g

    def __call__(self):
        if self.graph is None:
            if self.enabled:
                self.capture()
            else:
                self.out = self.fn()
                return self.out
        self.graph.replay()
        return self.out

    def release(self) -> None:
        """Destroy the captured graph now (the next call re-captures).  A graph holding
        RCCL work must be released BEFORE its communicator is aborted / destroyed: the
        graph's teardown hands RCCL's persistent plan back to the communicator, so a
        graph outliving it (a stray reference, a loop variable) blocks in that teardown
        (tools/rccl_two_graphs.py: the two-graph gather replays correctly either way)."""
        if self.graph is not None:
            torch.cuda.synchronize()
            self.graph.reset()
            self.graph = None
