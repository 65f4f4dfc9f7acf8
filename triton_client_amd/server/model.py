"""Servable model contract for the in-process KServe-v2 server.

A :class:`ServedModel` owns a Triton-compatible ``ModelConfig`` (the tensor
contract the reference's clients negotiate via ``ModelMetadata`` /
``ModelConfig``, e.g. ``examples/pointpillar_kitti/config.pbtxt``) and an
``execute`` that maps named numpy inputs to named numpy outputs — the role of
``TritonPythonModel.execute`` in the reference's Python-backend models
(``examples/pointpillar_kitti/1/model.py:119-186``).
"""
from __future__ import annotations

import collections
import threading
import time
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..proto import config_dtype_to_kserve, model_config_pb2 as mc, service_pb2 as pb

DT = {"FP32": mc.TYPE_FP32, "FP16": mc.TYPE_FP16, "INT32": mc.TYPE_INT32, "INT64": mc.TYPE_INT64,
      "UINT8": mc.TYPE_UINT8, "BOOL": mc.TYPE_BOOL, "FP64": mc.TYPE_FP64, "INT16": mc.TYPE_INT16}


def tensor_spec(name: str, dtype: str, dims: Sequence[int], fmt: Optional[str] = None,
                reshape: Optional[Sequence[int]] = None, output: bool = False):
    t = mc.ModelOutput() if output else mc.ModelInput()
    t.name = name
    t.data_type = DT[dtype]
    t.dims.extend(list(dims))
    if fmt and not output:
        t.format = {"NCHW": mc.ModelInput.FORMAT_NCHW, "NHWC": mc.ModelInput.FORMAT_NHWC}[fmt]
    if reshape:
        t.reshape.shape.extend(list(reshape))
    return t


@dataclass
class ModelStats:
    inference_count: int = 0
    execution_count: int = 0
    success_ns: int = 0
    fail_count: int = 0
    compute_ns: int = 0
    last_inference_ms: int = 0
    lock: threading.Lock = field(default_factory=threading.Lock)


class InferError(Exception):
    """Raised by execute() for a client error (bad shape/dtype) → INVALID_ARGUMENT."""


class _RWLock:
    """Many executions (shared) or one model load (exclusive).  A load builds
    and captures hipGraphs; a capture racing kernels that another thread
    launches (another model serving) can record or corrupt them, so no
    model executes while any model loads."""

    def __init__(self):
        self._cv = threading.Condition()
        self._readers = 0
        self._writer = False
        self._writers_waiting = 0  # new readers yield to a pending writer (no load starvation)

    def acquire_shared(self):
        with self._cv:
            while self._writer or self._writers_waiting:
                self._cv.wait()
            self._readers += 1

    def release_shared(self):
        with self._cv:
            self._readers -= 1
            if self._readers == 0:
                self._cv.notify_all()

    def acquire_exclusive(self):
        with self._cv:
            self._writers_waiting += 1
            try:
                while self._writer or self._readers:
                    self._cv.wait()
            finally:
                self._writers_waiting -= 1
            self._writer = True

    def release_exclusive(self):
        with self._cv:
            self._writer = False
            self._cv.notify_all()


GPU_PHASE = _RWLock()


class StageProfile:
    """Server-side stage clock for the served-path bench (``TCA_SERVER_PROFILE=<json path>``):
    per stage the summed seconds and count, over every request / execution thread;
    written by :meth:`dump` (the standalone server does at SIGTERM).  Disabled: one
    attribute test per stage."""

    def __init__(self, path: Optional[str]):
        self.path, self.on = path, bool(path)
        self.t: Dict[str, float] = collections.defaultdict(float)
        self.n: Dict[str, int] = collections.defaultdict(int)
        self.lock = threading.Lock()
        self.t0 = time.perf_counter()

    def add(self, stage: str, seconds: float, n: int = 1) -> None:
        with self.lock:
            self.t[stage] += seconds
            self.n[stage] += n

    def summary(self) -> dict:
        wall = time.perf_counter() - self.t0
        with self.lock:
            return {"wall_s": round(wall, 3),
                    "stages": {k: {"count": self.n[k], "total_s": round(v, 4),
                                   "ms_each": round(1e3 * v / max(1, self.n[k]), 4)} for k, v in sorted(self.t.items())}}

    def dump(self) -> None:
        if self.on:
            import json
            with open(self.path, "w") as f:
                json.dump(self.summary(), f)


def _profile_from_env() -> StageProfile:
    import os
    return StageProfile(os.environ.get("TCA_SERVER_PROFILE") or None)


PROFILE = _profile_from_env()


class _Pending:
    __slots__ = ("inputs", "requested", "encode", "out_dst", "done", "result", "exc")

    def __init__(self, inputs, requested, encode, out_dst=None):
        self.inputs, self.requested, self.encode, self.out_dst = inputs, requested, encode, out_dst
        self.done = threading.Event()
        self.result = None
        self.exc: Optional[BaseException] = None


class DynamicBatcher:
    """Server-side dynamic batching (Triton's ``dynamic_batching``, transparent
    to batch-1 clients: the reference's models are ``max_batch_size: 0``,
    ``examples/YOLOv5/config.pbtxt:3``).  Request threads enqueue and wait;
    one batcher thread takes the oldest request, waits up to ``delay_s`` for
    more (up to ``max_batch``), runs them as ONE ``execute_batch`` under the
    model lock and encodes every request's response from its slice before the
    next batch reuses the staging.  A batch that fails is re-run request by
    request so one bad request cannot fail its neighbours."""

    def __init__(self, model: "ServedModel", max_batch: int, delay_s: float):
        self.model, self.max_batch, self.delay_s = model, max_batch, delay_s
        self.q: "collections.deque[_Pending]" = collections.deque()
        self.cv = threading.Condition()
        self.stopped = False
        self.batches = 0
        self.forming = threading.Lock()
        self.inflight = 0  # pipelined: batches issued and not yet finished
        self.sets = model.plan_set_count() if model.pipelined() else 1
        if self.sets > 1:
            # pipelined: ONE batcher thread issues batch k + 1 on the next plan set (its own stream)
            # as soon as batch k is queued on the GPU; a finisher thread waits for each batch in
            # order and answers its requests (batches keep their full size: nothing splits them)
            self.threads = [threading.Thread(target=self._run_pipelined, name=f"batcher-{model.name}", daemon=True)]
        else:
            # one batcher thread per model instance (Triton instance_group count): instance k runs
            # its batches on its own plans, stream and lock, so one instance stages / encodes while
            # another's graph runs on the GPU
            self.threads = [threading.Thread(target=self._run, args=(k,), name=f"batcher-{model.name}-{k}",
                                             daemon=True) for k in range(max(1, model.instances))]
        for t in self.threads:
            t.start()

    def submit(self, inputs, requested, encode, out_dst=None):
        item = _Pending(inputs, requested, encode, out_dst)
        with self.cv:
            if self.stopped:
                raise InferError(f"model '{self.model.name}' is unloading")
            self.q.append(item)
            self.cv.notify()
        item.done.wait()
        if item.exc is not None:
            raise item.exc
        return item.result

    def stop(self, timeout_s: float = 60.0) -> None:
        """Stop taking requests and wait for the batch in flight (if any) to
        finish: the model frees its plans only after no batch runs on them.
        Raises :class:`InferError` if a batch is still running after
        ``timeout_s`` (e.g. stuck on a hung device wait): the caller must then
        leave the model loaded-but-not-ready rather than free live plans, and
        a control RPC never blocks forever."""
        with self.cv:
            self.stopped = True
            self.cv.notify_all()
        deadline = time.perf_counter() + timeout_s
        for t in self.threads:
            t.join(max(0.0, deadline - time.perf_counter()))
        stuck = [t.name for t in self.threads if t.is_alive()]
        if stuck:
            raise InferError(f"model '{self.model.name}': batcher threads {stuck} still running after "
                             f"{timeout_s:g} s; not unloaded")

    def _take(self):
        with self.cv:
            while not self.q and not self.stopped:
                self.cv.wait()
            if not self.q:
                return None
            deadline = time.perf_counter() + self.delay_s
            while len(self.q) < self.max_batch and not self.stopped:
                if self.inflight:
                    # pipelined, a batch on the GPU: issue the next one early only when it is full;
                    # otherwise keep gathering until the GPU frees up (the finisher notifies), so
                    # overlapping never splits the arriving requests into small batches
                    self.cv.wait()
                    continue
                left = deadline - time.perf_counter()
                if left <= 0:
                    break
                self.cv.wait(left)
            return [self.q.popleft() for _ in range(min(self.max_batch, len(self.q)))]

    def _run(self, k: int = 0) -> None:
        while True:
            # one instance forms a batch at a time: the next one gathers the requests that arrive
            # while this batch runs (two instances forming at once would split every batch in two)
            with self.forming:
                items = self._take()
            if items is None:
                return
            with self.cv:
                self.batches += 1
            m = self.model
            GPU_PHASE.acquire_shared()
            try:
                with m.stream_context(k):
                    self._execute(m, items, k)
            finally:
                GPU_PHASE.release_shared()

    def _run_pipelined(self) -> None:
        import queue
        m = self.model
        jobs: "queue.Queue" = queue.Queue()
        fin = threading.Thread(target=self._finisher, args=(jobs,), name=f"finisher-{m.name}", daemon=True)
        fin.start()
        k = 0
        try:
            while True:
                items = self._take()
                if items is None:
                    return
                with self.cv:
                    self.batches += 1
                s = k % self.sets
                k += 1
                GPU_PHASE.acquire_shared()
                lock = m.instance_lock(s)
                lock.acquire()  # plan set s is free once the finisher is done with its previous batch
                t0 = time.perf_counter()
                try:
                    dsts = [it.out_dst for it in items]
                    with m.stream_context(s):
                        finish = m.execute_batch_async([it.inputs for it in items], items[0].requested,
                                                       dsts=dsts if m.accepts_out_dst and any(dsts) else None, inst=s)
                except Exception:  # noqa: BLE001 - isolate the failing request(s) below
                    lock.release()
                    GPU_PHASE.release_shared()
                    self._isolate(m, items)
                    continue
                with self.cv:
                    self.inflight += 1
                jobs.put((items, finish, lock, t0))
        finally:
            jobs.put(None)
            fin.join()

    def _finisher(self, jobs) -> None:
        m = self.model
        while True:
            job = jobs.get()
            if job is None:
                return
            items, finish, lock, t0 = job
            try:
                outs = finish()
                t1 = time.perf_counter()
                for it, o in zip(items, outs):
                    if isinstance(o, BaseException):
                        it.exc = o
                        it.done.set()
                    else:
                        self._finish(it, o)
                if PROFILE.on:
                    PROFILE.add(f"{m.name}.execute_batch", t1 - t0)
                    PROFILE.add(f"{m.name}.batch_items", float(len(items)))
                    PROFILE.add(f"{m.name}.encode_in_batcher", time.perf_counter() - t1, len(items))
                failed = False
            except Exception:  # noqa: BLE001
                failed = True
            finally:
                lock.release()
                GPU_PHASE.release_shared()
                with self.cv:
                    self.inflight -= 1
                    self.cv.notify_all()
            if failed:
                self._isolate(m, items)

    def _isolate(self, m: "ServedModel", items) -> None:
        """Run a failed batch's unanswered requests one by one (one bad request cannot
        fail its neighbours)."""
        GPU_PHASE.acquire_shared()
        try:
            with m.instance_lock(0):
                for it in items:
                    if it.done.is_set():
                        continue
                    try:
                        self._finish(it, m.execute(it.inputs, it.requested))
                    except Exception as e:  # noqa: BLE001 - handed to the waiting request thread
                        it.exc = e
                        it.done.set()
        finally:
            GPU_PHASE.release_shared()

    def _execute(self, m: "ServedModel", items, k: int = 0) -> None:
        with m.instance_lock(k):
            try:
                t0 = time.perf_counter()
                dsts = [it.out_dst for it in items]
                kw = {"inst": k} if m.instances > 1 else {}
                if m.accepts_out_dst and any(d for d in dsts):
                    outs = m.execute_batch([it.inputs for it in items], items[0].requested, dsts=dsts, **kw)
                else:
                    outs = m.execute_batch([it.inputs for it in items], items[0].requested, **kw)
                t1 = time.perf_counter()
                for it, o in zip(items, outs):
                    if isinstance(o, BaseException):  # this request failed inside the batch (e.g. bad values)
                        it.exc = o
                        it.done.set()
                    else:
                        self._finish(it, o)
                if PROFILE.on:
                    PROFILE.add(f"{m.name}.execute_batch", t1 - t0)
                    PROFILE.add(f"{m.name}.batch_items", float(len(items)))
                    PROFILE.add(f"{m.name}.encode_in_batcher", time.perf_counter() - t1, len(items))
            except Exception:
                for it in items:  # isolate the failing request(s)
                    if it.done.is_set():
                        continue
                    try:
                        self._finish(it, m.execute(it.inputs, it.requested))
                    except Exception as e:  # noqa: BLE001 - handed to the waiting request thread
                        it.exc = e
                        it.done.set()

    @staticmethod
    def _finish(it: _Pending, out) -> None:
        try:
            it.result = it.encode(out) if it.encode is not None else out
        except Exception as e:  # noqa: BLE001
            it.exc = e
        it.done.set()


class ServedModel(ABC):
    platform = "amd_mi355x"
    backend = "triton_client_amd"
    max_batch_size = 0
    # server-side dynamic batching of concurrent batch-1 requests (DynamicBatcher);
    # a model sets dynamic_batch > 1 in load() once it has an execute_batch
    dynamic_batch = 1
    batch_delay_s = 0.0005
    # execute_batch(..., dsts=[per request {output: uint8 view of its shared-memory output
    # slice} or None]) writes outputs there directly (see models._direct_out)
    accepts_out_dst = False
    # inputs from a device shared-memory region arrive as torch tensors on the GPU when
    # the model reads them there (device_inputs), else as host copies
    device_inputs = False
    # Triton instance_group count: dynamic-batching executions in flight at once (a model with
    # instances > 1 takes execute_batch(..., inst=k) and keeps per-instance plans)
    instances = 1
    # batches in flight on one batcher (models with execute_batch_async(..., inst=k) -> finish():
    # plan set k issues on its own stream, finish() waits for that batch only)
    pipeline_depth = 1

    def __init__(self, name: str, version: str = "1"):
        self.name = name
        self.version = version
        self.ready = False
        self.stats = ModelStats()
        self._config: Optional[mc.ModelConfig] = None
        self._lock = threading.Lock()  # one execution at a time per instance (GPU graph buffers)
        self._batcher: Optional[DynamicBatcher] = None
        self._streams: Dict[int, object] = {}  # HIP streams of this model's own (per instance)
        self._inst_locks: Dict[int, threading.Lock] = {0: self._lock}

    def pipelined(self) -> bool:
        """Dynamic batches run pipelined (DynamicBatcher._run_pipelined)."""
        dev = getattr(self, "device", None)
        return (self.pipeline_depth > 1 and callable(getattr(self, "execute_batch_async", None))
                and getattr(dev, "type", None) == "cuda")

    def plan_set_count(self) -> int:
        """Plan sets a GPU model builds: one per batch in flight (pipelined) or per instance."""
        return max(1, self.instances, self.pipeline_depth if self.pipelined() else 1)

    def instance_lock(self, k: int = 0) -> threading.Lock:
        """Lock of instance k (instance 0: the model lock of direct executions)."""
        if k not in self._inst_locks:
            with self._lock:
                self._inst_locks.setdefault(k, threading.Lock())
        return self._inst_locks[k]

    def stream_context(self, k: int = 0):
        """Context running this model's executions (of instance k) on a stream of its own
        (GPU models; a no-op on the CPU): the batcher threads of two models, or two instances
        of one, would otherwise serialise on the default stream."""
        import contextlib
        dev = getattr(self, "device", None)
        if dev is None or getattr(dev, "type", None) != "cuda":
            return contextlib.nullcontext()
        import torch
        if k not in self._streams:
            self._streams[k] = torch.cuda.Stream(device=dev)
        return torch.cuda.stream(self._streams[k])

    # ---------------------------------------------------------------- contract
    @abstractmethod
    def inputs(self) -> List[mc.ModelInput]:
        ...

    @abstractmethod
    def outputs(self) -> List[mc.ModelOutput]:
        ...

    @abstractmethod
    def execute(self, inputs: Dict[str, np.ndarray], requested: Sequence[str]) -> Dict[str, np.ndarray]:
        ...

    def execute_batch(self, batch: Sequence[Dict[str, np.ndarray]], requested: Sequence[str]
                      ) -> List[Dict[str, np.ndarray]]:
        """Run several requests as one execution (dynamic batching).  The
        returned outputs may be views of staging that stays valid until the
        next execution; the batcher encodes every response before that."""
        raise NotImplementedError

    def load(self) -> None:
        """Allocate / build / warm up.  Sets ready."""
        self.ready = True

    def unload(self) -> None:
        if self._batcher is not None:
            try:
                self._batcher.stop()
            except InferError:
                self.ready = False  # no new requests; the plans stay allocated under the stuck batch
                raise
            self._batcher = None
        # no execution of this model (batched or direct) is mid-run past this point
        GPU_PHASE.acquire_exclusive()
        try:
            locks = [self.instance_lock(k) for k in range(self.plan_set_count())]
            for lk in locks:
                lk.acquire()
            try:
                self.ready = False
            finally:
                for lk in reversed(locks):
                    lk.release()
        finally:
            GPU_PHASE.release_exclusive()

    def instance_kind(self) -> int:
        return mc.ModelInstanceGroup.KIND_GPU

    # ---------------------------------------------------------------- derived
    def config(self) -> mc.ModelConfig:
        if self._config is None:
            c = mc.ModelConfig(name=self.name, platform=self.platform, backend=self.backend,
                               max_batch_size=self.max_batch_size)
            c.input.extend(self.inputs())
            c.output.extend(self.outputs())
            c.instance_group.add(kind=self.instance_kind(), count=max(1, self.instances))
            self._config = c
        return self._config

    def metadata(self) -> pb.ModelMetadataResponse:
        cfg = self.config()
        md = pb.ModelMetadataResponse(name=self.name, versions=[self.version], platform=self.platform)
        for t in cfg.input:
            shape = list(t.dims)
            md.inputs.add(name=t.name, datatype=config_dtype_to_kserve(t.data_type), shape=shape)
        for t in cfg.output:
            md.outputs.add(name=t.name, datatype=config_dtype_to_kserve(t.data_type), shape=list(t.dims))
        return md

    def validate(self, inputs: Dict[str, np.ndarray]) -> None:
        for spec in self.config().input:
            if spec.name not in inputs:
                raise InferError(f"missing input '{spec.name}' for model '{self.name}'")
            a = inputs[spec.name]
            dims = list(spec.reshape.shape) if len(spec.reshape.shape) else list(spec.dims)
            if len(dims) != a.ndim and list(spec.dims) and len(spec.dims) != a.ndim:
                raise InferError(f"input '{spec.name}': rank {a.ndim}, expected {len(dims)}")
            ref = dims if len(dims) == a.ndim else list(spec.dims)
            for d, s in zip(ref, a.shape):
                if d != -1 and d != s:
                    raise InferError(f"input '{spec.name}': shape {list(a.shape)} does not match {ref}")

    def __call__(self, inputs: Dict[str, np.ndarray], requested: Sequence[str], encode=None, out_dst=None):
        """Run the model; ``encode(outputs)`` (the response serialiser) runs
        under the model lock too, because GPU models return their reusable
        pinned output staging, which the next request overwrites."""
        t0 = time.perf_counter_ns()
        try:
            if not self.device_inputs and any(getattr(a, "is_cuda", False) for a in inputs.values()):
                inputs = {k: (a.cpu().numpy() if getattr(a, "is_cuda", False) else a) for k, a in inputs.items()}
            self.validate(inputs)
            if self.dynamic_batch > 1:
                if self._batcher is None:
                    with self._lock:
                        if self._batcher is None:
                            self._batcher = DynamicBatcher(self, self.dynamic_batch, self.batch_delay_s)
                t1 = time.perf_counter_ns()
                out = self._batcher.submit(inputs, requested, encode, out_dst)
                if PROFILE.on:
                    PROFILE.add(f"{self.name}.validate", (t1 - t0) * 1e-9)
                    PROFILE.add(f"{self.name}.submit_to_done", (time.perf_counter_ns() - t1) * 1e-9)
            else:
                GPU_PHASE.acquire_shared()
                try:
                    with self._lock, self.stream_context():
                        out = self.execute(inputs, requested)
                        if encode is not None:
                            out = encode(out)
                finally:
                    GPU_PHASE.release_shared()
        except Exception:
            with self.stats.lock:
                self.stats.fail_count += 1
            raise
        dt = time.perf_counter_ns() - t0
        with self.stats.lock:
            self.stats.inference_count += 1
            self.stats.execution_count = (self._batcher.batches if self._batcher is not None
                                          else self.stats.execution_count + 1)
            self.stats.success_ns += dt
            self.stats.compute_ns += dt
            self.stats.last_inference_ms = int(time.time() * 1000)
        return out


class EchoModel(ServedModel):
    """Identity model for protocol tests: output ``OUTPUT{i}`` = ``INPUT{i}``."""

    def __init__(self, name: str = "echo", n: int = 1, dtype: str = "FP32", dims=(-1,)):
        super().__init__(name)
        self.n, self.dtype, self.dims = n, dtype, list(dims)

    def inputs(self):
        return [tensor_spec(f"INPUT{i}", self.dtype, self.dims) for i in range(self.n)]

    def outputs(self):
        return [tensor_spec(f"OUTPUT{i}", self.dtype, self.dims, output=True) for i in range(self.n)]

    def instance_kind(self):
        return mc.ModelInstanceGroup.KIND_CPU

    def execute(self, inputs, requested):
        return {f"OUTPUT{i}": inputs[f"INPUT{i}"] for i in range(self.n)}

    def execute_batch(self, batch, requested):
        return [self.execute(x, requested) for x in batch]
