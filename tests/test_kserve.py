"""KServe-v2 protocol: runtime protos vs wire codec, server + channel round
trips over real gRPC on 127.0.0.1 (CPU models)."""
import os
import numpy as np
import pytest

from triton_client_amd.channel.grpc_channel import GRPCChannel
from triton_client_amd.channel.wire import encode_request, parse_response
from triton_client_amd.proto import model_config_pb2 as mc, parse_config_pbtxt, service_pb2 as pb
from triton_client_amd.server import EchoModel, FaultInjector, KServeServer, ModelRepository


class Flags:
    def __init__(self, model_name, model_version="", batch_size=1):
        self.model_name, self.model_version, self.batch_size = model_name, model_version, batch_size


@pytest.fixture()
def echo_server():
    repo = ModelRepository("cpu")
    repo.add(EchoModel("echo", n=2))
    srv = KServeServer(repo, "127.0.0.1:0").start()
    yield srv
    srv.stop()


def test_wire_encoder_matches_protobuf():
    a = np.random.rand(2, 3, 4).astype(np.float32)
    b = np.arange(7, dtype=np.int64)
    raw = encode_request("m", [("x", a), ("y", b)], ["o1", "o2"], "3", "id7")
    ref = pb.ModelInferRequest(model_name="m", model_version="3", id="id7")
    for n, arr, dt in (("x", a, "FP32"), ("y", b, "INT64")):
        t = ref.inputs.add(name=n, datatype=dt)
        t.shape.extend(arr.shape)
        ref.raw_input_contents.append(arr.tobytes())
    ref.outputs.add(name="o1")
    ref.outputs.add(name="o2")
    assert raw == ref.SerializeToString()


def test_wire_parser_zero_copy_views():
    resp = pb.ModelInferResponse(model_name="m")
    arrs = {"boxes": np.random.rand(5, 7).astype(np.float32), "labels": np.arange(5, dtype=np.int64),
            "empty": np.zeros((0, 7), np.float32)}
    for n, a in arrs.items():
        t = resp.outputs.add(name=n, datatype={"float32": "FP32", "int64": "INT64"}[str(a.dtype)])
        t.shape.extend(a.shape)
        resp.raw_output_contents.append(a.tobytes())
    data = resp.SerializeToString()
    pr = parse_response(data)
    assert pr.model_name == "m" and pr.order == list(arrs)
    for n, a in arrs.items():
        np.testing.assert_array_equal(pr[n], a)


def test_reference_config_pbtxt_parses():
    for f in ("examples/YOLOv5/config.pbtxt", "examples/pointpillar_kitti/config.pbtxt",
              "examples/RetinaNet_detectron/config.pbtxt", "examples/YOLOv4/config.pbtxt"):
        import os
        p = os.path.join("/root/reference", f)
        if not os.path.exists(p):
            pytest.skip("reference not mounted")
        cfg = parse_config_pbtxt(open(p).read())
        assert cfg.name and len(cfg.input) >= 1 and len(cfg.output) >= 1


def test_channel_round_trip_echo(echo_server):
    ch = GRPCChannel({"grpc_channel": echo_server.target}, Flags("echo"))
    md = ch.get_metadata()
    assert md["metadata_response"].name == "echo"
    assert [i.name for i in md["metadata_response"].inputs] == ["INPUT0", "INPUT1"]
    x0 = np.random.rand(10).astype(np.float32)
    x1 = np.random.rand(10).astype(np.float32)
    # reference-style mutable request
    for n, x in (("INPUT0", x0), ("INPUT1", x1)):
        t = ch.request.inputs.add(name=n, datatype="FP32")
        t.shape.extend(x.shape)
        ch.request.raw_input_contents.append(x.tobytes())
    ch.request.outputs.add(name="OUTPUT1")
    resp = ch.do_inference()
    assert resp.outputs[0].name == "OUTPUT1"
    np.testing.assert_array_equal(np.frombuffer(resp.raw_output_contents[0], np.float32), x1)
    # fast path
    pr = ch.infer_raw([("INPUT0", x0), ("INPUT1", x1)], ["OUTPUT0", "OUTPUT1"])
    np.testing.assert_array_equal(pr["OUTPUT0"], x0)
    # async + streaming
    fut = ch.do_inference_async()
    assert fut.result().outputs[0].name == "OUTPUT1"
    resps = list(ch.stream_inference([ch.request, ch.request]))
    assert len(resps) == 2 and not resps[0].error_message
    st = ch.model_statistics("echo")
    assert st.model_stats[0].inference_count >= 5
    ch.close()


def test_typed_contents_through_the_default_raw_server(echo_server):
    """A valid KServe request may carry its tensors as typed contents
    (InferInputTensor.contents.fp32_contents) instead of raw_input_contents.  The
    default server parses ModelInfer with the C++ codec, which must flag such an
    input so the request is served by the protobuf path, not rejected as 'missing
    input'."""
    from triton_client_amd.channel.wire import parse_request

    x0 = np.arange(6, dtype=np.float32) * 0.5
    x1 = -np.arange(6, dtype=np.float32)
    req = pb.ModelInferRequest(model_name="echo")
    for n, x in (("INPUT0", x0), ("INPUT1", x1)):
        t = req.inputs.add(name=n, datatype="FP32")
        t.shape.extend(x.shape)
        t.contents.fp32_contents.extend(x.tolist())
    req.outputs.add(name="OUTPUT0")
    req.outputs.add(name="OUTPUT1")
    data = req.SerializeToString()
    pr = parse_request(data)
    assert pr.has_params  # served by the protobuf path
    ch = GRPCChannel({"grpc_channel": echo_server.target}, Flags("echo"))
    ch.request.CopyFrom(req)
    resp = ch.do_inference()
    got = {o.name: np.frombuffer(r, np.float32) for o, r in zip(resp.outputs, resp.raw_output_contents)}
    np.testing.assert_array_equal(got["OUTPUT0"], x0)
    np.testing.assert_array_equal(got["OUTPUT1"], x1)
    ch.close()


def test_server_errors_and_faults():
    repo = ModelRepository("cpu")
    repo.add(EchoModel("echo"))
    fi = FaultInjector(drop_rate=1.0)
    with KServeServer(repo, "127.0.0.1:0", fault=fi) as srv:
        ch = GRPCChannel({"grpc_channel": srv.target}, Flags("echo"), retries=1)
        import grpc
        with pytest.raises(grpc.RpcError) as e:
            ch.infer_raw([("INPUT0", np.ones(3, np.float32))])
        assert e.value.code() == grpc.StatusCode.UNAVAILABLE
        fi.drop_rate = 0.0
        fi.corrupt_rate = 1.0
        pr = ch.infer_raw([("INPUT0", np.ones(3, np.float32))])
        assert (pr["OUTPUT0"] == 0).all()
        fi.corrupt_rate = 0.0
        with pytest.raises(grpc.RpcError) as e:
            ch.infer_raw([("WRONG", np.ones(3, np.float32))])
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        with pytest.raises(ConnectionError):
            GRPCChannel({"grpc_channel": srv.target}, Flags("nope"), wait_ready_s=0.3)
        idx = ch.fetch_channel().RepositoryIndex(pb.RepositoryIndexRequest())
        assert any(m.name == "echo" and m.state == "READY" for m in idx.models)
        ch.close()


class _PickyEcho(EchoModel):
    """Echo that rejects a request whose first value is negative (per-request error in a batch)."""

    def execute(self, inputs, requested):
        from triton_client_amd.server.model import InferError
        if float(inputs["INPUT0"].reshape(-1)[0]) < 0:
            raise InferError("negative")
        return super().execute(inputs, requested)

    def execute_batch(self, batch, requested):
        self.sizes.append(len(batch))
        return [self.execute(x, requested) for x in batch]


def test_dynamic_batching_concurrent_requests_and_isolation():
    """Concurrent batch-1 requests are executed in shared batches (fewer
    executions than requests), every caller gets its own result, and a bad
    request fails alone while the rest of its batch succeeds."""
    import threading

    from triton_client_amd.server.model import InferError

    m = _PickyEcho("echo")
    m.sizes = []
    m.dynamic_batch, m.batch_delay_s = 4, 0.02
    m.load()
    n = 24
    res, errs = [None] * n, [None] * n

    def call(i):
        x = np.full((3,), -1.0 if i == 5 else float(i), np.float32)
        try:
            res[i] = m({"INPUT0": x}, ["OUTPUT0"], encode=lambda o: o["OUTPUT0"].copy())
        except InferError as e:
            errs[i] = e

    ts = [threading.Thread(target=call, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert isinstance(errs[5], InferError) and res[5] is None
    for i in range(n):
        if i != 5:
            assert errs[i] is None and np.array_equal(res[i], np.full((3,), float(i), np.float32))
    assert sum(m.sizes) == n and max(m.sizes) <= 4 and len(m.sizes) < n
    assert m.stats.inference_count == n - 1 and m.stats.fail_count == 1
    m.unload()
    assert m._batcher is None


class _PipelinedEcho(_PickyEcho):
    """A model that claims a GPU and issues batches asynchronously: issue() returns at
    once, finish() blocks until the test releases that batch (the device's work)."""

    def __init__(self, name):
        super().__init__(name)
        import threading
        import types
        self.device = types.SimpleNamespace(type="cuda")
        self.pipeline_depth = 2
        self.sizes, self.sets, self.gates, self.in_flight, self.max_in_flight = [], [], [], 0, 0
        self.mu = threading.Lock()

    def stream_context(self, k=0):
        import contextlib
        return contextlib.nullcontext()

    def execute_batch_async(self, batch, requested, dsts=None, inst=0):
        import threading
        if any(float(x["INPUT0"].reshape(-1)[0]) == 7777.0 for x in batch):
            raise RuntimeError("issue failed")  # the whole batch falls back to per-request execute
        gate = threading.Event()
        with self.mu:
            self.sizes.append(len(batch))
            self.sets.append(inst)
            self.gates.append(gate)
            self.in_flight += 1
            self.max_in_flight = max(self.max_in_flight, self.in_flight)
        outs = []
        for x in batch:
            try:
                outs.append(super().execute(x, requested))
            except Exception as e:  # noqa: BLE001 - a per-request error entry, as the GPU plans return
                outs.append(e)

        def finish():
            assert gate.wait(10)
            with self.mu:
                self.in_flight -= 1
            return outs
        return finish


def test_pipelined_batcher_overlaps_batches_and_isolates_failures():
    """DynamicBatcher._run_pipelined: batch k + 1 is issued on the other plan set while batch k
    is still in flight (two at most), every caller gets its own result, a per-request error
    entry fails only that request, and a batch whose issue raises is re-run request by request."""
    import threading
    import time as _t

    from triton_client_amd.server.model import InferError

    m = _PipelinedEcho("pecho")
    m.dynamic_batch, m.batch_delay_s = 4, 0.01
    m.load()
    assert m.pipelined() and m.plan_set_count() == 2
    n = 24
    res, errs = [None] * n, [None] * n

    def call(i):
        v = -1.0 if i == 5 else (7777.0 if i == 11 else float(i))
        try:
            res[i] = m({"INPUT0": np.full((3,), v, np.float32)}, ["OUTPUT0"], encode=lambda o: o["OUTPUT0"].copy())
        except (InferError, RuntimeError) as e:
            errs[i] = e

    ts = [threading.Thread(target=call, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    released = 0
    deadline = _t.time() + 20
    while any(t.is_alive() for t in ts) and _t.time() < deadline:
        with m.mu:
            gates = list(m.gates)
        if released < len(gates):
            _t.sleep(0.02)  # let the batcher issue the next batch before releasing this one
            gates[released].set()
            released += 1
        else:
            _t.sleep(0.002)
    for t in ts:
        t.join(5)
    assert isinstance(errs[5], InferError)
    assert res[11] is not None and np.array_equal(res[11], np.full((3,), 7777.0, np.float32))  # isolated re-run
    for i in range(n):
        if i not in (5, 11):
            assert errs[i] is None and np.array_equal(res[i], np.full((3,), float(i), np.float32)), i
    assert m.max_in_flight == 2, m.max_in_flight  # overlapped, never more than the plan sets
    assert set(m.sets) == {0, 1}
    m.unload()
    assert m._batcher is None


def test_dynamic_batching_over_grpc():
    import concurrent.futures as cf

    repo = ModelRepository("cpu")
    m = EchoModel("echo", n=1)
    m.dynamic_batch, m.batch_delay_s = 8, 0.01
    repo.add(m)
    with KServeServer(repo, "127.0.0.1:0", max_workers=16) as srv:
        ch = GRPCChannel({"grpc_channel": srv.target}, Flags("echo"))
        xs = [np.arange(4, dtype=np.float32) + i for i in range(16)]
        with cf.ThreadPoolExecutor(16) as ex:
            outs = list(ex.map(lambda x: ch.infer_raw([("INPUT0", x)], ["OUTPUT0"]), xs))
        for x, o in zip(xs, outs):
            np.testing.assert_array_equal(o["OUTPUT0"], x)
        assert m._batcher is not None and m._batcher.batches <= 16
        ch.close()


def test_system_shared_memory_extension_echo():
    """Register / status / unregister, then an inference whose input and output
    live in the client's region: the messages carry only region references."""
    from triton_client_amd.channel.shm import ShmRegion, shm_params
    from triton_client_amd.channel.wire import parse_request
    from triton_client_amd.proto import service_pb2 as pbm

    repo = ModelRepository("cpu")
    repo.add(EchoModel("echo", n=1, dims=(-1, -1)))
    with KServeServer(repo, "127.0.0.1:0") as srv, ShmRegion(1 << 16, pin=False) as reg:
        ch = GRPCChannel({"grpc_channel": srv.target}, Flags("echo"))
        assert "system_shared_memory" in list(ch.server_metadata().extensions)
        ch.register_system_shared_memory("r0", reg.key, reg.byte_size)
        st = ch.system_shared_memory_status()
        assert st.regions["r0"].byte_size == reg.byte_size and st.regions["r0"].key == reg.key
        x = reg.view(0, np.float32, (4, 5))
        x[...] = np.arange(20, dtype=np.float32).reshape(4, 5)
        req = pbm.ModelInferRequest(model_name="echo", id="7")
        t = req.inputs.add(name="INPUT0", datatype="FP32", shape=[4, 5])
        shm_params(t, "r0", 0, 80)
        shm_params(req.outputs.add(name="OUTPUT0"), "r0", 4096, 80)
        raw = req.SerializeToString()
        assert len(raw) < 200 and parse_request(raw).has_params
        resp = pbm.ModelInferResponse.FromString(ch._grpc_stub.ModelInferRaw(raw))
        assert list(resp.outputs[0].shape) == [4, 5] and len(resp.raw_output_contents) == 0
        np.testing.assert_array_equal(reg.view(4096, np.float32, (4, 5)), x)
        # a slice past the region is a client error
        bad = pbm.ModelInferRequest(model_name="echo")
        shm_params(bad.inputs.add(name="INPUT0", datatype="FP32", shape=[1 << 15, 1]), "r0", 0, 4 << 15)
        import grpc
        with pytest.raises(grpc.RpcError) as ei:
            ch._grpc_stub.ModelInfer(bad)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        ch.unregister_system_shared_memory("r0")
        assert len(ch.system_shared_memory_status().regions) == 0
        ch.close()


def test_gpu_phase_lock_prefers_a_waiting_writer():
    """Under continuous overlapping executions (shared holders) a model load
    (exclusive) must still get in: once a writer waits, new readers queue."""
    import threading
    import time

    from triton_client_amd.server.model import _RWLock

    lk = _RWLock()
    lk.acquire_shared()  # an execution in flight
    order = []
    w = threading.Thread(target=lambda: (lk.acquire_exclusive(), order.append("w"), lk.release_exclusive()))
    w.start()
    time.sleep(0.05)  # the writer is waiting now
    r = threading.Thread(target=lambda: (lk.acquire_shared(), order.append("r"), lk.release_shared()))
    r.start()
    time.sleep(0.05)
    assert order == []  # the new reader yields to the pending writer
    lk.release_shared()
    w.join(2)
    r.join(2)
    assert order == ["w", "r"]


def test_shm_unregister_waits_for_in_flight_executions(tmp_path):
    """Unpinning a registered region must not race an execution that may be
    DMA'ing from it: unregister waits until no execution holds GPU_PHASE."""
    import os
    import threading
    import time

    from triton_client_amd.server.model import GPU_PHASE
    from triton_client_amd.server.shm import SharedMemoryRegistry

    key = f"tca_test_{os.getpid()}"
    path = os.path.join("/dev/shm", key)
    with open(path, "wb") as f:
        f.write(bytes(4096))
    try:
        reg = SharedMemoryRegistry(pin=False)
        reg.register("r0", key, 0, 4096)
        GPU_PHASE.acquire_shared()  # an execution in flight
        done = threading.Event()
        t = threading.Thread(target=lambda: (reg.unregister("r0"), done.set()))
        t.start()
        time.sleep(0.05)
        assert not done.is_set()
        GPU_PHASE.release_shared()
        t.join(2)
        assert done.is_set() and reg.status() == []
    finally:
        os.unlink(path)


def test_device_region_lease_defers_close(monkeypatch):
    """A device region a queued request still holds stays mapped through an
    unregister (its name is gone at once); the last release closes it.  A region
    on another device than the server's models is refused."""
    import torch

    from triton_client_amd.server.model import InferError
    from triton_client_amd.server.shm import Region, SharedMemoryRegistry

    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    closed = []

    class Dev:
        device = "cpu"

        def close(self):
            closed.append(1)

    reg = SharedMemoryRegistry(pin=False, device_id=0)
    reg._regions["a"] = Region("a", "", 0, 64, None, dev=Dev())
    held = reg.lease(["a", "a"])
    assert len(held) == 1 and held[0].inflight == 1
    reg.unregister("", device=True)  # "unregister all", e.g. from another client
    assert closed == [] and reg.status(device=True) == []
    with pytest.raises(InferError):
        reg.lease(["a"])
    reg.release(held)
    assert closed == [1]
    reg._regions["b"] = Region("b", "", 0, 64, None, dev=Dev())
    reg.release(reg.lease(["b"]))  # not unregistered: stays open
    reg.unregister("b", device=True)
    assert closed == [1, 1]
    with pytest.raises(InferError, match="device 1"):
        reg.register_device("c", bytes(64), 1, 64)


def test_multi_process_server_shares_the_port_and_stops_cleanly():
    """--procs 3: three server processes on one port (SO_REUSEPORT); every connection is
    served, and SIGTERM to the parent ends the children too (the port is free again)."""
    import socket
    import subprocess
    import sys
    import time

    import grpc

    from triton_client_amd.channel.wire import encode_request, parse_response
    from triton_client_amd.proto import SERVICE

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-m", "triton_client_amd.server", "--host", "127.0.0.1", "--port", str(port),
                          "--models", "echo", "--device", "cpu", "--metrics-port", "0", "--procs", "3"], cwd=root)
    try:
        deadline = time.time() + 120
        served = 0
        for i in range(6):
            while True:
                ch = grpc.insecure_channel(f"127.0.0.1:{port}")
                f = ch.unary_unary(f"/{SERVICE}/ModelInfer", request_serializer=None, response_deserializer=None)
                try:
                    x = np.arange(4 + i, dtype=np.float32)
                    r = parse_response(f(encode_request("echo", [("INPUT0", x)]), timeout=20))
                    assert np.array_equal(r["OUTPUT0"], x)
                    served += 1
                    break
                except grpc.RpcError:
                    assert time.time() < deadline, "server did not come up"
                    time.sleep(0.5)
                finally:
                    ch.close()
        assert served == 6
    finally:
        p.terminate()
        assert p.wait(60) == 0
    with socket.socket() as sk:  # no child process still listens on the port
        # (SO_REUSEADDR: closed connections in TIME_WAIT must not count, a listener still does)
        sk.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        sk.bind(("127.0.0.1", port))
