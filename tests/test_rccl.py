"""Native RCCL communicator (csrc/runtime/rccl_comm.cpp, parallel/rccl.py).

CPU: the runtime library exports the communicator ABI with declared argtypes.
GPU (world 1 — a one-GPU box cannot hold two ranks of one RCCL communicator):
grouped send/recv to self, MAX all-reduce, broadcast, async-error polling and
the FrameExchange plumbing through the native path."""
import pytest
import torch

from triton_client_amd import _native

SYMS = ("tca_rccl_unique_id_bytes", "tca_rccl_get_unique_id", "tca_rccl_comm_init", "tca_rccl_comm_destroy",
        "tca_rccl_comm_abort", "tca_rccl_async_error", "tca_rccl_error_string", "tca_rccl_group_p2p",
        "tca_rccl_allreduce_max_f64", "tca_rccl_broadcast", "tca_rccl_comm_count")


def test_runtime_exports_rccl_abi():
    lib = _native.runtime()
    for s in SYMS:
        assert getattr(lib, s).argtypes is not None, s
    assert lib.tca_rccl_unique_id_bytes() == 128
    assert lib.tca_rccl_error_string(0) == b"no error"


@pytest.mark.gpu
def test_native_comm_world1():
    from triton_client_amd.parallel.rccl import RECV, SEND, NativeComm

    torch.cuda.set_device(0)
    comm = NativeComm(0, 1)
    try:
        assert comm.async_error() is None
        assert comm.count() == 1
        a = torch.arange(1000, dtype=torch.float32, device="cuda")
        b = torch.empty_like(a)
        odd_src = torch.arange(7, dtype=torch.uint8, device="cuda")  # byte path (7 B)
        odd_dst = torch.zeros_like(odd_src)
        comm.group_p2p([(SEND, a, 0), (RECV, b, 0), (SEND, odd_src, 0), (RECV, odd_dst, 0)])
        torch.cuda.synchronize()
        assert torch.equal(a, b) and torch.equal(odd_src, odd_dst)
        t = torch.tensor([3.5, -1.0], dtype=torch.float64, device="cuda")
        comm.allreduce_max_(t)
        x = torch.randn(33, device="cuda")
        y = x.clone()
        comm.broadcast_(y, 0)
        torch.cuda.synchronize()
        assert t.tolist() == [3.5, -1.0] and torch.equal(x, y)
        with pytest.raises(ValueError):
            comm.group_p2p([(SEND, a.cpu(), 0)])
        with pytest.raises(ValueError):
            comm.group_p2p([(SEND, a, 1)])
        assert comm.async_error() is None
    finally:
        comm.close()


@pytest.mark.gpu
def test_frame_exchange_native_ops():
    """FrameExchange's op list through the native group on one rank."""
    from triton_client_amd.parallel.dp import DistInfo, FrameExchange
    from triton_client_amd.parallel.rccl import NativeComm

    comm = NativeComm(0, 1)
    try:
        ex = FrameExchange(DistInfo(0, 1, 0, torch.device("cuda", 0)), native=comm)
        src = torch.randint(0, 255, (3, 64, 64, 3), dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        ex._run([(0, src, 0), (1, dst, 0)])
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
    finally:
        comm.close()


@pytest.mark.gpu
def test_native_p2p_plan_graph_capture():
    """The grouped p2p plan is plain stream work: it can be captured into a
    hipGraph with the pipeline step and replayed (the bench's in-graph gather)."""
    from triton_client_amd.parallel.rccl import RECV, SEND, NativeComm

    torch.cuda.set_device(0)
    comm = NativeComm(0, 1)
    try:
        a = torch.arange(4096, dtype=torch.float32, device="cuda")
        b = torch.zeros_like(a)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            comm.group_p2p([(SEND, a, 0), (RECV, b, 0)])  # warm-up outside capture
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            a.add_(1.0)
            comm.group_p2p([(SEND, a, 0), (RECV, b, 0)])
        b.zero_()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        ok = torch.equal(b, torch.arange(4096, dtype=torch.float32, device="cuda") + 2.0)
        del g  # the graph holds RCCL work: release it before the communicator goes
        torch.cuda.synchronize()
        assert ok
    finally:
        comm.abort()  # never block on teardown of a communicator a graph has used


@pytest.mark.gpu
def test_native_gather_plan_in_step_graph():
    """The bench's in-graph detection gather: a step producing the detection buffers
    (mixed dtypes: boxes / scores fp32, classes / counts int32, as the 2D and 3D
    results) followed by the grouped gather plan, captured as ONE graph with
    GraphRunner and replayed.  At world 1 the peer is this rank itself: rank 0's
    receives and a worker's sends of the same plan, in one RCCL group."""
    from triton_client_amd.parallel.rccl import RECV, SEND, NativeComm
    from triton_client_amd.pipelines.graph import GraphRunner

    torch.cuda.set_device(0)
    comm = NativeComm(0, 1)
    try:
        seed = torch.zeros(1, device="cuda")
        src = [torch.zeros((32, 300, 4), device="cuda"), torch.zeros((32, 300), device="cuda"),
               torch.zeros((32, 300), dtype=torch.int32, device="cuda"),
               torch.zeros((32,), dtype=torch.int32, device="cuda"), torch.zeros((32, 500, 7), device="cuda")]
        dst = [torch.empty_like(t) for t in src]

        def step():
            for k, t in enumerate(src):  # the "pipeline": every result buffer rewritten from the input
                t.copy_((seed + k).expand_as(t).to(t.dtype) if t.dtype != torch.int32 else (seed + k).to(torch.int32).expand_as(t))
            comm.group_p2p([(RECV, d, 0) for d in dst] + [(SEND, s, 0) for s in src])
            return src
        run = GraphRunner(step)
        for v in (3.0, 7.0, 11.0):
            seed.fill_(v)
            run()
            torch.cuda.synchronize()
            for k, (d, s) in enumerate(zip(dst, src)):
                assert torch.equal(d, s) and float(d.reshape(-1)[0]) == v + k
        run.release()  # the graph holds RCCL work: release it before the communicator goes
    finally:
        comm.abort()


@pytest.mark.gpu
def test_native_gather_plan_in_two_double_buffered_graphs():
    """The bench's default double-buffered step with the gather inside: two graphs,
    one per input set, each capturing its own copy of the grouped plan over the ONE
    communicator and gathering into its own receive buffers, replayed alternately
    (what every rank does, in the same order) — each replay delivers its own step."""
    from triton_client_amd.parallel.rccl import RECV, SEND, NativeComm
    from triton_client_amd.pipelines.graph import GraphRunner

    torch.cuda.set_device(0)
    comm = NativeComm(0, 1)
    runs = []
    try:
        inputs = [torch.zeros(1, device="cuda"), torch.zeros(1, device="cuda")]
        src = [torch.zeros((32, 300, 4), device="cuda"), torch.zeros((32,), dtype=torch.int32, device="cuda")]
        dst = [[torch.empty_like(t) for t in src] for _ in range(2)]

        def step(k):
            def fn():
                src[0].copy_(inputs[k].expand_as(src[0]))
                src[1].copy_(inputs[k].to(torch.int32).expand_as(src[1]))
                comm.group_p2p([(RECV, d, 0) for d in dst[k]] + [(SEND, s, 0) for s in src])
                return src
            return fn
        runs += [GraphRunner(step(0)), GraphRunner(step(1))]
        for run in runs:
            run.capture()
        for t, v in enumerate((2.0, 5.0, 9.0, 13.0)):
            k = t % 2
            inputs[k].fill_(v)
            runs[k]()
            torch.cuda.synchronize()
            assert float(dst[k][0].reshape(-1)[0]) == v and int(dst[k][1][0]) == int(v)
            if t:  # the other set still holds the previous step's gather
                prev = (2.0, 5.0, 9.0, 13.0)[t - 1]
                assert float(dst[1 - k][0].reshape(-1)[-1]) == prev
    finally:
        for r in runs:  # the graphs go before the communicator (GraphRunner.release)
            r.release()
        comm.abort()


@pytest.mark.gpu
def test_native_selftest_world1():
    """bench.py's pre-flight of the native communicator (parallel/rccl.py native_selftest): the
    gather plan eagerly and in two alternately replayed graphs, values checked on rank 0."""
    from triton_client_amd.parallel.rccl import NativeComm, native_selftest

    torch.cuda.set_device(0)
    comm = NativeComm(0, 1)
    try:
        ok, why = native_selftest(comm, 0, 1, timeout_s=30)
        assert ok, why
    finally:
        comm.abort()
