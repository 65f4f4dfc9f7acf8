"""The served path's host-copy contract: a request built from pinned staging
copies each tensor exactly once (the C++ encoder writing into the bytes gRPC
sends) — no NumPy conversion, no tobytes(), no bytearray -> bytes copy — and
the server's parse gives views into the request bytes."""
import numpy as np
import pytest
import torch

from triton_client_amd import _native
from triton_client_amd.channel import wire
from triton_client_amd.proto import service_pb2


def _native_ok():
    try:
        _native.runtime()
        return True
    except Exception:
        return False


pytestmark = pytest.mark.skipif(not _native_ok(), reason="native runtime not built")


def test_encode_from_staging_is_one_copy(monkeypatch):
    stage = torch.arange(3 * 64 * 64, dtype=torch.float32).reshape(1, 3, 64, 64)
    ids = torch.arange(10, dtype=torch.int32)

    def boom(*a, **k):
        raise AssertionError("host copy outside the encoder")

    monkeypatch.setattr(torch.Tensor, "numpy", boom)
    monkeypatch.setattr(torch.Tensor, "tolist", boom)
    monkeypatch.setattr(torch.Tensor, "contiguous", boom)  # staging is contiguous: no repack either
    monkeypatch.setattr(np, "ascontiguousarray", boom)
    monkeypatch.setattr(wire._Mem, "view", boom)  # the protobuf fallback's copy
    raw = wire.encode_request("m", [("images", stage), ("ids", ids)], ["output"])
    monkeypatch.undo()
    assert type(raw) is bytes
    req = service_pb2.ModelInferRequest()
    req.ParseFromString(raw)
    assert req.raw_input_contents[0] == stage.numpy().tobytes()
    assert req.raw_input_contents[1] == ids.numpy().tobytes()
    assert [list(t.shape) for t in req.inputs] == [[1, 3, 64, 64], [10]]
    assert [t.datatype for t in req.inputs] == ["FP32", "INT32"]


def test_server_parse_is_views_and_response_round_trips():
    a = np.random.default_rng(0).standard_normal((2, 5, 7)).astype(np.float32)
    raw = wire.encode_request("m", [("x", a)], ["y"], "2", "id7")
    p = wire.parse_request(raw)
    assert (p.model_name, p.model_version, p.id, p.outputs) == ("m", "2", "id7", ["y"])
    x = p.inputs["x"]
    assert not x.flags.owndata and not x.flags.writeable  # a view into the request bytes
    np.testing.assert_array_equal(x, a)
    out = torch.from_numpy(a * 2)
    resp = wire.parse_response(wire.encode_response("m", [("y", out)], "2", "id7"))
    np.testing.assert_array_equal(resp["y"], a * 2)


def test_device_tensor_refused():
    if not torch.cuda.is_available():
        t = torch.zeros(2, device="meta")
    else:
        t = torch.zeros(2, device="cuda")
    with pytest.raises(ValueError):
        wire.encode_request("m", [("x", t)])


def test_runtime_published_only_after_signatures(monkeypatch):
    """A thread on runtime()'s lock-free fast path must never get the library
    before its argtypes are declared (pointers would be truncated to C ints:
    the served-path segfault under concurrent first requests)."""
    from triton_client_amd import _runtime_sigs

    seen = []
    real = _runtime_sigs.declare

    def spy(lib):
        seen.append(_native._RUNTIME)
        real(lib)

    monkeypatch.setattr(_native, "_RUNTIME", None)
    monkeypatch.setattr(_runtime_sigs, "declare", spy)
    lib = _native.runtime()
    assert seen == [None] and _native._RUNTIME is lib


def test_concurrent_first_parse_requests():
    """Many threads parse requests while the runtime loads for the first time."""
    import threading

    from triton_client_amd.proto import service_pb2 as pb

    req = pb.ModelInferRequest(model_name="m", id="7")
    t = req.inputs.add(name="x", datatype="FP32", shape=[4, 8])
    req.raw_input_contents.append(np.arange(32, dtype=np.float32).tobytes())
    data = req.SerializeToString()
    _native._RUNTIME = None
    errs = []

    def work():
        try:
            for _ in range(50):
                p = wire.parse_request(data)
                assert p.inputs["x"].shape == (4, 8) and float(p.inputs["x"][3, 7]) == 31.0
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work) for _ in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:3]
