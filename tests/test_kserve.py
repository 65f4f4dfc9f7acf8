"""KServe-v2 protocol: runtime protos vs wire codec, server + channel round
trips over real gRPC on 127.0.0.1 (CPU models)."""
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
