"""YOLOv4 (CSPDarknet53-SPP-PANet): layer graph, fused plan, K5 decode, served contract."""
import numpy as np
import pytest
import torch

from triton_client_amd.models.common import fuse_model, randomize_bn
from triton_client_amd.models.yolov4 import YOLOV4_OUTPUTS, build_yolov4, decode_reference, post_processing


def _model(img=128, seed=0):
    m = build_yolov4(80, img, seed)
    randomize_bn(m, 5)
    m = fuse_model(m.eval())
    with torch.no_grad():  # tame the random-init activations (calibration does this on the GPU path)
        for name, mod in m.layers.items():
            mod.conv.weight.mul_(0.35)
    return m


def test_fast_graph_cpu_matches_module():
    from triton_client_amd.models.fast import FastGraph
    m = _model()
    x = torch.rand(2, 3, 128, 128)
    with torch.no_grad():
        ref = m(x)
        f = FastGraph(m, 2, (128, 128), device="cpu", outputs=YOLOV4_OUTPUTS)
        f.input_view()[:, :3].copy_(x)
        outs = f.forward()
    assert sum(1 for o in f.ops if o[0] in ("copy", "add")) == 0  # every route in place, every add fused
    for r, o in zip(ref, outs):
        torch.testing.assert_close(o.nchw()[:, :255], r, rtol=1e-4, atol=1e-4)


def test_decode_matches_reference_semantics():
    """boxes/confs layout of yolo_forward_dynamic: rows anchor-major per level."""
    m = _model()
    with torch.no_grad():
        outs = m(torch.rand(1, 3, 128, 128))
    boxes, confs = decode_reference(outs, 80)
    assert boxes.shape == (1, 3 * (16 * 16 + 8 * 8 + 4 * 4), 1, 4) and confs.shape[2] == 80
    # row 1 of level 0 = anchor 0, y 0, x 1: centre x = (sig(tx) + 1) / W
    o = outs[0][0].float().view(3, 85, 16, 16)
    cx = (torch.sigmoid(o[0, 0, 0, 1]) + 1) / 16
    assert abs(((boxes[0, 1, 0, 0] + boxes[0, 1, 0, 2]) / 2).item() - cx.item()) < 1e-6
    per = post_processing(boxes.numpy(), confs.numpy(), 0.0, 0.6)[0]
    assert per.shape[1] == 6 and len(per) > 0


@pytest.mark.gpu
def test_yolov4_decode_gpu_matches_cpu(cuda):
    from triton_client_amd.ops.conv import NHWC
    from triton_client_amd.ops.yolov4 import Yolov4Postprocess
    m = _model()
    with torch.no_grad():
        outs = m(torch.rand(2, 3, 128, 128))
    outs = [o + torch.tensor([0, 0, 0, 0, 2.0] + [2.0] * 80).repeat(3).view(1, -1, 1, 1) for o in outs]
    nh = [NHWC(torch.nn.functional.pad(o, (0, 0, 0, 0, 0, 1)).permute(0, 2, 3, 1).contiguous()) for o in outs]
    cpu = Yolov4Postprocess(80, (128, 128), device="cpu")(nh, full=True)
    gpu = Yolov4Postprocess(80, (128, 128), device=cuda)([NHWC(h.t.to(cuda)) for h in nh], full=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(gpu[1].cpu().numpy(), cpu[1].numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gpu[2].cpu().numpy(), cpu[2].numpy(), rtol=1e-4, atol=1e-6)
    for c, g in zip(cpu[0].per_image(), gpu[0].per_image()):
        assert abs(len(c["score"]) - len(g["score"])) <= 2
        k = min(len(c["score"]), len(g["score"]), 40)
        np.testing.assert_allclose(np.sort(g["score"])[::-1][:k], np.sort(c["score"])[::-1][:k], rtol=1e-5)


@pytest.mark.gpu
def test_yolov4_pipeline_and_served_model(cuda):
    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov4client, client_for_model
    from triton_client_amd.inference import RemoteDetector2D
    from triton_client_amd.pipelines import GraphRunner, Yolov4Pipeline
    from triton_client_amd.server import KServeServer, ModelRepository
    from triton_client_amd.utils.synthetic import camera_frame
    pipe = Yolov4Pipeline(batch=2, src_hw=(360, 640), img=256, device=cuda)
    for b in range(2):
        pipe.frames[b].copy_(torch.from_numpy(camera_frame(360, 640, b)))
    pipe.calibrate_detection_density(50.0)
    run = GraphRunner(pipe.step)
    g1, g2 = run().per_image(), run().per_image()
    assert sum(len(x["score"]) for x in g1) > 0  # the calibrated prior is a per-batch average
    for a, b in zip(g1, g2):
        np.testing.assert_array_equal(a["box"], b["box"])
    repo = ModelRepository("cuda")
    repo.load("YOLOv4")
    with KServeServer(repo, "127.0.0.1:0") as srv:
        class F:
            model_name, model_version, batch_size = "YOLOv4", "", 1
        ch = GRPCChannel({"grpc_channel": srv.target}, F())
        client = client_for_model("YOLOv4", ch.get_metadata()["config_response"].config)
        assert isinstance(client, Yolov4client)
        d = RemoteDetector2D(ch, client).detect([camera_frame(480, 640, 1)])[0]
        assert d.shape[1] == 6 and len(d) > 0
        assert d[:, [0, 2]].max() <= 640 + 1e-3
        ch.close()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_fast_graph_gpu_vs_fp64_module(cuda, precision):
    """The YOLOv4 plan against an fp64 evaluation of the fused module: relative
    L2 per head below the precision's bound (fp32 split-product 2e-4, bf16 2e-2;
    tests/test_fast_plans.py PLAN_REL_L2)."""
    from triton_client_amd.models.fast import FastGraph
    m = _model()
    x = torch.rand(2, 3, 128, 128)
    with torch.no_grad():
        ref = m.double()(x.double())
    dt = torch.float32 if precision == "fp32" else torch.bfloat16
    f = FastGraph(m.float().to(cuda, dt), 2, (128, 128), device=cuda, outputs=YOLOV4_OUTPUTS, precision=precision)
    f.input_view()[:, :3].copy_(x.to(cuda, dt))
    outs = f.forward()
    torch.cuda.synchronize()
    assert outs[0].t.dtype == dt
    errs = []
    for r, o in zip(ref, outs):
        g = o.nchw()[:, :255].double().cpu()
        errs.append(((g - r).norm() / r.norm()).item())
    print(precision, "yolov4 rel L2", errs)
    assert max(errs) < {"fp32": 2e-4, "bf16": 2e-2}[precision], errs
