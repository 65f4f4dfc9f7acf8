"""Detectron2 RetinaNet / FCOS (ResNet-50-FPN): fused plan vs module, decode, kernels."""
import numpy as np
import pytest
import torch

from triton_client_amd.config.detectron import DetectronConfig
from triton_client_amd.models.common import fuse_model, randomize_bn
from triton_client_amd.models.detectron import build_detectron, decode_reference
from triton_client_amd.ops.conv import NHWC


def _model(arch, hw=(128, 160), seed=0):
    cfg = DetectronConfig(arch=arch, input_hw=hw, num_classes=8)
    m = build_detectron(cfg, seed)
    randomize_bn(m, 4)
    m = fuse_model(m.eval())
    with torch.no_grad():  # keep activations O(1) through 16 residual blocks (random init)
        for blk in m.backbone.stages.modules():
            if hasattr(blk, "conv3"):
                blk.conv3.conv.weight.mul_(0.2)
        if arch == "fcos":
            for gn in [x for x in m.head.modules() if isinstance(x, torch.nn.GroupNorm)]:
                gn.weight.uniform_(0.5, 1.5)
                gn.bias.uniform_(-0.2, 0.2)
    return m


def _fast_inputs(m, x):
    """NHWC x8 normalised input for the plan (what K1 writes)."""
    xn = (x - m.mean) / m.std
    z = torch.zeros(x.shape[0], x.shape[2], x.shape[3], 8)
    z[..., :3] = xn.permute(0, 2, 3, 1)
    return z


@pytest.mark.parametrize("arch", ["retinanet", "fcos"])
def test_fast_detectron_cpu_matches_module(arch):
    from triton_client_amd.models.fast import FastDetectron
    m = _model(arch)
    x = torch.rand(2, 3, 128, 160) * 255
    with torch.no_grad():
        ref = m(x)
        f = FastDetectron(m, 2, device="cpu")
        f.x.t.copy_(_fast_inputs(m, x))
        outs = f.forward()
    assert f.level_hw == [tuple(r[0].shape[2:]) for r in ref] == m.cfg.level_hw()
    for r, o in zip(ref, outs):
        for rt, ot in zip(r, o):
            torch.testing.assert_close(ot.nchw(), rt, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("arch", ["retinanet", "fcos"])
def test_decode_reference_and_postprocess_cpu(arch):
    from triton_client_amd.ops.detectron import DetectronPostprocess
    m = _model(arch)
    cfg = m.cfg
    with torch.no_grad():
        ref = m(torch.rand(1, 3, 128, 160) * 255)
    # shift the class logits so a few hundred candidates pass the threshold
    ref = [tuple(t + (2.5 if i == 0 else 0.0) for i, t in enumerate(o)) for o in ref]
    res = decode_reference(ref, cfg)[0]
    assert 0 < len(res[1]) <= cfg.max_detections
    assert (np.diff(res[1]) <= 1e-7).all() and (res[0][:, 2] >= res[0][:, 0]).all()
    pp = DetectronPostprocess(cfg, 1, device="cpu")
    outs = [tuple(NHWC(t.permute(0, 2, 3, 1).contiguous()) for t in o) for o in ref]
    got = pp(outs).per_image()[0]
    np.testing.assert_allclose(got["score"], res[1], rtol=1e-6)


@pytest.mark.gpu
def test_group_norm_kernel(cuda):
    from triton_client_amd.ops.detectron import group_norm_nhwc
    x = torch.randn(2, 13, 21, 256 + 16) * 3 + 1
    g, b = torch.rand(256) + 0.5, torch.randn(256) * 0.1
    xg = x.to(cuda, torch.bfloat16)
    out = torch.zeros_like(xg)
    group_norm_nhwc(NHWC(xg, 16, 256), g.to(cuda), b.to(cuda), 32, 1e-5, True, out=NHWC(out, 16, 256))
    torch.cuda.synchronize()
    ref = torch.relu(torch.nn.functional.group_norm(xg[..., 16:].float().cpu().permute(0, 3, 1, 2), 32, g, b, 1e-5))
    got = out[..., 16:].float().cpu().permute(0, 3, 1, 2)
    assert (got - ref).abs().max().item() < 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["retinanet", "fcos"])
def test_detectron_decode_gpu_matches_cpu(cuda, arch):
    from triton_client_amd.ops.detectron import DetectronPostprocess
    m = _model(arch)
    cfg = m.cfg
    with torch.no_grad():
        ref = m(torch.rand(2, 3, 128, 160) * 255)
    ref = [tuple(t + (2.5 if i == 0 else 0.0) for i, t in enumerate(o)) for o in ref]
    cpu = DetectronPostprocess(cfg, 2, device="cpu")([tuple(NHWC(t.permute(0, 2, 3, 1).contiguous()) for t in o)
                                                      for o in ref]).per_image()
    gpu = DetectronPostprocess(cfg, 2, device=cuda)([tuple(NHWC(t.permute(0, 2, 3, 1).contiguous().to(cuda))
                                                           for t in o) for o in ref])
    torch.cuda.synchronize()
    for c, g in zip(cpu, gpu.per_image()):
        assert abs(len(c["score"]) - len(g["score"])) <= 2
        k = min(len(c["score"]), len(g["score"]), 30)
        np.testing.assert_allclose(g["score"][:k], c["score"][:k], rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["retinanet", "fcos"])
def test_fast_detectron_gpu_vs_fp32(cuda, arch):
    from triton_client_amd.models.fast import FastDetectron
    m = _model(arch)
    x = torch.rand(2, 3, 128, 160) * 255
    with torch.no_grad():
        ref = m(x)
    f = FastDetectron(m, 2, device=cuda)
    f.x.t.copy_(_fast_inputs(m, x).to(cuda))
    outs = f.forward()
    torch.cuda.synchronize()
    for r, o in zip(ref, outs):
        for rt, ot in zip(r, o):
            err = (ot.nchw().float().cpu() - rt).abs().max().item()
            assert err < 0.08 * max(1.0, rt.abs().max().item()), err


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["retinanet", "fcos"])
def test_detectron_pipeline_graph(cuda, arch):
    from triton_client_amd.pipelines import DetectronPipeline, GraphRunner
    from triton_client_amd.utils.synthetic import camera_frame
    cfg = DetectronConfig(arch=arch, input_hw=(256, 384))
    pipe = DetectronPipeline(batch=2, src_hw=(360, 640), cfg=cfg, device=cuda)
    for b in range(2):
        pipe.frames[b].copy_(torch.from_numpy(camera_frame(360, 640, b)))
    d = pipe.calibrate_detection_density(200.0)
    assert -30 < d < 30
    e = pipe.step().per_image()
    torch.cuda.synchronize()
    run = GraphRunner(pipe.step)
    g1 = run().per_image()
    g2 = run().per_image()
    assert all(len(x["score"]) > 0 for x in e)
    for a, b in zip(g1, g2):
        np.testing.assert_array_equal(a["box"], b["box"])
    for x in e:
        assert x["box"][:, [0, 2]].max() <= 640 + 1e-3 and x["box"][:, [1, 3]].max() <= 360 + 1e-3
        assert len(x["score"]) <= cfg.max_detections


@pytest.mark.gpu
def test_detectron_served_contract(cuda):
    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import FCOS_client, client_for_model
    from triton_client_amd.inference import RemoteDetector2D
    from triton_client_amd.server import KServeServer, ModelRepository
    from triton_client_amd.utils.synthetic import camera_frame
    repo = ModelRepository("cuda")
    repo.load("test_model")
    with KServeServer(repo, "127.0.0.1:0") as srv:
        class F:
            model_name, model_version, batch_size = "test_model", "", 1
        ch = GRPCChannel({"grpc_channel": srv.target}, F())
        cfg = ch.get_metadata()["config_response"].config
        assert [o.name for o in cfg.output] == ["bboxex__0", "classes__1", "scores__2", "dims__3"]
        client = client_for_model("test_model", cfg)
        assert isinstance(client, FCOS_client)
        eng = RemoteDetector2D(ch, client, conf_thres=0.05)
        d = eng.detect([camera_frame(480, 640, 3)])[0]
        assert d.shape[1] == 6 and len(d) > 0
        ch.close()


@pytest.mark.gpu
def test_served_test_model_fp32_matches_local_engine(cuda):
    """The served ``test_model`` (RetinaNet, examples/RetinaNet_detectron/config.pbtxt:
    FP32 input__00 [3, 640, 480]) runs the fp32 plan, normalisation folded into the
    input-layout kernel, as a captured batch plan; its kept set equals the local fp32
    engine's on the same frame (stretch at the model size: the same input values),
    singly and inside a dynamic batch."""
    from triton_client_amd.inference.engines import LocalDetector2D
    from triton_client_amd.server.models import DetectronModel
    from triton_client_amd.utils.synthetic import camera_frame

    served = DetectronModel("test_model", device=cuda)
    served.load()
    assert served.pipe.precision == "fp32"
    assert next(served.model.parameters()).dtype == torch.float32
    local = LocalDetector2D(family="retinanet", img=(640, 480), batch=2, letterbox=False, device=cuda)
    local.calibrate_synthetic(0)
    frame = camera_frame(640, 480, 11)
    want = local.detect([frame])[0]
    x = np.ascontiguousarray(frame.transpose(2, 0, 1)).astype(np.float32)
    one = served.execute({"input__00": x}, None)
    many = served.execute_batch([{"input__00": x}, {"input__00": x[:, ::-1].copy()}, {"input__00": x}], None)
    assert len(want) > 0

    def unmatched(box, score, cls):
        """Kept-set comparison independent of output order (NMS breaks near-ties freely, and the
        two paths' scores differ in the last bits): each expected detection must pair with an
        unused served one of the same class, box within 2e-3 px + 1e-4 relative, score within 1e-4."""
        used = np.zeros(len(score), bool)
        miss = 0
        for row in want:
            ok = (~used & (cls == row[5]) & (np.abs(score - row[4]) <= 1e-4)
                  & np.all(np.abs(box - row[None, :4]) <= 2e-3 + 1e-4 * np.abs(row[None, :4]), 1))
            idx = np.flatnonzero(ok)
            if len(idx) == 0:
                miss += 1
            else:
                used[idx[np.argmin(np.abs(score[idx] - row[4]))]] = True
        return miss
    for got in (one, many[0], many[2]):
        assert got["dims__3"].tolist() == [[640, 480]]
        assert len(got["scores__2"]) == len(want)
        assert unmatched(got["bboxex__0"], got["scores__2"], got["classes__1"]) == 0


def test_reference_model_repository_families():
    """Every config.pbtxt of the reference maps to a served model family with the
    same tensor contract (no model is loaded)."""
    import os
    import shutil
    import tempfile
    from triton_client_amd.server.repository import ModelRepository
    root = tempfile.mkdtemp()
    try:
        for d, f in (("YOLOv5nCROP", "examples/YOLOv5/config.pbtxt"), ("YOLOv4", "examples/YOLOv4/config.pbtxt"),
                     ("test_model", "examples/RetinaNet_detectron/config.pbtxt"),
                     ("pointpillar_kitti", "examples/pointpillar_kitti/config.pbtxt")):
            src = os.path.join("/root/reference", f)
            if not os.path.exists(src):
                pytest.skip("reference configs not mounted")
            os.makedirs(os.path.join(root, d))
            shutil.copy(src, os.path.join(root, d, "config.pbtxt"))
        repo = ModelRepository.from_directory(root, device="cpu", load=False)
        by = {m.name: m for m in repo.models()}
        assert type(by["YOLOv4"]).__name__ == "YoloV4Model"
        assert [o.name for o in by["YOLOv4"].config().output] == ["confs", "boxes"]
        assert list(by["YOLOv4"].config().output[0].dims) == [1, 16128, 80]
        assert type(by["test_model"]).__name__ == "DetectronModel"
        assert list(by["test_model"].config().input[0].dims) == [3, 640, 480]
        assert [o.name for o in by["test_model"].config().output] == ["bboxex__0", "classes__1", "scores__2", "dims__3"]
        assert type(by["pointpillar_kitti"]).__name__ == "PointPillarsModel"
    finally:
        shutil.rmtree(root)


@pytest.mark.gpu
def test_group_norm_kernel_fp32(cuda):
    from triton_client_amd.ops.detectron import group_norm_nhwc
    x = torch.randn(2, 13, 21, 256 + 16) * 3 + 1
    g, b = torch.rand(256) + 0.5, torch.randn(256) * 0.1
    xg = x.to(cuda)
    out = torch.zeros_like(xg)
    group_norm_nhwc(NHWC(xg, 16, 256), g.to(cuda), b.to(cuda), 32, 1e-5, True, out=NHWC(out, 16, 256))
    torch.cuda.synchronize()
    ref = torch.relu(torch.nn.functional.group_norm(x[..., 16:].double().permute(0, 3, 1, 2), 32, g.double(),
                                                    b.double(), 1e-5))
    got = out[..., 16:].double().cpu().permute(0, 3, 1, 2)
    assert (got - ref).abs().max().item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["retinanet", "fcos"])
def test_fast_detectron_fp32_vs_fp64_module(cuda, arch):
    """fp32 mode (the reference's libtorch fp32 serving precision): split-product
    convs, fp32 activations, fp32 GroupNorm, against the fp64 module."""
    import copy

    from triton_client_amd.models.fast import FastDetectron
    m = _model(arch)
    x = torch.rand(2, 3, 128, 160) * 255
    with torch.no_grad():
        ref = copy.deepcopy(m).double()(x.double())
    f = FastDetectron(m, 2, device=cuda, precision="fp32")
    assert f.x.t.dtype == torch.float32
    f.x.t.copy_(_fast_inputs(m, x).to(cuda))
    outs = f.forward()
    torch.cuda.synchronize()
    for r, o in zip(ref, outs):
        for rt, ot in zip(r, o):
            got = ot.nchw().double().cpu()
            rel = ((got - rt).norm() / rt.norm().clamp_min(1e-30)).item()
            assert rel < 1e-4, rel


@pytest.mark.gpu
def test_detectron_pipeline_fp32(cuda):
    from triton_client_amd.pipelines import DetectronPipeline, GraphRunner
    from triton_client_amd.utils.synthetic import camera_frame
    cfg = DetectronConfig(arch="retinanet", input_hw=(256, 384))
    pipe = DetectronPipeline(batch=2, src_hw=(360, 640), cfg=cfg, device=cuda, precision="fp32")
    for b in range(2):
        pipe.frames[b].copy_(torch.from_numpy(camera_frame(360, 640, b)))
    pipe.calibrate_detection_density(200.0)
    e = pipe.step().per_image()
    g = GraphRunner(pipe.step)().per_image()
    torch.cuda.synchronize()
    assert all(len(x["score"]) > 0 for x in e)
    for a, b in zip(e, g):
        np.testing.assert_array_equal(a["box"], b["box"])
