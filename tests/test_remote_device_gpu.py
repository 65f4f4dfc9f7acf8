"""The reference's default architecture — ``main.py`` / ``main3d.py`` as a KServe
client of a model server — with the client's per-frame numerics on the MI355X.

* K3 on a decoded response (``tca_yolo_filter_decoded``) + K4 against the CPU
  postprocess (``--device cpu``, config 1): the same kept sets.
* ``main.py -m YOLOv5nCOCO`` and ``main3d.py -m pointpillar_kitti`` with default
  flags against the in-process server: the device path runs (GPU decode,
  preprocess, K3/K4, voxeliser) and publishes what the CPU client publishes.
Reference: ``communicator/ros_inference.py:117-175``,
``communicator/ros_inference3d.py:120-150``, ``clients/preprocess/preprocess_3d.py:30-52``,
``clients/postprocess/yolov5_postprocess.py:28-125``.
"""
import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu


def _pred(B, N, nc, seed=0):
    rng = np.random.default_rng(seed)
    p = np.zeros((B, N, nc + 5), np.float32)
    p[..., :2] = rng.uniform(0, 640, (B, N, 2))
    p[..., 2:4] = rng.uniform(4, 200, (B, N, 2))
    p[..., 4] = rng.beta(0.4, 4, (B, N))
    p[..., 5:] = rng.beta(0.5, 3, (B, N, nc))
    return p


def _same(c, g, atol=1e-3):
    cc, gc = c.count.numpy(), g.count.cpu().numpy()
    np.testing.assert_array_equal(cc, gc)
    for b in range(len(cc)):
        k = int(cc[b])
        np.testing.assert_array_equal(c.cls[b, :k].numpy(), g.cls[b, :k].cpu().numpy())
        np.testing.assert_array_equal(c.score[b, :k].numpy(), g.score[b, :k].cpu().numpy())
        np.testing.assert_allclose(c.box[b, :k].numpy(), g.box[b, :k].cpu().numpy(), atol=atol, rtol=1e-6)


@pytest.mark.parametrize("kw", [dict(), dict(multi_label=True), dict(classes=[0, 2, 5, 63]), dict(agnostic=True)])
def test_filter_decoded_matches_cpu_postprocess(cuda, kw):
    from triton_client_amd.ops.image import frame_xform
    from triton_client_amd.ops.yolo import YoloPostprocess

    pred = _pred(3, 25200, 80)
    xf = frame_xform((720, 1280), (640, 640), "stretch")[0]
    anchors = np.zeros((3, 3, 2), np.float32)
    cpu = YoloPostprocess(80, anchors, conf_thres=0.3, device="cpu", **kw)
    gpu = YoloPostprocess(80, anchors, conf_thres=0.3, device=cuda, **kw)
    c = cpu.postprocess_decoded(pred, xf)
    g = gpu.filter_decoded(torch.from_numpy(pred).to(cuda), xf)
    assert int(c.count.sum()) > 30
    _same(c, g)
    # no xform: model-input pixels, the reference's extract_boxes output
    _same(cpu.postprocess_decoded(pred[:1]), gpu.filter_decoded(torch.from_numpy(pred[:1]).to(cuda)))


def test_yolov4_filter_decoded_matches_cpu(cuda):
    from triton_client_amd.ops.image import frame_xform
    from triton_client_amd.ops.yolov4 import Yolov4Postprocess

    rng = np.random.default_rng(1)
    B, N, nc = 2, 16128, 80
    x1 = rng.uniform(0, 0.9, (B, N, 1, 2)).astype(np.float32)
    boxes = np.concatenate([x1, x1 + rng.uniform(0.01, 0.3, (B, N, 1, 2)).astype(np.float32)], -1)
    confs = (rng.beta(0.3, 6, (B, N, nc)) * rng.beta(0.6, 2, (B, N, 1))).astype(np.float32)
    xf = frame_xform((720, 1280), (512, 512), "stretch")[0]
    cpu = Yolov4Postprocess(nc, (512, 512), 0.4, 0.6, device="cpu")
    gpu = Yolov4Postprocess(nc, (512, 512), 0.4, 0.6, device=cuda)
    c = cpu.decoded_cpu(boxes, confs, xf)
    g = gpu.filter_decoded(torch.from_numpy(boxes).to(cuda), torch.from_numpy(confs).to(cuda), xf)
    assert int(c.count.sum()) > 10
    # per-class NMS order differs (CPU: class-major, then score); compare as sets
    for b in range(B):
        k = int(c.count[b])
        assert k == int(g.count[b])
        rc = sorted(zip(c.cls[b, :k].tolist(), c.score[b, :k].tolist()))
        rg = sorted(zip(g.cls[b, :k].cpu().tolist(), g.score[b, :k].cpu().tolist()))
        assert rc == rg


def test_yolov5_client_extract_boxes_on_device(cuda):
    from triton_client_amd.clients import Yolov5postprocess

    pred = _pred(1, 25200, 80, seed=3)
    a = Yolov5postprocess("cpu").extract_boxes(pred, conf_thres=0.3)
    b = Yolov5postprocess(cuda).extract_boxes(pred, conf_thres=0.3)
    assert len(a[0]) > 5 and a[0].shape == b[0].shape
    np.testing.assert_array_equal(a[0][:, 4:], b[0][:, 4:])
    np.testing.assert_allclose(a[0][:, :4], b[0][:, :4], atol=1e-3)


@pytest.fixture(scope="module")
def served(cuda):
    from triton_client_amd.server import KServeServer, ModelRepository

    repo = ModelRepository("cuda")
    repo.load("YOLOv5nCOCO")
    repo.load("pointpillar_kitti")
    srv = KServeServer(repo, "127.0.0.1:0").start()
    yield srv
    srv.stop()


@pytest.fixture(scope="module")
def served_proc(cuda):
    """The same models in a server PROCESS: device shared memory maps the client's allocation by
    HIP IPC handle, which a process cannot open on its own allocation."""
    import os
    import socket
    import subprocess
    import sys

    from triton_client_amd.channel.grpc_channel import GRPCChannel

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srv = subprocess.Popen([sys.executable, "-m", "triton_client_amd.server", "--host", "127.0.0.1", "--port",
                            str(port), "--models", "YOLOv5nCOCO,pointpillar_kitti", "--device", "cuda",
                            "--metrics-port", "0"], cwd=root)

    class F:
        model_name, model_version, batch_size = "YOLOv5nCOCO", "", 1

    class S:
        target = f"127.0.0.1:{port}"
    try:
        GRPCChannel({"grpc_channel": S.target}, F(), wait_ready_s=240.0).close()
        yield S
    finally:
        srv.terminate()
        srv.wait(60)


def _run_main(mod, argv, topics):
    """Run an entry point on the in-process topic bus; -> {topic: [messages]}."""
    from triton_client_amd.ros import default_bus, reset_default_bus

    reset_default_bus()
    got = {t: [] for t in topics}
    for t in topics:
        default_bus().subscribe(t, got[t].append)
    assert mod.main(argv) == 0
    reset_default_bus()
    return got


def _dets_by_seq(msgs_):
    return {m.header.seq: np.asarray(m.detections.columns["dets"], np.float32) for m in msgs_}


@pytest.mark.parametrize("raw", [True, False], ids=["rgb8", "jpeg"])
def test_main_default_flags_remote_on_device(cuda, served, tmp_path, monkeypatch, raw):
    """``main.py -m YOLOv5nCOCO`` with default flags (remote engine, --device auto): the
    device path runs and publishes the CPU client's detections.  Raw frames: identical
    kept sets.  JPEG: the GPU IDCT differs from libjpeg (the CPU client's PIL decode) by
    <= 4 LSB in rare pixels (tests/test_jpeg_gpu.py), which the random-init detector
    amplifies, so the JPEG case is held to the detection-level tolerance (same class,
    IoU > 0.5, counts within 10%)."""
    from triton_client_amd.cli import main as main2d, record
    from triton_client_amd.inference import remote_live

    cam = str(tmp_path / "cam.bag")
    assert record.main([cam, "--frames", "6", "--cam", "720x1280"] + (["--raw"] if raw else [])) == 0
    params = tmp_path / "p.yaml"
    params.write_text(yaml.safe_dump({"grpc_channel": served.target, "sub_topic": "/camera/color/image_raw",
                                      "pub_topic": "/det", "gt_topic": "/gt"}))
    calls = []
    orig = remote_live.RemoteLiveCamera.run

    def counted(self, key, batch, draw, names):
        calls.append((key[0], len(batch)))
        return orig(self, key, batch, draw, names)

    monkeypatch.setattr(remote_live.RemoteLiveCamera, "run", counted)
    base = ["-m", "YOLOv5nCOCO", "--params", str(params), "--play", cam, "--spin-timeout", "120"]
    gpu = _run_main(main2d, base, ["/det", "/det/detections"])
    assert len(calls) == 6 and {k for k, _ in calls} == {"frames" if raw else "jpeg"}
    cpu = _run_main(main2d, base + ["--device", "cpu"], ["/det", "/det/detections"])
    assert len(calls) == 6  # the CPU client does not take the device path
    g, c = _dets_by_seq(gpu["/det/detections"]), _dets_by_seq(cpu["/det/detections"])
    assert sorted(g) == sorted(c) and len(g) == 6
    assert all(m.width == 1280 and m.height == 720 for m in gpu["/det"])
    total = sum(len(v) for v in c.values())
    assert total > 6
    if raw:
        for s in c:
            assert g[s].shape == c[s].shape, s
            np.testing.assert_array_equal(g[s][:, 5], c[s][:, 5])
            np.testing.assert_allclose(g[s][:, 4], c[s][:, 4], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(g[s][:, :4], c[s][:, :4], atol=0.05)
    else:
        from triton_client_amd.ops.golden import box_iou_np
        ok = 0
        for s in c:
            a, b = g[s], c[s]
            if len(a) and len(b):
                iou = box_iou_np(a[:, :4], b[:, :4]) * (a[:, 5:6] == b[None, :, 5])
                ok += int((iou.max(1) > 0.5).sum())
        ng = sum(len(v) for v in g.values())
        assert abs(ng - total) <= max(2, total // 10) and ok >= 0.85 * ng, (ok, ng, total)


@pytest.mark.parametrize("wire", ["devshm", "shm"])
def test_main_shared_memory_wire_on_device(cuda, served, served_proc, tmp_path, monkeypatch, wire):
    """``main.py -m YOLOv5nCOCO --wire devshm|shm``: the device path runs on the shared-memory
    wires (K1 writes the model input into the registered region, the server writes the output
    back there; devshm: a GPU allocation shared by HIP IPC handle, K3/K4 read the output in
    place) and publishes the CPU client's detections."""
    from triton_client_amd.cli import main as main2d, record
    from triton_client_amd.inference import remote_live

    cam = str(tmp_path / "cam.bag")
    assert record.main([cam, "--frames", "6", "--cam", "720x1280", "--raw"]) == 0
    params = tmp_path / "p.yaml"
    srv = served_proc if wire == "devshm" else served
    params.write_text(yaml.safe_dump({"grpc_channel": srv.target, "sub_topic": "/camera/color/image_raw",
                                      "pub_topic": "/det", "gt_topic": "/gt"}))
    calls = []
    orig = remote_live.RemoteLiveCamera._rpc_shm

    def counted(self, x, n):
        calls.append((self.det.wire, n))
        return orig(self, x, n)

    monkeypatch.setattr(remote_live.RemoteLiveCamera, "_rpc_shm", counted)
    errs = []
    orig_run = remote_live.RemoteLiveCamera.run

    def run(self, *a, **k):  # the bus thread swallows callback errors: keep them for the assert
        try:
            return orig_run(self, *a, **k)
        except BaseException as e:
            errs.append(e)
            raise
    monkeypatch.setattr(remote_live.RemoteLiveCamera, "run", run)
    base = ["-m", "YOLOv5nCOCO", "--params", str(params), "--play", cam, "--spin-timeout", "120"]
    gpu = _run_main(main2d, base + ["--wire", wire], ["/det", "/det/detections"])
    if errs:
        raise errs[0]
    assert len(calls) == 6 and {w for w, _ in calls} == {wire}
    cpu = _run_main(main2d, base + ["--device", "cpu"], ["/det", "/det/detections"])
    g, c = _dets_by_seq(gpu["/det/detections"]), _dets_by_seq(cpu["/det/detections"])
    assert sorted(g) == sorted(c) and len(g) == 6
    assert sum(len(v) for v in c.values()) > 6
    for s in c:
        assert g[s].shape == c[s].shape, s
        np.testing.assert_array_equal(g[s][:, 5], c[s][:, 5])
        np.testing.assert_allclose(g[s][:, 4], c[s][:, 4], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g[s][:, :4], c[s][:, :4], atol=0.05)


@pytest.mark.parametrize("wire", ["raw", "devshm"])
def test_main3d_default_flags_remote_on_device(cuda, served, served_proc, tmp_path, monkeypatch, wire):
    """``main3d.py -m pointpillar_kitti`` with default flags: the client unpacks and
    voxelises on the GPU (K6 + K7) and publishes the CPU client's boxes."""
    from triton_client_amd.cli import main3d, record
    from triton_client_amd.clients.detector_3d_client import PointpillarPreprocess

    pc = str(tmp_path / "pc.bag")
    assert record.main([pc, "--frames", "3", "--no-camera", "--lidar"]) == 0
    params = tmp_path / "p3.yaml"
    params.write_text(yaml.safe_dump({"grpc_channel": (served_proc if wire == "devshm" else served).target,
                                      "sub_topic": "/ai_test_field/sensors/os_cloud_node/points",
                                      "pub_topic": "/det3d", "gt_topic": "/gt"}))
    calls = []
    orig = PointpillarPreprocess.filter_cloud_gpu

    def counted(self, *a, **k):
        calls.append(self.device.type)
        return orig(self, *a, **k)

    monkeypatch.setattr(PointpillarPreprocess, "filter_cloud_gpu", counted)
    base = ["-m", "pointpillar_kitti", "--params", str(params), "--play", pc, "--spin-timeout", "120",
            "--labels", "all", "--score-thresh", "0"]
    gpu = _run_main(main3d, base + ["--wire", wire], ["/det3d"])
    assert calls == ["cuda"] * 3
    cpu = _run_main(main3d, base + ["--device", "cpu"], ["/det3d"])
    assert len(calls) == 3
    g = {m.header.seq: m for m in gpu["/det3d"]}
    c = {m.header.seq: m for m in cpu["/det3d"]}
    assert sorted(g) == sorted(c) and len(g) == 3
    # the random-init head scores many boxes alike, so the two clients' float-level differences
    # (GPU vs NumPy unpack: i / max(i) rounding) can reorder equal-looking scores: compare as sets
    for s in c:
        gb = [(b.label, b.pose.position.x, b.pose.position.y, b.pose.position.z, b.value) for b in g[s].boxes]
        cb = [(b.label, b.pose.position.x, b.pose.position.y, b.pose.position.z, b.value) for b in c[s].boxes]
        assert len(cb) > 0 and abs(len(gb) - len(cb)) <= max(1, len(cb) // 50), (len(gb), len(cb))
        cb_arr = np.asarray(cb, np.float64)
        hit = 0
        for lab, x, y, z, v in gb:
            d = np.abs(cb_arr[:, 1:4] - [x, y, z]).max(1)
            hit += int(((cb_arr[:, 0] == lab) & (d < 1e-3) & (np.abs(cb_arr[:, 4] - v) < 1e-4)).any())
        assert hit >= 0.98 * len(gb), (hit, len(gb))
