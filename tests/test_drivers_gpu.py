"""Local MI355X engines and GPU-served models behind the KServe server."""
import numpy as np
import pytest
import torch

from triton_client_amd.ros import compat, msgs
from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

pytestmark = pytest.mark.gpu


def _cloud(seed, rings=32, cols=1024):
    pts = lidar_sweep(LidarSpec(rings=rings, azimuth_steps=cols, sensor_height=3.23), seed)
    return compat.create_cloud_xyzi(np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4), msgs.Header(seq=seed))


def test_local_2d_engine_gpu_batches_and_is_deterministic(cuda):
    from triton_client_amd.inference import LocalDetector2D

    eng = LocalDetector2D(batch=4, device=cuda, letterbox=True)
    frames = [camera_frame(360, 640, s) for s in range(6)] + [camera_frame(240, 320, 9)]
    a = eng.detect(frames)
    b = eng.detect(frames[::-1])[::-1]
    assert len(a) == 7 and sum(len(x) for x in a) > 0
    for x, y in zip(a, b):  # micro-batch position must not matter
        np.testing.assert_array_equal(x, y)
    for x, f in zip(a, frames):
        if len(x):
            assert x[:, [0, 2]].max() <= f.shape[1] + 1e-3 and x[:, [1, 3]].max() <= f.shape[0] + 1e-3
    assert len(eng._pipes) == 2  # one captured pipeline per source geometry


def test_local_3d_engine_gpu(cuda):
    from triton_client_amd.inference import LocalDetector3D

    eng = LocalDetector3D(batch=2, device=cuda, calibrate_target=500.0)
    clouds = [_cloud(s) for s in range(3)]
    a = eng.detect(clouds)
    b = eng.detect(clouds)
    assert len(a) == 3 and all(len(p["pred_scores"]) > 0 for p in a)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x["pred_boxes"], y["pred_boxes"])
    for p in a:
        assert np.isfinite(p["pred_boxes"]).all() and set(np.unique(p["pred_labels"])) <= {1, 2, 3}
        assert (p["pred_scores"] >= 0.1 - 1e-6).all()


@pytest.mark.parametrize("family,labels,dim", [("second_iou", {1, 2, 3}, 7), ("centerpoint", set(range(10)), 9)])
def test_local_3d_engine_families_gpu(cuda, family, labels, dim):
    """main3d.py -m second_iou / centerpoint_pp --engine local: the family's
    graph-captured pipeline behind the same Detector3D interface."""
    from triton_client_amd.inference import LocalDetector3D

    eng = LocalDetector3D(batch=2, device=cuda, family=family)
    clouds = [_cloud(s, 64, 1875) for s in range(3)]
    a = eng.detect(clouds)
    b = eng.detect(clouds[::-1])[::-1]
    assert len(a) == 3 and all(len(p["pred_scores"]) > 0 for p in a)
    for x, y in zip(a, b):  # micro-batch position must not matter
        np.testing.assert_array_equal(x["pred_boxes"], y["pred_boxes"])
    for p in a:
        assert p["pred_boxes"].shape[1] == dim and np.isfinite(p["pred_boxes"]).all()
        assert set(np.unique(p["pred_labels"])) <= labels


def test_served_path_matches_local_engines(cuda):
    """The zero-copy served path (client GPU preprocess / voxelise -> pinned
    staging -> C++ encoder -> KServe -> GPU model -> C++ encoder) keeps the
    same detections as the local engines running the same weights."""
    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov5client, client_for_model
    from triton_client_amd.inference import LocalDetector2D, LocalDetector3D, RemoteDetector2D, RemoteDetector3D
    from triton_client_amd.ops.golden import box_iou_np
    from triton_client_amd.server import KServeServer, ModelRepository

    repo = ModelRepository("cuda")
    repo.load("YOLOv5nCOCO")
    repo.load("pointpillar_kitti")
    s2, s3 = repo.get("YOLOv5nCOCO"), repo.get("pointpillar_kitti")
    frames = [camera_frame(480, 640, s) for s in (1, 2, 3)]
    clouds = [_cloud(s, 64, 1875) for s in (4, 5)]
    with KServeServer(repo, "127.0.0.1:0") as srv:
        class F:
            model_version, batch_size = "", 1

        f2, f3 = F(), F()
        f2.model_name, f3.model_name = "YOLOv5nCOCO", "pointpillar_kitti"
        p = {"grpc_channel": srv.target}
        ch2, ch3 = GRPCChannel(p, f2), GRPCChannel(p, f3)
        r2 = RemoteDetector2D(ch2, Yolov5client(), device=cuda, mode="async").detect(frames)
        cfg3 = ch3.get_metadata()["config_response"]
        rem3 = RemoteDetector3D(ch3, client_for_model("pointpillar_kitti", getattr(cfg3, "config", cfg3)), device=cuda)
        r3 = rem3.detect(clouds)
        st = ch3.model_statistics("pointpillar_kitti")
        assert st.model_stats[0].inference_count >= 2
        ch2.close()
        ch3.close()
    loc2 = LocalDetector2D(batch=1, device=cuda, letterbox=False, calibrate_target=None)
    loc2.model = s2.model  # the served weights (calibrated head prior included)
    l2 = loc2.detect(frames)
    ok = tot_r = tot_l = 0
    for a, b in zip(r2, l2):
        tot_r, tot_l = tot_r + len(a), tot_l + len(b)
        if len(a) and len(b):
            iou = box_iou_np(a[:, :4], b[:, :4]) * (a[:, 5:6] == b[None, :, 5])
            ok += int((iou.max(1) > 0.95).sum())
    assert tot_r > 10 and ok >= 0.95 * tot_r and abs(tot_r - tot_l) <= max(2, tot_r // 30), (ok, tot_r, tot_l)
    loc3 = LocalDetector3D(batch=1, device=cuda, calibrate_target=None)
    loc3.model, loc3.cfg = s3.model, s3.cfg
    l3 = loc3.detect(clouds)
    for a, b in zip(r3, l3):
        na, nb = len(a["pred_scores"]), len(b["pred_scores"])
        assert na > 0 and abs(na - nb) <= max(2, na // 50), (na, nb)
        np.testing.assert_allclose(np.sort(a["pred_scores"])[-20:], np.sort(b["pred_scores"])[-20:], rtol=1e-4,
                                   atol=1e-5)


def test_served_dynamic_batch_matches_single_requests(cuda):
    """Server-side dynamic batching: a batch of requests through the models'
    batch plans returns what each request gets alone."""
    from triton_client_amd.ops.golden import preprocess_image
    from triton_client_amd.ops.lidar import voxelize_np
    from triton_client_amd.server import ModelRepository

    repo = ModelRepository("cuda")
    s2, s3 = repo.load("YOLOv5nCOCO"), repo.load("pointpillar_kitti")
    assert s2.dynamic_batch > 1 and s3.dynamic_batch > 1
    imgs = [preprocess_image(camera_frame(480, 640, s), (640, 640), "stretch", layout="NCHW")[None] for s in range(3)]
    single = [s2.execute({"images": x}, ["output"])["output"].clone() for x in imgs]
    batch = s2.execute_batch([{"images": x} for x in imgs], ["output"])
    for a, b in zip(single, batch):
        d = (a - b["output"]).abs().max().item()
        assert d <= 1e-3 * max(1.0, a.abs().max().item()), d
    reqs = []
    for s in (4, 5, 6):
        pts = lidar_sweep(LidarSpec(rings=64, azimuth_steps=1875, sensor_height=3.23), s)
        pts = np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4)
        vox, co, n = voxelize_np(pts, s3.cfg.voxel)[:3]
        co4 = np.concatenate([np.zeros((len(co), 1), np.int32), co.astype(np.int32)], 1)
        reqs.append({"voxels": vox.astype(np.float32), "voxel_coords": co4, "voxel_num_points": n.astype(np.int32)})
    single3 = [{k: v.copy() for k, v in s3.execute(r, []).items()} for r in reqs]
    batch3 = s3.execute_batch(reqs, [])
    for a, b in zip(single3, batch3):
        na, nb = len(a["pred_scores"]), len(b["pred_scores"])
        assert na > 0 and abs(na - nb) <= max(2, na // 50), (na, nb)
        np.testing.assert_allclose(np.sort(a["pred_scores"])[-20:], np.sort(b["pred_scores"])[-20:], rtol=1e-4,
                                   atol=1e-5)
    # the device range check inside the plan (tca_voxel_check): a request with a cell outside
    # the grid (reaching execute_batch unvalidated) gets its error, its neighbours their boxes
    bad = {k: v.copy() for k, v in reqs[1].items()}
    bad["voxel_coords"][7, 3] = int(s3.cfg.voxel.grid_size[0]) + 5
    mixed = s3.execute_batch([reqs[0], bad, reqs[2]], [])
    from triton_client_amd.server.model import InferError
    assert isinstance(mixed[1], InferError) and not isinstance(mixed[0], Exception)
    for a, b in ((single3[0], mixed[0]), (single3[2], mixed[2])):
        assert abs(len(a["pred_scores"]) - len(b["pred_scores"])) <= max(2, len(a["pred_scores"]) // 50)
    with pytest.raises(InferError):
        s3.execute(bad, [])


def test_served_shared_memory_matches_raw_wire(cuda):
    """KServe system shared memory (inputs and the 2D output in the client's
    pinned region, messages carrying only references) returns the raw-wire
    path's detections."""
    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov5client, client_for_model
    from triton_client_amd.inference import RemoteDetector2D, RemoteDetector3D
    from triton_client_amd.server import KServeServer, ModelRepository

    repo = ModelRepository("cuda")
    repo.load("YOLOv5nCOCO")
    repo.load("pointpillar_kitti")
    frames = [camera_frame(480, 640, s) for s in (1, 2, 3, 4, 5)]
    clouds = [_cloud(s, 64, 1875) for s in (4, 5, 6)]
    with KServeServer(repo, "127.0.0.1:0") as srv:
        class F:
            model_version, batch_size = "", 1

        f2, f3 = F(), F()
        f2.model_name, f3.model_name = "YOLOv5nCOCO", "pointpillar_kitti"
        p = {"grpc_channel": srv.target}
        ch2, ch3 = GRPCChannel(p, f2), GRPCChannel(p, f3)
        cfg3 = ch3.get_metadata()["config_response"]
        out = {}
        for wire in ("raw", "shm"):
            d2 = RemoteDetector2D(ch2, Yolov5client(), device=cuda, mode="async", wire=wire)
            d3 = RemoteDetector3D(ch3, client_for_model("pointpillar_kitti", getattr(cfg3, "config", cfg3)),
                                  device=cuda, mode="async", wire=wire)
            d2.window = d3.window = 2  # slots are reused within the call
            out[wire] = (d2.detect(frames), d3.detect(clouds))
            if wire == "shm":
                assert len(ch2.system_shared_memory_status().regions) == 2
                d2.close_shm()
                d3.close_shm()
        assert len(ch2.system_shared_memory_status().regions) == 0
        ch2.close()
        ch3.close()
    for a, b in zip(out["raw"][0], out["shm"][0]):
        np.testing.assert_array_equal(a, b)
    assert sum(len(a) for a in out["raw"][0]) > 10
    for a, b in zip(out["raw"][1], out["shm"][1]):
        assert len(a["pred_scores"]) > 0
        np.testing.assert_array_equal(a["pred_boxes"], b["pred_boxes"])


def test_served_device_shared_memory_matches_raw_wire(cuda):
    """Device shared memory (HIP IPC handles registered with a server in another process:
    the camera input and 2D output, and the voxel tensors, stay in GPU buffers; only
    region references cross gRPC) returns the raw-wire path's detections."""
    import os
    import socket
    import subprocess
    import sys

    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov5client, client_for_model
    from triton_client_amd.inference import RemoteDetector2D, RemoteDetector3D

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srv = subprocess.Popen([sys.executable, "-m", "triton_client_amd.server", "--host", "127.0.0.1", "--port",
                            str(port), "--models", "YOLOv5nCOCO,pointpillar_kitti", "--device", "cuda",
                            "--metrics-port", "0"], cwd=root)
    try:
        frames = [camera_frame(480, 640, s) for s in (1, 2, 3, 4, 5)]
        clouds = [_cloud(s, 64, 1875) for s in (4, 5, 6)]

        class F:
            model_version, batch_size = "", 1

        f2, f3 = F(), F()
        f2.model_name, f3.model_name = "YOLOv5nCOCO", "pointpillar_kitti"
        p = {"grpc_channel": f"127.0.0.1:{port}"}
        ch2, ch3 = GRPCChannel(p, f2, wait_ready_s=240.0), GRPCChannel(p, f3, wait_ready_s=240.0)
        cfg3 = ch3.get_metadata()["config_response"]
        out = {}
        for wire in ("raw", "devshm"):
            d2 = RemoteDetector2D(ch2, Yolov5client(), device=cuda, mode="async", wire=wire)
            d3 = RemoteDetector3D(ch3, client_for_model("pointpillar_kitti", getattr(cfg3, "config", cfg3)),
                                  device=cuda, mode="async", wire=wire)
            d2.window = d3.window = 2  # slots are reused within the call
            out[wire] = (d2.detect(frames), d3.detect(clouds))
            if wire == "devshm":
                assert len(ch2.cuda_shared_memory_status().regions) == 2
                assert len(ch2.system_shared_memory_status().regions) == 0
                d2.close_shm()
                d3.close_shm()
        assert len(ch2.cuda_shared_memory_status().regions) == 0
        # a registration claiming more bytes than the handle maps, or another GPU, is refused
        import grpc
        from triton_client_amd.utils.hip_ipc import DeviceAllocation
        alloc = DeviceAllocation(1 << 20, cuda)
        for nbytes, dev in ((4 << 20, alloc.device_id), (1 << 20, alloc.device_id + 1)):
            with pytest.raises(grpc.RpcError):
                ch2.register_cuda_shared_memory("bad", alloc.handle, dev, nbytes)
        ch2.register_cuda_shared_memory("ok", alloc.handle, alloc.device_id, 1 << 20)
        assert len(ch2.cuda_shared_memory_status().regions) == 1
        ch2.unregister_cuda_shared_memory("ok")
        ch2.close()
        ch3.close()
        alloc.close()
    finally:
        srv.terminate()
        srv.wait(60)
    for a, b in zip(out["raw"][0], out["devshm"][0]):
        np.testing.assert_array_equal(a, b)
    assert sum(len(a) for a in out["raw"][0]) > 10
    for a, b in zip(out["raw"][1], out["devshm"][1]):
        assert len(a["pred_scores"]) > 0
        np.testing.assert_array_equal(a["pred_boxes"], b["pred_boxes"])
