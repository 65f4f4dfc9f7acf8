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


def test_gpu_server_models_over_kserve(cuda):
    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Pointpillars_client, Yolov5client
    from triton_client_amd.inference import RemoteDetector2D, RemoteDetector3D
    from triton_client_amd.server import KServeServer, ModelRepository

    repo = ModelRepository("cuda")
    repo.load("YOLOv5nCOCO")
    repo.load("pointpillar_kitti")
    with KServeServer(repo, "127.0.0.1:0") as srv:
        class F:
            model_version, batch_size = "", 1

        f2, f3 = F(), F()
        f2.model_name, f3.model_name = "YOLOv5nCOCO", "pointpillar_kitti"
        p = {"grpc_channel": srv.target}
        ch2, ch3 = GRPCChannel(p, f2), GRPCChannel(p, f3)
        d2 = RemoteDetector2D(ch2, Yolov5client(), device=cuda).detect([camera_frame(480, 640, 1)])
        assert len(d2) == 1 and d2[0].shape[1] == 6 and len(d2[0]) > 0
        d3 = RemoteDetector3D(ch3, Pointpillars_client()).detect([_cloud(4, 64, 1875)])
        assert len(d3[0]["pred_scores"]) > 0
        st = ch3.model_statistics("pointpillar_kitti")
        assert st.model_stats[0].inference_count >= 1
        ch2.close()
        ch3.close()
