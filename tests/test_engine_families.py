"""Local-engine family selection (cli/engines.py camera_spec / lidar_family) and
the device-side packing of CenterPoint's per-task NMS segments for the
data-parallel gather (inference/engines.py pack_task_segments), on the CPU."""
import numpy as np
import pytest
import torch

from triton_client_amd.cli.engines import camera_spec, lidar_family
from triton_client_amd.inference.engines import pack_task_segments
from triton_client_amd.ops.centerpoint import DET3D_ORDER, CenterPointResult
from triton_client_amd.ops.yolo import NmsResult


@pytest.mark.parametrize("name,family,img", [
    ("YOLOv5n", "yolov5", (640, 640)), ("YOLOv5nCOCO", "yolov5", (640, 640)), ("YOLOv5nCROP", "yolov5", (512, 512)),
    ("weed_detector", "yolov5", (512, 512)), ("YOLOv4", "yolov4", (512, 512)), ("test_model", "retinanet", (640, 480)),
    ("RetinaNet_detectron", "retinanet", (800, 1344)), ("FCOS_detectron", "fcos", (800, 1344)),
    ("fcos_weed_detector", "fcos", (800, 1344))])
def test_camera_spec_families(name, family, img):
    fam, _, nc, hw, names = camera_spec(name, 80)
    assert (fam, hw) == (family, img)
    assert nc == (2 if ("weed" in name.lower() or "crop" in name.lower()) else 80)


def test_camera_spec_unknown_name_raises():
    with pytest.raises(ValueError, match="no local camera engine"):
        camera_spec("pointpillar_kitti", 80)


def test_lidar_family_names():
    assert lidar_family("second_iou") == "second_iou"
    assert lidar_family("centerpoint_pp") == "centerpoint"
    assert lidar_family("pointpillar_kitti") == "pointpillars"


def test_pack_task_segments_matches_per_image():
    """Fixed-size device rows == CenterPointResult.per_image (task order, det3d box
    order), including a frame whose segments overflow max_out."""
    rng = np.random.default_rng(0)
    B, T, mo = 3, 6, 83
    counts = rng.integers(0, mo + 1, size=(B, T)).astype(np.int32)
    counts[2] = mo  # 6 x 83 = 498 rows: truncated at max_out = 400 below
    box = torch.from_numpy(rng.standard_normal((B * T, mo, 9)).astype(np.float32))
    score = torch.from_numpy(rng.random((B * T, mo)).astype(np.float32))
    cls = torch.from_numpy(rng.integers(0, 10, (B * T, mo)).astype(np.int32))
    res = CenterPointResult(NmsResult(box, score, cls, torch.from_numpy(counts.reshape(-1))), B, T)
    want = res.per_image()
    for max_out in (500, 400):
        b, s, lab, c = pack_task_segments(res, B, max_out)
        assert b.shape == (B, max_out, 9) and s.shape == (B, max_out) and lab.dtype == torch.int64
        for i in range(B):
            k = min(int(counts[i].sum()), max_out)
            assert int(c[i]) == k
            np.testing.assert_array_equal(b[i, :k].numpy(), want[i]["pred_boxes"][:k])
            np.testing.assert_array_equal(s[i, :k].numpy(), want[i]["pred_scores"][:k])
            np.testing.assert_array_equal(lab[i, :k].numpy(), want[i]["pred_labels"][:k])
            assert (s[i, k:] == 0).all()
    assert list(DET3D_ORDER) == [0, 1, 2, 3, 4, 5, 7, 8, 6]


def test_export_weights_reproduces_calibrated_engine(tmp_path):
    """export_weights (fused, calibrated) -> --weights: the reloaded engines give the
    same detections bit for bit, with no re-calibration (camera and LiDAR)."""
    from triton_client_amd.inference.engines import LocalDetector2D, LocalDetector3D, export_weights
    from triton_client_amd.ros.compat import create_cloud_xyzi
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    frames = [camera_frame(120, 160, 3 + i) for i in range(2)]
    a = LocalDetector2D(img=128, batch=2, device="cpu", graph=False)
    want = a.detect(frames)
    export_weights(a.model, str(tmp_path / "cam.pt"))
    b = LocalDetector2D(img=128, batch=2, device="cpu", graph=False, weights=str(tmp_path / "cam.pt"))
    assert b.calibrate_target is None
    got = b.detect(frames)
    assert sum(len(d) for d in want) > 0
    for x, y in zip(want, got):
        np.testing.assert_array_equal(x, y)

    spec = LidarSpec(rings=16, azimuth_steps=512, sensor_height=3.23)
    clouds = [create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, 40).tobytes(), np.float32).reshape(-1, 4))]
    a3 = LocalDetector3D(batch=1, device="cpu", graph=False, max_points=16384)
    want3 = a3.detect(clouds)
    export_weights(a3.model, str(tmp_path / "pc.pt"))
    b3 = LocalDetector3D(batch=1, device="cpu", graph=False, max_points=16384, weights=str(tmp_path / "pc.pt"))
    got3 = b3.detect(clouds)
    for x, y in zip(want3, got3):
        assert x.keys() == y.keys()
        for k in x:
            np.testing.assert_array_equal(np.asarray(x[k]), np.asarray(y[k]))
