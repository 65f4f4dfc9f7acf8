"""Inference drivers end to end on the CPU.

Covers ROS topic bus → engine → published messages, bag replay, and the
evaluator.  Remote engines go over real gRPC to the in-process KServe server
on 127.0.0.1 (CPU models).  Local engines use the CPU path of the same
pipelines.  This mirrors the reference's only integration path, bag replay
(SURVEY §4), with synthetic data.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

from triton_client_amd.channel.grpc_channel import GRPCChannel
from triton_client_amd.clients import FCOS_client, Pointpillars_client, Yolov5client
from triton_client_amd.config.lidar import KITTI_PILLARS, PointPillarsConfig
from triton_client_amd.inference import (BagInference2D, BagInference3D, Detector2D, EvaluateInference,
                                         LocalDetector2D, LocalDetector3D, RemoteDetector2D, RemoteDetector3D,
                                         RosInference, RosInference3D, boxes_to_detection3d, detections_to_msg)
from triton_client_amd.ros import Bag, TopicBus, compat, msgs
from triton_client_amd.server import KServeServer, ModelRepository
from triton_client_amd.server.models import PointPillarsModel, YoloV5Model
from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

torch.set_num_threads(4)

SMALL_PP = PointPillarsConfig(
    voxel=dataclasses.replace(KITTI_PILLARS, point_cloud_range=(0.0, -19.84, -3.0, 34.56, 19.84, 1.0),
                              max_voxels=8000),
    score_thresh=0.005, nms_pre_max=48, nms_post_max=12)


class Flags:
    def __init__(self, model_name):
        self.model_name, self.model_version, self.batch_size = model_name, "", 1


@pytest.fixture(scope="module")
def server():
    repo = ModelRepository("cpu")
    repo.add(YoloV5Model("YOLOv5n", img=128, device="cpu"))
    repo.add(PointPillarsModel("pointpillar_kitti", cfg=SMALL_PP, device="cpu"))
    srv = KServeServer(repo, "127.0.0.1:0").start()
    yield srv
    srv.stop()


def _params(srv, **kw):
    p = {"grpc_channel": srv.target, "sub_topic": "/cam", "pub_topic": "/det", "gt_topic": "/gt"}
    p.update(kw)
    return p


def _jpeg_msg(seq, h=96, w=160):
    img = camera_frame(h, w, seq)
    return msgs.CompressedImage(header=msgs.Header(seq=seq, frame_id="cam"), format="jpeg",
                                data=compat.jpeg_encode(img)), img


def _cloud(seed=0, rings=16, cols=256):
    pts = lidar_sweep(LidarSpec(rings=rings, azimuth_steps=cols, sensor_height=3.23), seed)
    raw = np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4)
    return compat.create_cloud_xyzi(raw, msgs.Header(seq=seed, frame_id="lidar"))


# ------------------------------------------------------------------------------- 2D
def test_remote_2d_modes_agree(server):
    ch = GRPCChannel(_params(server), Flags("YOLOv5n"))
    frames = [camera_frame(96, 160, s) for s in range(3)]
    ref = RemoteDetector2D(ch, Yolov5client(), conf_thres=0.01).detect(frames)
    for mode, wire in (("sync", "proto"), ("async", "raw"), ("stream", "raw")):
        got = RemoteDetector2D(ch, Yolov5client(), conf_thres=0.01, mode=mode, wire=wire).detect(frames)
        for a, b in zip(ref, got):
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-4)
    for d in ref:  # boxes are in original-frame pixels
        assert d.shape[1] == 6
        if len(d):
            assert d[:, [0, 2]].max() <= 160 + 1e-3 and d[:, [1, 3]].max() <= 96 + 1e-3
    ch.close()


def test_ros_inference_publishes_annotated_frames(server):
    bus = TopicBus()
    ch = GRPCChannel(_params(server), Flags("YOLOv5n"))
    drv = RosInference(ch, Yolov5client(), bus=bus, conf_thres=0.01, queue_size=None)
    got, dets = [], []
    bus.subscribe("/det", got.append)
    bus.subscribe("/det/detections", dets.append)
    drv.start_inference(spin=False)
    sent = []
    for s in range(3):
        m, img = _jpeg_msg(s)
        sent.append(m)
        bus.publish("/cam", m)
    bus.publish("/cam", compat.numpy_to_imgmsg(camera_frame(96, 160, 7), header=msgs.Header(seq=7)))  # raw Image
    assert bus.wait_idle(60)
    drv.stop()
    bus.close()
    assert [m.header.seq for m in got] == [0, 1, 2, 7]  # input header copied (A4)
    assert all(m.width == 160 and m.height == 96 and m.encoding == "rgb8" for m in got)
    assert len(dets) == 4 and isinstance(dets[0], msgs.Detection2DArray)
    ch.close()


def test_fcos_client_decodes_server_detections():
    """FCOS/RetinaNet servers return final boxes/classes/scores (no client NMS)."""
    from triton_client_amd.proto import service_pb2 as pb

    r = pb.ModelInferResponse(model_name="fcos")
    arrs = [("boxes", "FP32", np.array([[1, 2, 30, 40], [5, 5, 9, 9]], np.float32)),
            ("classes", "INT64", np.array([3, 7], np.int64)),
            ("scores", "FP32", np.array([0.9, 0.2], np.float32)),
            ("image_dims", "INT64", np.array([480, 640], np.int64))]
    for n, dt, a in arrs:
        t = r.outputs.add(name=n, datatype=dt)
        t.shape.extend(a.shape)
        r.raw_output_contents.append(a.tobytes())
    d = FCOS_client().get_postprocess().extract_boxes(r, conf_thres=0.5)[0]
    np.testing.assert_allclose(d, [[1, 2, 30, 40, 0.9, 3]])


def test_local_2d_cpu_engine_matches_module():
    eng = LocalDetector2D(img=128, batch=2, device="cpu", calibrate_target=20.0, letterbox=True, conf_thres=0.3)
    frames = [camera_frame(96, 160, s) for s in range(3)]
    out = eng.detect(frames)
    assert len(out) == 3 and all(o.shape[1] == 6 for o in out)
    assert sum(len(o) for o in out) > 0  # calibrated head prior yields detections
    again = eng.detect(frames[1:2])
    np.testing.assert_allclose(again[0], out[1], rtol=1e-5, atol=1e-4)


def test_bag_inference_2d(tmp_path, server):
    bag = str(tmp_path / "cam.bag")
    with Bag(bag, "w") as b:
        for s in range(5):
            b.write("/cam", _jpeg_msg(s)[0])
            b.write("/other", msgs.Header(seq=s))
    ch = GRPCChannel(_params(server), Flags("YOLOv5n"))
    out_dir, out_bag = str(tmp_path / "png"), str(tmp_path / "out.bag")
    drv = BagInference2D(ch, Yolov5client(), bagfile=bag, out_dir=out_dir, out_bag=out_bag, batch=2,
                         conf_thres=0.01)
    assert drv.start_inference() == 5
    assert sorted(os.listdir(out_dir)) == [f"{i:04}.png" for i in range(5)]
    with Bag(out_bag) as b:
        topics = [t for t, _, _ in b.read_messages()]
    assert topics.count("/cam") == 5 and topics.count("/det") == 5 and topics.count("/det/detections") == 5
    # resume from the 3rd frame
    drv2 = BagInference2D(ch, Yolov5client(), bagfile=bag, out_dir=None, batch=2, start_seq=3, save_png=False)
    assert drv2.start_inference() == 2 and [s for s, _ in drv2.results] == [3, 4]
    ch.close()


# ------------------------------------------------------------------------------- 3D
def test_remote_and_local_3d_agree(server):
    ch = GRPCChannel(_params(server, sub_topic="/pc"), Flags("pointpillar_kitti"))
    remote = RemoteDetector3D(ch, Pointpillars_client())
    assert remote.pre.cfg == SMALL_PP.voxel  # voxel geometry from the served model's config (A9)
    local = LocalDetector3D(cfg=SMALL_PP, device="cpu", calibrate_target=None)
    cloud = _cloud(1)
    r, l_ = remote.detect([cloud])[0], local.detect([cloud])[0]
    assert len(r["pred_boxes"]) == SMALL_PP.nms_post_max
    assert len(l_["pred_boxes"]) == len(r["pred_boxes"])
    np.testing.assert_allclose(np.sort(r["pred_scores"]), np.sort(l_["pred_scores"]), rtol=1e-4, atol=1e-5)
    ch.close()


def test_ros_inference3d_and_bag(tmp_path, server):
    ch = GRPCChannel(_params(server, sub_topic="/pc", pub_topic="/boxes"), Flags("pointpillar_kitti"))
    bus = TopicBus()
    drv = RosInference3D(ch, Pointpillars_client(), bus=bus, labels=None, score_thresh=0.0)
    got = []
    bus.subscribe("/boxes", got.append)
    drv.start_inference(spin=False)
    bus.publish("/pc", _cloud(2))
    assert bus.wait_idle(120)
    drv.stop()
    bus.close()
    assert len(got) == 1 and isinstance(got[0], msgs.BoundingBoxArray) and got[0].header.seq == 2
    assert len(got[0].boxes) == SMALL_PP.nms_post_max
    # default reference filter (Pedestrian, score > 0.5) on random weights publishes nothing
    assert len(RosInference3D(ch, Pointpillars_client()).process([_cloud(2)])[0][0].boxes) == 0

    bag = str(tmp_path / "pc.bag")
    with Bag(bag, "w") as b:
        for s in range(3):
            b.write("/pc", _cloud(s))
    drv = BagInference3D(ch, Pointpillars_client(), bagfile=bag, batch=2, labels=None, score_thresh=0.0)
    assert drv.start_inference() == 3
    with Bag(str(tmp_path / "pc_output.bag")) as b:
        msgs_out = list(b.read_messages())
    assert [t for t, _, _ in msgs_out] == ["/pc", "/boxes"] * 3
    assert isinstance(msgs_out[1][1], msgs.BoundingBoxArray)
    ch.close()


def test_detection3d_yaw_index_follows_box_dim():
    pred7 = {"pred_boxes": np.array([[1, 2, 3, 4, 5, 6, 0.5]], np.float32), "pred_scores": np.array([0.9]),
             "pred_labels": np.array([2])}
    pred9 = {"pred_boxes": np.array([[1, 2, 3, 4, 5, 6, 0.1, 0.2, 1.0]], np.float32),
             "pred_scores": np.array([0.9]), "pred_labels": np.array([2])}
    q7 = boxes_to_detection3d(pred7, [0], msgs.Header()).detections[0].bbox.center.orientation
    q9 = boxes_to_detection3d(pred9, [0], msgs.Header()).detections[0].bbox.center.orientation
    assert abs(q7.z - np.sin(0.25)) < 1e-6 and abs(q9.z - np.sin(0.5)) < 1e-6


# ------------------------------------------------------------------------------- evaluation
class OracleDetector(Detector2D):
    """Returns the ground truth of the frame (looked up by a pixel tag)."""

    def __init__(self, gts):
        self.gts, self.names = gts, ["a", "b"]

    def detect(self, frames):
        out = []
        for f in frames:
            g = self.gts[int(f[0, 0, 0])].copy()
            g[:, 4] = 0.9
            out.append(g.astype(np.float32))
        return out


def _eval_data(n=6):
    gts, imgs = {}, {}
    for s in range(n):
        img = np.zeros((64, 96, 3), np.uint8)
        img[0, 0, 0] = s
        imgs[s] = img
        gts[s] = np.array([[10 + s, 5, 40 + s, 30, 1.0, s % 2]], np.float64)
    return gts, imgs


def _gt_msg(s, g):
    d = detections_to_msg(g, msgs.Header(seq=1000 + s))
    for det in d.detections:
        det.source_img.header.seq = s
    return d


def test_evaluate_inference_live_and_bag(tmp_path):
    gts, imgs = _eval_data()
    # live: gt arrives before / after images in arbitrary order; the bag then repeats
    bus = TopicBus()
    ev = EvaluateInference(engine=OracleDetector(gts), params={"sub_topic": "/img", "gt_topic": "/gt"}, bus=bus,
                           metrics_port=None)
    ev.start_inference(spin=False)
    for s in (3, 1, 0, 2, 5, 4):
        bus.publish("/gt", _gt_msg(s, gts[s]))
    for s in range(6):
        bus.publish("/img", compat.numpy_to_imgmsg(imgs[s], header=msgs.Header(seq=s)))
    bus.publish("/img", compat.numpy_to_imgmsg(imgs[0], header=msgs.Header(seq=0)))  # loop → done
    bus.publish("/gt", _gt_msg(0, gts[0]))
    assert ev.done.wait(30)
    s = ev.finish()
    bus.close()
    assert s.matched_images == 6 and abs(s.map - 0.995) < 1e-6
    # offline from a bag
    bag = str(tmp_path / "eval.bag")
    with Bag(bag, "w") as b:
        for k in range(6):
            b.write("/img", compat.numpy_to_imgmsg(imgs[k], header=msgs.Header(seq=k)))
            b.write("/gt", _gt_msg(k, gts[k]))
    ev2 = EvaluateInference(engine=OracleDetector(gts), params={"sub_topic": "/img", "gt_topic": "/gt"},
                            metrics_port=None)
    s2 = ev2.evaluate_bag(bag, batch=4)
    assert s2.matched_images == 6 and abs(s2.map50 - 0.995) < 1e-6


def test_centerpoint_served_over_kserve():
    """centerpoint_pp contract: 5-feature voxels in (voxel geometry from the served
    config), 9-d det3d boxes out; Detection3DArray reads yaw at index 8."""
    from triton_client_amd.config.lidar import NUSC_PILLARS, CenterPointConfig
    from triton_client_amd.server.models import CenterPointModel
    v = dataclasses.replace(NUSC_PILLARS, point_cloud_range=(-12.8, -12.8, -5.0, 12.8, 12.8, 3.0), max_voxels=4000)
    cfg = CenterPointConfig(voxel=v, score_thresh=0.0, nms_pre_max=16, nms_post_max=4)
    repo = ModelRepository("cpu")
    repo.add(CenterPointModel("centerpoint_pp", cfg=cfg, device="cpu"))
    with KServeServer(repo, "127.0.0.1:0") as srv:
        ch = GRPCChannel({"grpc_channel": srv.target}, Flags("centerpoint_pp"))
        eng = RemoteDetector3D(ch, Pointpillars_client(), z_offset=0.0)
        assert eng.pre.cfg.num_point_features == 5 and eng.pre.cfg == v
        p = eng.detect([_cloud(3)])[0]
        assert p["pred_boxes"].shape[1] == 9 and len(p["pred_scores"]) == 6 * 4
        assert set(np.unique(p["pred_labels"])) <= set(range(10))
        m = boxes_to_detection3d(p, [0], msgs.Header())
        q = m.detections[0].bbox.center.orientation
        assert abs(q.z - np.sin(p["pred_boxes"][0, 8] / 2)) < 1e-5
        ch.close()
    # the in-process engine (same seed, same voxeliser) returns the served result
    local = LocalDetector3D(cfg=cfg, device="cpu", family="centerpoint", z_offset=0.0)
    assert local.family == "centerpoint" and local.box_dim == 9
    lp = local.detect([_cloud(3)])[0]
    np.testing.assert_allclose(np.sort(lp["pred_scores"]), np.sort(p["pred_scores"]), rtol=1e-5, atol=1e-6)


def test_second_iou_served_over_kserve():
    """second_iou contract (examples/second_iou/config.pbtxt): the client voxelises
    with the served SECOND geometry (5 points per voxel, 0.05 m x 0.05 m x 0.1 m),
    the server runs the sparse 3D backbone + RoI IoU head, 7-d boxes come back."""
    from triton_client_amd.config.lidar import KITTI_SECOND_VOXELS, SecondIoUConfig
    from triton_client_amd.server.models import SecondIoUModel
    v = dataclasses.replace(KITTI_SECOND_VOXELS, point_cloud_range=(0.0, -12.8, -3.0, 25.6, 12.8, 1.0),
                            max_voxels=16000)
    cfg = SecondIoUConfig(voxel=v, score_thresh=0.0)
    repo = ModelRepository("cpu")
    repo.add(SecondIoUModel("second_iou", cfg=cfg, device="cpu"))
    with KServeServer(repo, "127.0.0.1:0") as srv:
        ch = GRPCChannel({"grpc_channel": srv.target}, Flags("second_iou"))
        eng = RemoteDetector3D(ch, Pointpillars_client(), z_offset=0.0)
        assert eng.pre.cfg == v and eng.pre.cfg.max_points_per_voxel == 5
        p = eng.detect([_cloud(2)])[0]
        assert p["pred_boxes"].shape[1] == 7 and 0 < len(p["pred_scores"]) <= cfg.nms_post_max
        assert set(np.unique(p["pred_labels"])) <= {1, 2, 3}
        ch.close()
    local = LocalDetector3D(cfg=cfg, device="cpu", family="second_iou", z_offset=0.0)
    lp = local.detect([_cloud(2)])[0]
    assert lp["pred_boxes"].shape == p["pred_boxes"].shape
    np.testing.assert_allclose(np.sort(lp["pred_scores"]), np.sort(p["pred_scores"]), rtol=1e-5, atol=1e-6)
    from triton_client_amd.cli.engines import lidar_family
    assert [lidar_family(n) for n in ("second_iou", "pointpillar_kitti", "centerpoint_pp")] == [
        "second_iou", "pointpillars", "centerpoint"]


def test_check_voxel_inputs_rejects_out_of_range_cells():
    """Host-side validation of served voxel inputs (the GPU consumers index the canvas
    with these coordinates): cells outside the grid and counts outside [1, P] are refused."""
    from triton_client_amd.server.model import InferError
    from triton_client_amd.server.models import check_voxel_inputs

    V, P = 5, 32
    grid = (432, 496, 1)
    ok = {"voxels": np.zeros((V, P, 4), np.float32), "voxel_coords": np.zeros((V, 4), np.int32),
          "voxel_num_points": np.ones((V,), np.int32)}
    assert check_voxel_inputs(ok, P, 100, grid) == V
    for key, idx, val in (("voxel_coords", (2, 3), 432), ("voxel_coords", (1, 2), -1), ("voxel_coords", (0, 1), 1),
                          ("voxel_num_points", (3,), 0), ("voxel_num_points", (4,), P + 1)):
        bad = {k: v.copy() for k, v in ok.items()}
        bad[key][idx] = val
        with pytest.raises(InferError):
            check_voxel_inputs(bad, P, 100, grid)
