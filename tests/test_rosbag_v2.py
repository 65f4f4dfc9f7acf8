"""ROS bag v2.0 I/O (ros/rosbag_v2.py, ros/rosmsg.py) against a hand-built
fixture (tests/fixtures/make_ros1_bag.py writes it byte by byte, without this
package's codec), round trips of every message type the drivers write, and
bag2d / bag3d replaying the fixture into ROS v2 output bags."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures"))
from make_ros1_bag import cloud, jpeg  # noqa: E402
from triton_client_amd.ros import Bag, compat, msgs, rosmsg
from triton_client_amd.ros.bag import stitch
from triton_client_amd.ros.rosbag_v2 import RawMessage

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "ros1_sensors.bag")


def test_md5_matches_published_sums():
    known = {"std_msgs/Header": "2176decaecbce78abc3b96ef049fabed",
             "sensor_msgs/Image": "060021388200f6f0f447d0fcd9c64743",
             "sensor_msgs/CompressedImage": "8f7a12909da2c9d3332d540a0977563f",
             "sensor_msgs/PointCloud2": "1158d486dd51d683ce2f1be655c3c181",
             "sensor_msgs/PointField": "268eacb2962780ceac86cbd17e328150",
             "geometry_msgs/Pose": "e45d45a5a1ce597b249e23fb30fc871f",
             "geometry_msgs/PoseWithCovariance": "c23e848cf1b7533a8d7c259073a97e6f",
             "geometry_msgs/Pose2D": "938fa65709584ad8e77d238529be13b8"}
    for t, m in known.items():
        assert rosmsg.md5sum(t) == m, t


def test_fixture_reads():
    with Bag(FIX) as b:
        info = b.get_type_and_topic_info()
        assert {k: v["count"] for k, v in info.items()} == {
            "/camera/color/image_raw": 3, "/camera/color/image_raw_rgb": 2,
            "/ai_test_field/sensors/os_cloud_node/points": 2, "/diagnostics_raw": 1}
        got = list(b.read_messages())
    cams = [m for t, m, _ in got if t == "/camera/color/image_raw"]
    assert [m.header.seq for m in cams] == [0, 1, 2] and cams[1].header.stamp == msgs.Time(101, 0)
    assert cams[2].format == "jpeg" and cams[2].data == jpeg(2)
    assert compat.jpeg_decode_rgb(cams[0].data).shape == (48, 64, 3)
    rgb = [m for t, m, _ in got if t == "/camera/color/image_raw_rgb"]
    assert rgb[1].encoding == "rgb8" and (rgb[1].height, rgb[1].width, rgb[1].step) == (24, 32, 96)
    assert compat.imgmsg_to_numpy(rgb[1], "rgb8")[0, 0].tolist() == [47, 47, 47]
    pcs = [m for t, m, _ in got if t.endswith("points")]
    assert [f.name for f in pcs[0].fields] == ["x", "y", "z", "intensity"]
    np.testing.assert_array_equal(np.frombuffer(pcs[1].data, np.float32).reshape(-1, 4), cloud(11))
    raw = [m for t, m, _ in got if t == "/diagnostics_raw"][0]
    assert isinstance(raw, RawMessage) and raw.type == "acme_msgs/Opaque" and raw.data == b"\x01\x02\x03\x04"


def _all_types():
    h = msgs.Header(seq=7, stamp=msgs.Time(5, 6), frame_id="f")
    pose = msgs.Pose(msgs.Point(1.0, 2.0, 3.0), msgs.Quaternion(0.0, 0.0, 0.6, 0.8))
    box = msgs.BoundingBox(header=h, pose=pose, dimensions=msgs.Vector3(4.0, 1.5, 1.6), value=0.75, label=2)
    img = msgs.Image(header=h, height=2, width=2, encoding="rgb8", step=6, data=bytes(range(12)))
    hyp = msgs.ObjectHypothesisWithPose(id=3, score=0.9, pose=pose)
    d2 = msgs.Detection2D(header=h, results=[hyp], bbox=msgs.BoundingBox2D(msgs.Pose2D(5.0, 6.0, 0.0), 2.0, 3.0),
                          source_img=img)
    d3 = msgs.Detection3D(header=h, results=[hyp], bbox=msgs.BoundingBox3D(pose, msgs.Vector3(1.0, 2.0, 3.0)))
    pc = msgs.PointCloud2(header=h, height=1, width=2, fields=[msgs.PointField("x", 0, 7, 1)], point_step=4,
                          row_step=8, data=b"\x00" * 8, is_dense=True)
    return [("/img", img), ("/cimg", msgs.CompressedImage(header=h, format="jpeg", data=b"\xff\xd8xyz")),
            ("/pc", pc), ("/boxes", msgs.BoundingBoxArray(header=h, boxes=[box, box])),
            ("/d2", msgs.Detection2DArray(header=h, detections=[d2])),
            ("/d3", msgs.Detection3DArray(header=h, detections=[d3, d3]))]


@pytest.mark.parametrize("compression", ["none", "bz2"])
def test_write_read_round_trip(tmp_path, compression):
    path = str(tmp_path / "rt.bag")
    items = _all_types()
    with Bag(path, "w", compression=compression) as b:
        for k in range(3):
            for topic, m in items:
                b.write(topic, m, msgs.Time(10 + k, k))
    with Bag(path) as b:
        got = list(b.read_messages())
        assert b.get_message_count(["/d3"]) == 3
    assert len(got) == 3 * len(items)
    for (topic, m, t), (want_topic, want) in zip(got, items * 3):
        assert topic == want_topic and m == want, topic
    assert got[-1][2] == msgs.Time(12, 2)


def test_stitch_and_resume(tmp_path):
    out = str(tmp_path / "first4.bag")
    assert stitch(FIX, out, n=4) == 4
    with Bag(out) as b:
        assert [t for t, _, _ in b.read_messages()] == ["/camera/color/image_raw"] * 3 + ["/camera/color/image_raw_rgb"]
    with Bag(FIX) as b:
        seqs = [m.header.seq for _, m, _ in b.read_messages(["/camera/color/image_raw"], start_seq=1)]
    assert seqs == [1, 2]


def test_bag2d_bag3d_replay_fixture(tmp_path):
    from triton_client_amd.cli import bag2d, bag3d

    ob = str(tmp_path / "cam_out.bag")
    assert bag2d.main(["--bag", FIX, "--engine", "local", "--device", "cpu", "--out", "", "--out-bag", ob,
                       "--frames-per-step", "2"]) == 0
    with Bag(ob) as b:
        info = b.get_type_and_topic_info()
    assert info["/camera/color/image_raw"]["count"] == 3
    assert info["/aver_01/camera_color/detection"]["type"] == "sensor_msgs/Image"
    assert info["/aver_01/camera_color/detection/detections"]["type"] == "vision_msgs/Detection2DArray"
    ob3 = str(tmp_path / "pc_out.bag")
    assert bag3d.main(["--bag", FIX, "--engine", "local", "--device", "cpu", "--out-bag", ob3, "--labels", "all",
                       "--score-thresh", "0"]) == 0
    with Bag(ob3) as b:
        out = [m for t, m, _ in b.read_messages(topics=["/detections_3d"])]
        assert b.get_type_and_topic_info()["/detections_3d"]["md5sum"] == rosmsg.md5sum(
            "jsk_recognition_msgs/BoundingBoxArray")
    assert len(out) == 2 and [m.header.seq for m in out] == [0, 1]
