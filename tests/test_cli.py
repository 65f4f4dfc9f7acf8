"""Entry points (main/main3d/bag2d/bag3d/evaluate/record) on the CPU with
synthetic bags; remote engines against the in-process KServe server."""
import json
import os

import pytest
import yaml

from triton_client_amd.cli import bag2d, bag3d, evaluate, main as main2d, main3d, record
from triton_client_amd.ros import Bag, reset_default_bus
from triton_client_amd.server import KServeServer, ModelRepository
from triton_client_amd.server.models import YoloV5Model


@pytest.fixture(scope="module")
def bags(tmp_path_factory):
    d = tmp_path_factory.mktemp("bags")
    cam, pc = str(d / "cam.bag"), str(d / "pc.bag")
    assert record.main([cam, "--frames", "4", "--cam", "96x160", "--gt"]) == 0
    assert record.main([pc, "--frames", "2", "--no-camera", "--lidar", "--rings", "16", "--columns", "256"]) == 0
    return d, cam, pc


@pytest.fixture(scope="module")
def server():
    repo = ModelRepository("cpu")
    repo.add(YoloV5Model("YOLOv5n", img=128, device="cpu"))
    srv = KServeServer(repo, "127.0.0.1:0").start()
    yield srv
    srv.stop()


def test_reference_flags_parse():
    f = main2d.parse_args(["-v", "-a", "-m", "YOLOv5nCROP", "-x", "1", "-b", "2", "-c", "2", "-s", "VGG", "-i", "local"])
    assert (f.verbose, f.async_set, f.model_name, f.model_version, f.batch_size, f.classes, f.scaling,
            f.image_src) == (True, True, "YOLOv5nCROP", "1", 2, 2, "VGG", "local")
    f3 = main3d.parse_args(["--streaming"])
    assert f3.streaming and f3.model_name == "pointpillar_kitti" and f3.score_thresh == 0.5 and f3.labels == "2"


def test_bag2d_local_and_remote(bags, server, tmp_path):
    d, cam, _ = bags
    out = str(tmp_path / "png")
    assert bag2d.main(["--bag", cam, "--engine", "local", "--device", "cpu", "--out", out,
                       "--frames-per-step", "2"]) == 0
    assert len(os.listdir(out)) == 4
    params = tmp_path / "p.yaml"
    params.write_text(yaml.safe_dump({"grpc_channel": server.target, "sub_topic": "/camera/color/image_raw",
                                      "pub_topic": "/det", "gt_topic": "/camera/color/Detection2DArray"}))
    ob = str(tmp_path / "o.bag")
    assert bag2d.main(["--bag", cam, "--params", str(params), "-m", "YOLOv5n", "--out", "", "--out-bag", ob,
                       "-a"]) == 0
    with Bag(ob) as b:
        assert sum(1 for t, _, _ in b.read_messages(topics=["/det"])) == 4


def test_bag3d_local(bags, tmp_path):
    _, _, pc = bags
    ob = str(tmp_path / "pc_out.bag")
    assert bag3d.main(["--bag", pc, "--engine", "local", "--device", "cpu", "--out-bag", ob, "--labels", "all",
                       "--score-thresh", "0"]) == 0
    with Bag(ob) as b:
        out = [m for t, m, _ in b.read_messages(topics=["/detections_3d"])]
    assert len(out) == 2 and all(len(m.boxes) > 0 for m in out)


def test_evaluate_bag(bags, tmp_path):
    _, cam, _ = bags
    js = str(tmp_path / "eval.json")
    assert evaluate.main(["--bag", cam, "--engine", "local", "--device", "cpu", "-m", "YOLOv5nCROP",
                          "--eval-port", "0", "--json", js]) == 0
    s = json.load(open(js))
    assert s["matched_images"] == 4 and 0.0 <= s["map50_95"] <= 1.0


def test_main_plays_bag_through_topic_bus(bags, server, tmp_path):
    _, cam, _ = bags
    reset_default_bus()
    params = tmp_path / "p.yaml"
    params.write_text(yaml.safe_dump({"grpc_channel": server.target, "sub_topic": "/camera/color/image_raw",
                                      "pub_topic": "/det", "gt_topic": "/gt"}))
    assert main2d.main(["--params", str(params), "--play", cam, "--spin-timeout", "60"]) == 0
    reset_default_bus()


def test_bag2d_data_parallel_torchrun(bags, tmp_path):
    """torchrun --nproc-per-node 2 bag2d --engine local: frames sharded over 2 gloo ranks."""
    import socket
    import subprocess
    import sys

    _, cam, _ = bags
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ob = str(tmp_path / "dp.bag")
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "triton_client_amd.cli.bag2d",
                        "--bag", cam, "--engine", "local", "--device", "cpu", "--out", "", "--out-bag", ob,
                        "--frames-per-step", "4", "-m", "YOLOv5nCROP"],
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    with Bag(ob) as b:
        dets = [m for t, m, _ in b.read_messages(topics=["/aver_01/camera_color/detection/detections"])]
    assert len(dets) == 4 and [d.header.seq for d in dets] == [0, 1, 2, 3]


def test_bagtools_and_bev(bags, tmp_path):
    import numpy as np
    from triton_client_amd.cli import bagtools
    from triton_client_amd.utils.visualize import boxes_to_corners_3d, render_bev
    _, cam, pc = bags
    assert bagtools.main(["info", cam]) == 0
    dst = str(tmp_path / "cut.bag")
    assert bagtools.main(["stitch", cam, dst, "-n", "3"]) == 0
    with Bag(dst) as b:
        assert b.get_message_count() == 3
    out = str(tmp_path / "pcs")
    assert bagtools.main(["extract-pc", pc, out, "--bev", "--scene"]) == 0
    files = sorted(os.listdir(out))
    assert files == ["000000.npy", "000000.png", "000000_scene.png", "000001.npy", "000001.png", "000001_scene.png"]
    pts = np.load(os.path.join(out, "000000.npy"))
    assert pts.shape[1] == 4 and np.isfinite(pts).all()
    c = boxes_to_corners_3d(np.array([[1.0, 2.0, 0.0, 4.0, 2.0, 1.5, np.pi / 2]]))
    np.testing.assert_allclose(c[0, :, 0].max() - c[0, :, 0].min(), 2.0, atol=1e-9)  # rotated 90°: x extent = dy
    img = render_bev(pts, boxes=np.array([[20.0, 0.0, -1.0, 4.0, 2.0, 1.5, 0.3]]))
    assert img.shape == (691, 794, 3) and (img[..., 1] == 230).any()
