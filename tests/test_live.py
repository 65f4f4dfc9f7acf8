"""The live drivers' device path (inference/live.py, pipelines/stream.py): GPU
annotation with labels, columnar messages, host staging copies, and — on the
GPU — published results equal to the per-frame engine path's."""
import ctypes
import io
import pickle

import numpy as np
import pytest
import torch

from triton_client_amd.ros import compat, msgs, rosmsg
from triton_client_amd.utils.draw import draw_detections, label_text, names_table, text_mask


# ------------------------------------------------------------------ labels (host painter)
@pytest.mark.parametrize("conf,want", [(0.125, "0.12"), (0.375, "0.38"), (0.625, "0.62"), (0.875, "0.88"),
                                       (0.3, "0.30"), (0.99999, "1.00"), (1.0, "1.00"), (0.0, "0.00"),
                                       (-0.2, "0.00"), (float("nan"), "0.00"), (12.3456, "12.35")])
def test_label_text_rounds_half_even_like_format(conf, want):
    assert label_text(3, conf, ["a", "b", "c", "truck"]) == f"truck {want}"
    if np.isfinite(conf) and conf >= 0:  # the exact-value rounding is what '{:.2f}' does
        assert want == f"{float(np.float32(conf)):.2f}"


def test_label_text_names_and_ids():
    assert label_text(5, 0.5, ["x"]) == "5 0.50"          # id outside the table
    assert label_text(0, 0.5, None) == "0 0.50"
    assert label_text(0, 0.5, ["café"]) == "caf? 0.50"  # non-ASCII -> '?'
    assert label_text(0, 0.5, ["n" * 40]) == "n" * 31 + " 0.50"
    t = names_table(["person", "café", "n" * 40])
    assert t.shape == (3, 32) and bytes(t[0, :7]) == b"person\0" and bytes(t[1, :4]) == b"caf?"
    assert t[2, 31] == 0 and bytes(t[2, :31]) == b"n" * 31


def test_label_pixels_and_clipping():
    img = np.zeros((40, 60, 3), np.uint8)
    d = np.array([[10.0, 20.0, 50.0, 35.0, 0.9, 1]], np.float32)  # class 0 is black
    draw_detections(img, d, ["x", "ab"], thickness=1)
    m = text_mask("ab 0.90")
    assert m.shape == (11, 42)
    # label at (x1 + 2, y1 - 11), drawn over the rectangle
    region = img[9:20, 12:54]
    assert ((region.sum(-1) > 0) >= m).all()
    # near the edges: clipped, no error
    img2 = np.zeros((12, 16, 3), np.uint8)
    draw_detections(img2, np.array([[-5, 3, 30, 30, 0.5, 1]], np.float32), None)
    assert img2.any()


# ------------------------------------------------------------------ columnar messages
def _pred(n=7, seed=0, dim=7):
    g = np.random.default_rng(seed)
    return {"pred_boxes": g.normal(0, 5, (n, dim)).astype(np.float32),
            "pred_scores": g.uniform(0, 1, n).astype(np.float32),
            "pred_labels": g.integers(1, 4, n).astype(np.int64)}


def test_array_list_builds_once_and_behaves_like_a_list():
    calls = []

    def build():
        calls.append(1)
        return [1, 2, 3]
    a = msgs.ArrayList(3, build, {"k": 1})
    assert len(a) == 3 and bool(a) and not a.built and not calls
    assert list(a) == [1, 2, 3] and a[1] == 2 and a == [1, 2, 3] and len(calls) == 1
    a.append(4)
    assert len(a) == 4 and a[-1] == 4 and len(calls) == 1
    b = pickle.loads(pickle.dumps(msgs.ArrayList(2, lambda: ["x", "y"])))
    assert b == ["x", "y"] and type(b) is list
    assert msgs.to_dict(msgs.BoundingBoxArray(boxes=msgs.ArrayList(0, list)))["boxes"] == []


@pytest.mark.parametrize("dim", [7, 9])
def test_jsk_columns_match_object_message_and_serialise_identically(dim):
    from triton_client_amd.inference.ros_inference3d import boxes_to_jsk, select_boxes

    p = _pred(40, 1, dim)
    hdr = msgs.Header(seq=7, stamp=msgs.Time(3, 4), frame_id="os")
    idx = select_boxes(p, (2,), 0.5)
    lazy = boxes_to_jsk(p, idx, hdr)
    assert len(lazy.boxes) == len(idx) > 0 and not lazy.boxes.built
    fast = rosmsg.serialize(lazy)  # packed from the columns
    assert not lazy.boxes.built
    # the reference's per-box construction (ros_inference3d.py:158-178)
    yi = 8 if dim >= 9 else 6
    ref = msgs.BoundingBoxArray(header=hdr)
    for i in idx:
        x = p["pred_boxes"][i]
        ref.boxes.append(msgs.BoundingBox(
            header=hdr, pose=msgs.Pose(msgs.Point(float(x[0]), float(x[1]), float(x[2])),
                                       compat.yaw2quaternion(float(x[yi]))),
            dimensions=msgs.Vector3(float(x[4]), float(x[3]), float(x[5])),
            value=float(p["pred_scores"][i]), label=int(p["pred_labels"][i])))
    assert list(lazy.boxes) == ref.boxes  # builds
    assert fast == rosmsg.serialize(ref)
    back = rosmsg.deserialize(fast, "jsk_recognition_msgs/BoundingBoxArray")
    assert back.boxes == ref.boxes


def test_detection2d_columns():
    from triton_client_amd.inference.ros_inference import detections_to_msg

    d = np.array([[1, 2, 11, 22, 0.5, 3], [0, 0, 4, 4, 0.25, 1]], np.float32)
    m = detections_to_msg(d, msgs.Header(seq=1))
    assert len(m.detections) == 2 and not m.detections.built
    np.testing.assert_array_equal(m.detections.columns["dets"], d)
    det = m.detections[0]
    assert det.results[0].id == 3 and det.bbox.size_x == 10 and det.bbox.center.y == 12
    rosmsg.serialize(m)


# ------------------------------------------------------------------ host staging copies
def test_host_gather_copy():
    from triton_client_amd import _native
    from triton_client_amd.inference.live import gather_copy

    try:
        _native.runtime()
    except _native.NativeError:
        pytest.skip("runtime library not built")
    g = np.random.default_rng(0)
    srcs = [g.integers(0, 255, n, dtype=np.uint8).tobytes() for n in (0, 5, 3 << 20, 1 << 20, 12345)]
    dst = np.zeros(sum(len(s) for s in srcs) + 64, np.uint8)
    offs = np.cumsum([0] + [len(s) for s in srcs])[:-1]
    gather_copy([dst.ctypes.data + int(o) for o in offs], [memoryview(s) for s in srcs], [len(s) for s in srcs], 4)
    np.testing.assert_array_equal(dst[:-64], np.frombuffer(b"".join(srcs), np.uint8))
    assert not dst[-64:].any()
    rt = _native.runtime()
    assert rt.tca_host_gather_copy(-1, None, None, None, 1) == -1


def test_flatten_rebuild_results():
    from triton_client_amd.ops.centerpoint import CenterPointResult
    from triton_client_amd.ops.nms import NmsResult
    from triton_client_amd.pipelines.stream import flatten_tensors, rebuild

    r = NmsResult(torch.zeros(2, 3, 4), torch.ones(2, 3), torch.zeros(2, 3, dtype=torch.int32),
                  torch.tensor([1, 2], dtype=torch.int32))
    c = CenterPointResult(r, 1, 2)
    ts = flatten_tensors(c)
    assert len(ts) == 4 and ts[3] is r.count
    c2 = rebuild(c, [t + 1 for t in ts])
    assert isinstance(c2, CenterPointResult) and c2.batch == 1 and c2.ntask == 2
    assert torch.equal(c2.nms.score, r.score + 1)


# ------------------------------------------------------------------ GPU
def _annot_case(B=3, H=200, W=320, K=30, seed=0):
    g = np.random.default_rng(seed)
    frames = g.integers(0, 255, (B, H, W, 3), dtype=np.uint8)
    box = np.zeros((B, K, 4), np.float32)
    c = g.uniform(-10, [W + 10, H + 10], (B, K, 2))
    box[..., :2], box[..., 2:] = c, c + g.uniform(0, 60, (B, K, 2))
    box[0, 0] = (10.5, 11.5, 12.5, 13.5)
    box[0, 1] = (30, 30, 20, 40)          # x2 < x1: neither box nor label
    box[1, 0] = (-50, -50, W + 50, H + 50)
    box[1, 1] = (W - 3, H - 2, W + 9, H + 9)  # label runs off the right / bottom edge
    score = g.uniform(0, 1, (B, K)).astype(np.float32)
    score[0, 2], score[0, 3] = 0.125, 0.375  # half-even ties
    cls = g.integers(0, 90, (B, K)).astype(np.int32)  # ids past the names table print as numbers
    count = np.array([K, 7, 0], np.int32)[:B]
    return frames, box, score, cls, count


@pytest.mark.gpu
@pytest.mark.parametrize("t", [1, 3])
def test_draw_annotations_kernel_pixel_exact(cuda, t):
    from triton_client_amd.ops.image import draw_annotations_

    names = ["person", "café", "n" * 40] + [f"cls{i}" for i in range(77)]
    frames, box, score, cls, count = _annot_case(seed=t)
    f = torch.from_numpy(frames).to(cuda)
    nd = torch.from_numpy(names_table(names)).to(cuda)
    draw_annotations_(f, torch.from_numpy(box).to(cuda), torch.from_numpy(score).to(cuda),
                      torch.from_numpy(cls).to(cuda), torch.from_numpy(count).to(cuda), nd, thickness=t)
    want = draw_annotations_(torch.from_numpy(frames.copy()), torch.from_numpy(box), torch.from_numpy(score),
                             torch.from_numpy(cls), torch.from_numpy(count), names=names, thickness=t).numpy()
    got = f.cpu().numpy()
    assert (want != frames).any()
    np.testing.assert_array_equal(got, want)
    # no names table: numeric labels
    f = torch.from_numpy(frames).to(cuda)
    draw_annotations_(f, torch.from_numpy(box).to(cuda), torch.from_numpy(score).to(cuda),
                      torch.from_numpy(cls).to(cuda), torch.from_numpy(count).to(cuda), None, thickness=t)
    want = draw_annotations_(torch.from_numpy(frames.copy()), torch.from_numpy(box), torch.from_numpy(score),
                             torch.from_numpy(cls), torch.from_numpy(count), names=None, thickness=t).numpy()
    np.testing.assert_array_equal(f.cpu().numpy(), want)


def _jpeg(img, q=90):
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG", quality=q)
    return buf.getvalue()


@pytest.mark.gpu
def test_live_camera_matches_engine_path(cuda):
    """JPEG and raw Image messages through the live device path publish the
    engine path's detections (same decoded pixels) and the host painter's
    annotated frame, bit for bit; partial batches and several workers alike."""
    from triton_client_amd.inference import LocalDetector2D
    from triton_client_amd.ops.jpeg import JpegBatchDecoder
    from triton_client_amd.utils.synthetic import camera_frame

    H, W = 360, 640
    eng = LocalDetector2D(batch=4, device=cuda, letterbox=True, calibrate_target=100.0)
    rgb = [camera_frame(H, W, s) for s in range(6)]
    eng.detect(rgb[:1])  # calibrates the shared model once
    names = [f"c{i}" for i in range(80)]
    jp = [_jpeg(f) for f in rgb]
    # the GPU decoder's pixels (what the live path's frames hold)
    dec = JpegBatchDecoder(len(jp), cuda)
    out = torch.empty((len(jp), H, W, 3), dtype=torch.uint8, device=cuda)
    dec.decode(jp, out)
    decoded = list(out.cpu().numpy())
    live = eng.live()
    cm = [msgs.CompressedImage(header=msgs.Header(seq=i + 1), format="jpeg", data=d) for i, d in enumerate(jp)]
    im = [compat.numpy_to_imgmsg(f, "rgb8", msgs.Header(seq=i + 1)) for i, f in enumerate(rgb)]
    for frames_in, ref_frames in ((cm, decoded), (im, rgb)):
        got = live.process(frames_in, draw=True, names=names)  # 6 = one full + one partial batch
        ref = eng.detect(ref_frames)
        assert sum(len(r) for r in ref) > 0
        for (img_msg, d), r, f, m in zip(got, ref, ref_frames, frames_in):
            np.testing.assert_array_equal(d, r)
            assert img_msg.header is m.header and (img_msg.height, img_msg.width, img_msg.step) == (H, W, 3 * W)
            pub = compat.imgmsg_to_numpy(img_msg, "rgb8")
            np.testing.assert_array_equal(pub, draw_detections(f.copy(), r, names))
    # concurrent callers (the driver's workers) get the same answers
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(3) as ex:
        outs = list(ex.map(lambda _: live.process(im, draw=True, names=names), range(3)))
    for o in outs:
        for (_, d), r in zip(o, eng.detect(rgb)):
            np.testing.assert_array_equal(d, r)


@pytest.mark.gpu
def test_live_lidar_matches_engine_path(cuda):
    from triton_client_amd.inference import LocalDetector3D
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep

    eng = LocalDetector3D(batch=2, device=cuda, calibrate_target=500.0)
    clouds = []
    for s in range(5):
        pts = lidar_sweep(LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23), s)
        clouds.append(compat.create_cloud_xyzi(np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4),
                                               msgs.Header(seq=s)))
    ref = eng.detect(clouds)
    got = eng.live().process(clouds)
    assert all(len(p["pred_scores"]) > 0 for p in ref)
    for a, b in zip(got, ref):
        for k in ("pred_boxes", "pred_scores", "pred_labels"):
            np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.gpu
def test_live_drivers_publish_engine_results(cuda):
    """RosInference / RosInference3D with workers over the topic bus: every
    published message carries the engine path's detections, in seq order."""
    import threading

    from triton_client_amd.inference import LocalDetector2D, LocalDetector3D, RosInference, RosInference3D
    from triton_client_amd.inference.ros_inference3d import select_boxes
    from triton_client_amd.ros.bus import TopicBus
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    bus = TopicBus()
    e2 = LocalDetector2D(batch=4, device=cuda, letterbox=True, calibrate_target=100.0)
    rgb = [camera_frame(360, 640, s) for s in range(10)]
    ref2 = e2.detect(rgb)
    e3 = LocalDetector3D(batch=4, device=cuda, calibrate_target=2000.0)
    clouds = []
    for s in range(10):
        pts = lidar_sweep(LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23), s)
        clouds.append(compat.create_cloud_xyzi(np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4),
                                               msgs.Header(seq=s + 1)))
    ref3 = e3.detect(clouds)
    got2, got3, done = [], [], threading.Event()

    def on(lst):
        def cb(m):
            lst.append(m)
            if len(got2) + len(got3) >= 2 * len(rgb):
                done.set()
        return cb
    compat.Subscriber("/cam_out/detections", msgs.Detection2DArray, on(got2), bus=bus)
    compat.Subscriber("/pc_out", msgs.BoundingBoxArray, on(got3), bus=bus)
    d2 = RosInference(engine=e2, params={"sub_topic": "/cam", "pub_topic": "/cam_out"}, bus=bus, batch=4, workers=2,
                      queue_size=64)
    d3 = RosInference3D(engine=e3, params={"sub_topic": "/pc", "pub_topic": "/pc_out"}, bus=bus, batch=4, workers=2,
                        queue_size=64)
    d2.start_inference(spin=False)
    d3.start_inference(spin=False)
    p2 = compat.Publisher("/cam", msgs.Image, bus=bus)
    p3 = compat.Publisher("/pc", msgs.PointCloud2, bus=bus)
    for i, (f, c) in enumerate(zip(rgb, clouds)):
        p2.publish(compat.numpy_to_imgmsg(f, "rgb8", msgs.Header(seq=i + 1)))
        p3.publish(c)
    assert done.wait(120)
    d2.stop()
    d3.stop()
    bus.close()
    assert [m.header.seq for m in got2] == list(range(1, 11))
    assert [m.header.seq for m in got3] == list(range(1, 11))
    for m, r in zip(got2, ref2):
        np.testing.assert_array_equal(m.detections.columns["dets"], r)
    for m, r in zip(got3, ref3):
        idx = select_boxes(r, (2,), 0.5)
        np.testing.assert_array_equal(m.boxes.columns["value"], r["pred_scores"][idx])
        np.testing.assert_array_equal(m.boxes.columns["position"], r["pred_boxes"][idx, :3].astype(np.float64))


@pytest.mark.gpu
def test_engines_build_while_another_streams(cuda):
    """Two live camera engines of new geometries build (pipeline, warm-ups, two graph
    captures each) while a third streams: the streaming engine's submissions keep
    completing during the builds -- only the capture windows exclude them
    (pipelines/graph.py CaptureGate) -- and every thread finishes."""
    import threading
    import time

    from triton_client_amd.inference import LocalDetector2D
    from triton_client_amd.pipelines.graph import capture_gate
    from triton_client_amd.utils.synthetic import camera_frame

    eng = LocalDetector2D(batch=4, device=cuda, letterbox=True, calibrate_target=100.0)
    names = [f"c{i}" for i in range(80)]
    live = eng.live()
    base = [compat.numpy_to_imgmsg(camera_frame(360, 640, s), "rgb8", msgs.Header(seq=s)) for s in range(4)]
    want = live.process(base, draw=True, names=names)
    stop, stamps, errors = threading.Event(), [], []

    def stream():
        try:
            while not stop.is_set():
                got = live.process(base, draw=True, names=names)
                for (_, d), (_, w) in zip(got, want):
                    np.testing.assert_array_equal(d, w)
                stamps.append(time.monotonic())
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def build(hw, seed):
        try:
            m = [compat.numpy_to_imgmsg(camera_frame(hw[0], hw[1], seed), "rgb8", msgs.Header(seq=seed))]
            assert len(live.process(m, draw=True, names=names)) == 1
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    st = threading.Thread(target=stream)
    st.start()
    time.sleep(0.3)
    caps0 = capture_gate(cuda).captures
    t0 = time.monotonic()
    builders = [threading.Thread(target=build, args=(hw, 9 + i)) for i, hw in enumerate([(480, 848), (300, 500)])]
    for b in builders:
        b.start()
    for b in builders:
        b.join(300)
    t1 = time.monotonic()
    stop.set()
    st.join(60)
    assert not errors, errors
    assert not st.is_alive() and not any(b.is_alive() for b in builders)
    assert capture_gate(cuda).captures - caps0 >= 4  # two graphs per new engine
    during = [s for s in stamps if t0 < s < t1]
    gaps = np.diff([t0] + during + [t1])
    assert len(during) >= 3 and gaps.max() < 0.8 * (t1 - t0), (len(during), float(gaps.max()), t1 - t0)
