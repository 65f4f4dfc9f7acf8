"""CPU paths of the per-frame ops vs the sequential golden references
(runs on the GPU-less host)."""
import struct

import numpy as np
import pytest
import torch

from triton_client_amd.config.lidar import KITTI_PILLARS, KITTI_SECOND_VOXELS, NUSC_PILLARS, PointPillarsConfig
from triton_client_amd.ops import golden
from triton_client_amd.ops.image import preprocess
from triton_client_amd.ops.lidar import AnchorPostprocess, PointLayout, Voxelizer, pc2_unpack, voxelize_np
from triton_client_amd.ops.yolo import YoloPostprocess, detections_nx6


def synth_cloud(n, seed=0, nan_frac=0.02, pcr=(0, -40, -3, 70.4, 40, 1)):
    rng = np.random.default_rng(seed)
    # clustered points so that voxels get many points (exercise the P cap)
    centers = rng.uniform([pcr[0] - 5, pcr[1] - 5, pcr[2]], [pcr[3] + 5, pcr[4] + 5, pcr[5]], size=(max(1, n // 200), 3))
    idx = rng.integers(0, len(centers), n)
    sig = np.where(rng.random((n, 1)) < 0.5, 0.03, 0.3)
    xyz = centers[idx] + rng.normal(0, 1.0, size=(n, 3)) * sig
    inten = rng.uniform(0, 255, size=(n, 1))
    p = np.concatenate([xyz, inten], 1).astype(np.float32)
    nanm = rng.random(n) < nan_frac
    p[nanm, rng.integers(0, 4, nanm.sum())] = np.nan
    return p


def test_resize_matches_manual_bilinear():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    out = golden.resize_bilinear_u8(img, 20, 31, quantize=False)
    # independent per-pixel evaluation
    for y in (0, 7, 19):
        for x in (0, 13, 30):
            fy = (y + 0.5) * 37 / 20 - 0.5
            fx = (x + 0.5) * 53 / 31 - 0.5
            y0 = int(np.floor(fy)); ay = fy - y0
            x0 = int(np.floor(fx)); ax = fx - x0
            if y0 < 0: y0, ay = 0, 0.0
            if x0 < 0: x0, ax = 0, 0.0
            if y0 >= 36: y0, ay = 36, 0.0
            if x0 >= 52: x0, ax = 52, 0.0
            y1, x1 = min(y0 + 1, 36), min(x0 + 1, 52)
            f = img.astype(np.float64)
            v = (1 - ay) * ((1 - ax) * f[y0, x0] + ax * f[y0, x1]) + ay * ((1 - ax) * f[y1, x0] + ax * f[y1, x1])
            np.testing.assert_allclose(out[y, x], v, atol=1e-3)


@pytest.mark.parametrize("mode", ["stretch", "letterbox"])
def test_preprocess_cpu_letterbox_geometry(mode):
    rng = np.random.default_rng(1)
    frames = torch.from_numpy(rng.integers(0, 256, size=(2, 72, 128, 3), dtype=np.uint8))
    out, xf = preprocess(frames, (64, 64), mode=mode, scaling="COCO")
    assert out.shape == (2, 3, 64, 64)
    if mode == "letterbox":
        # 128x72 -> 64x36, padded top/bottom with 114/255
        assert xf.pad_y == 14 and xf.pad_x == 0
        np.testing.assert_allclose(out[0, :, 0, :].numpy(), 114 / 255.0, atol=1e-6)
    else:
        assert xf.pad_x == 0 and xf.pad_y == 0
    assert float(out.max()) <= 1.0 and float(out.min()) >= 0.0


def test_scaling_presets():
    frames = torch.full((1, 4, 4, 3), 200, dtype=torch.uint8)
    o, _ = preprocess(frames, (4, 4), scaling="INCEPTION")
    np.testing.assert_allclose(o.numpy(), 200 / 127.5 - 1, rtol=1e-6)
    o, _ = preprocess(frames, (4, 4), scaling="VGG")
    np.testing.assert_allclose(o[0, :, 0, 0].numpy(), [77, 83, 96])


def test_nms_greedy_vs_bruteforce():
    rng = np.random.default_rng(2)
    n = 200
    xy = rng.uniform(0, 100, (n, 2))
    wh = rng.uniform(5, 30, (n, 2))
    boxes = np.concatenate([xy, xy + wh], 1).astype(np.float32)
    scores = rng.random(n).astype(np.float32)
    cls = rng.integers(0, 3, n)
    keep = golden.nms_greedy(boxes, scores, 0.45, cls)
    # brute-force check of the greedy invariants
    kept = set(keep)
    order = np.argsort(-scores, kind="stable")
    for i in order:
        sup = any(golden.box_iou_np(boxes[[k]], boxes[[i]])[0, 0] > 0.45 and cls[k] == cls[i] and scores[k] > scores[i]
                  for k in kept if k != i)
        assert (i in kept) == (not sup)


def test_rotated_iou_axis_aligned_matches_aa_iou():
    a = np.array([0, 0, 0, 4, 2, 1, 0], np.float64)
    b = np.array([1, 0.5, 0, 4, 2, 1, 0], np.float64)
    aa = golden.box_iou_np(np.array([[-2, -1, 2, 1]]), np.array([[-1, -0.5, 3, 1.5]]))[0, 0]
    np.testing.assert_allclose(golden.rotated_iou_bev(a, [b])[0], aa, rtol=1e-9)
    # 90-degree rotation of a square is the same square
    s = np.array([0, 0, 0, 2, 2, 1, 0.0])
    r = np.array([0, 0, 0, 2, 2, 1, np.pi / 2])
    np.testing.assert_allclose(golden.rotated_iou_bev(s, [r])[0], 1.0, atol=1e-9)
    # 45-degree rotated square vs axis-aligned: octagon area = 8(sqrt2-1)
    r45 = np.array([0, 0, 0, 2, 2, 1, np.pi / 4])
    inter = 8 * (np.sqrt(2) - 1)
    np.testing.assert_allclose(golden.rotated_iou_bev(s, [r45])[0], inter / (8 - inter), rtol=1e-9)


def _pc2_bytes(p, step=16):
    return p.astype(np.float32).tobytes() if step == 16 else None


def test_pc2_unpack_cpu_vs_read_points():
    p = synth_cloud(3000, seed=3)
    data = p.tobytes()
    ref = golden.pc2_read_points(data, len(p), 16, (0, 4, 8, 12), (7, 7, 7, 7))
    ref[:, 3] /= ref[:, 3].max()
    ref[:, 2] += 1.5
    pts, cnt = pc2_unpack(None, torch.frombuffer(bytearray(data), dtype=torch.uint8),
                          torch.tensor([0]), torch.tensor([len(p)], dtype=torch.int32), PointLayout.xyzi_f32(),
                          4096, True, 1.5)
    assert int(cnt[0]) == len(ref)
    np.testing.assert_allclose(pts[0, :len(ref)].numpy(), ref, rtol=1e-6, atol=1e-6)


def test_pc2_mixed_field_types():
    # x,y,z float32, padding, intensity uint16 (Ouster-like 24 B record)
    n = 100
    rng = np.random.default_rng(4)
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("pad", "<u4"), ("i", "<u2"), ("r", "<u2"), ("t", "<u4")])
    rec["x"], rec["y"], rec["z"] = rng.normal(size=(3, n))
    rec["i"] = rng.integers(0, 60000, n)
    data = rec.tobytes()
    lay = PointLayout(rec.dtype.itemsize, (0, 4, 8, 16), (7, 7, 7, 4))
    pts, cnt = pc2_unpack(None, torch.frombuffer(bytearray(data), dtype=torch.uint8), torch.tensor([0]),
                          torch.tensor([n], dtype=torch.int32), lay, 128, False, 0.0)
    ref = golden.pc2_read_points(data, n, rec.dtype.itemsize, (0, 4, 8, 16), (7, 7, 7, 4))
    np.testing.assert_allclose(pts[0, :n].numpy(), ref)


@pytest.mark.parametrize("vcfg", [KITTI_PILLARS, KITTI_SECOND_VOXELS, NUSC_PILLARS])
def test_voxelize_np_matches_sequential(vcfg):
    import dataclasses
    cfg = dataclasses.replace(vcfg, max_voxels=300)  # force the max_voxels cap
    r = cfg.point_cloud_range
    p = synth_cloud(4000, seed=5, nan_frac=0.0, pcr=r)
    if cfg.num_point_features == 5:
        p = np.concatenate([p, np.zeros((len(p), 1), np.float32)], 1)
    v1, c1, n1 = golden.voxelize_sequential(p, r, cfg.voxel_size, cfg.max_points_per_voxel, cfg.max_voxels)
    v2, c2, n2, _ = voxelize_np(p, cfg)
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(n1, n2)
    np.testing.assert_array_equal(v1, v2)
    assert n1.max() == cfg.max_points_per_voxel  # the per-voxel cap was exercised


def test_yolo_postprocess_cpu_semantics():
    from triton_client_amd.models.yolov5 import DEFAULT_ANCHORS
    rng = np.random.default_rng(6)
    N, nc = 500, 4
    pred = np.zeros((1, N, 5 + nc), np.float32)
    pred[0, :, :2] = rng.uniform(50, 500, (N, 2))
    pred[0, :, 2:4] = rng.uniform(10, 80, (N, 2))
    pred[0, :, 4] = rng.random(N)
    pred[0, :, 5:] = rng.random((N, nc))
    pp = YoloPostprocess(nc, DEFAULT_ANCHORS, conf_thres=0.3, iou_thres=0.45, device="cpu")
    res = pp.postprocess_decoded(pred)
    det = detections_nx6(res)[0]
    # reference semantics, re-derived: filter obj, conf = obj*cls, best class, conf filter, class-aware greedy NMS
    x = pred[0][pred[0, :, 4] > 0.3]
    conf = x[:, 5:] * x[:, 4:5]
    j = conf.argmax(1)
    c = conf[np.arange(len(j)), j]
    m = c > 0.3
    b = np.stack([x[:, 0] - x[:, 2] / 2, x[:, 1] - x[:, 3] / 2, x[:, 0] + x[:, 2] / 2, x[:, 1] + x[:, 3] / 2], 1)[m]
    keep = golden.nms_greedy(b, c[m], 0.45, j[m])
    np.testing.assert_allclose(det[:, :4], b[keep], rtol=1e-6)
    np.testing.assert_array_equal(det[:, 5].astype(int), j[m][keep])


def test_anchor_postprocess_cpu_runs():
    cfg = PointPillarsConfig()
    ap = AnchorPostprocess(cfg, 1, device="cpu")
    H, W, A, C = ap.H, ap.W, ap.A, ap.C
    g = torch.Generator().manual_seed(0)
    cls = torch.randn(1, A * C, H, W, generator=g) - 3.0
    box = torch.randn(1, A * 7, H, W, generator=g) * 0.1
    dr = torch.randn(1, A * 2, H, W, generator=g)
    res = ap.cpu(cls, box, dr)
    n = int(res.count[0])
    assert 0 < n <= cfg.nms_post_max
    b = res.box[0, :n].numpy().astype(np.float64)
    # kept boxes respect the NMS threshold pairwise
    for i in range(min(n, 40)):
        ious = golden.rotated_iou_bev(b[i], b[i + 1:min(n, 40)])
        assert np.all(ious <= cfg.nms_thresh + 1e-6)
