"""K15 box annotation (csrc/kernels/draw.hip, ops.image.draw_boxes_) against the
host painter utils.draw (reference ros_inference.py:149-169 rectangles)."""
import numpy as np
import pytest
import torch

from triton_client_amd.ops.image import draw_boxes_
from triton_client_amd.utils.draw import draw_detections


def _case(B=3, H=72, W=96, K=12, seed=0):
    g = np.random.default_rng(seed)
    frames = g.integers(0, 255, (B, H, W, 3), dtype=np.uint8)
    box = np.zeros((B, K, 4), np.float32)
    c = g.uniform(-10, [W + 10, H + 10], (B, K, 2))
    wh = g.uniform(0, 40, (B, K, 2))
    box[..., :2], box[..., 2:] = c, c + wh
    box[0, 0] = (10.5, 11.5, 12.5, 13.5)   # round-half-even corners
    box[0, 1] = (30, 30, 20, 40)           # x2 < x1: skipped
    box[1, 0] = (-50, -50, W + 50, H + 50)  # clipped to the frame
    cls = g.integers(0, 80, (B, K)).astype(np.int32)
    count = np.array([K, 5, 0], np.int32)[:B]
    return frames, box, cls, count


def _host(frames, box, cls, count, t):
    out = frames.copy()
    for b in range(len(out)):
        k = int(count[b])
        dets = np.concatenate([box[b, :k], np.ones((k, 1), np.float32), cls[b, :k, None].astype(np.float32)], 1)
        draw_detections(out[b], dets, labels=False, thickness=t)
    return out


@pytest.mark.parametrize("t", [1, 2, 5])
def test_draw_boxes_cpu_matches_host_painter(t):
    frames, box, cls, count = _case()
    got = draw_boxes_(torch.from_numpy(frames.copy()), torch.from_numpy(box), torch.from_numpy(cls),
                      torch.from_numpy(count), t).numpy()
    np.testing.assert_array_equal(got, _host(frames, box, cls, count, t))


@pytest.mark.gpu
@pytest.mark.parametrize("t", [1, 2, 5])
def test_draw_boxes_kernel_pixel_exact(cuda, t):
    frames, box, cls, count = _case(B=3, H=360, W=640, K=40, seed=t)
    f = torch.from_numpy(frames).to(cuda)
    draw_boxes_(f, torch.from_numpy(box).to(cuda), torch.from_numpy(cls).to(cuda), torch.from_numpy(count).to(cuda), t)
    np.testing.assert_array_equal(f.cpu().numpy(), _host(frames, box, cls, count, t))


@pytest.mark.gpu
def test_local_2d_detect_annotated(cuda):
    from triton_client_amd.inference import LocalDetector2D
    from triton_client_amd.utils.synthetic import camera_frame

    eng = LocalDetector2D(batch=2, device=cuda, letterbox=True)
    frames = [camera_frame(360, 640, s) for s in range(3)]
    dets, imgs = eng.detect_annotated(frames)
    ref = eng.detect(frames)
    assert sum(len(d) for d in dets) > 0
    for d, r, img, f in zip(dets, ref, imgs, frames):
        np.testing.assert_array_equal(d, r)
        want = draw_detections(f.copy(), d, labels=False)
        np.testing.assert_array_equal(img, want)
