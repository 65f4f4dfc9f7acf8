"""YOLOv5 decode at output sizes that are not a multiple of 4 floats, and the class
filter's order (best class over ALL classes first, then the ``classes`` filter drops the
row), against a direct transcription of the reference's order.

Reference: ``clients/postprocess/yolov5_postprocess.py:84-92`` (``x[:, 5:].max(1)``, then
``x[(x[:, 5:6] == classes).any(1)]``).  Sizes: a served YOLOv5 at img 416 has N = 10647
rows, at 608 N = 22743; with nc = 80 both B = 1 outputs hold an odd number of floats.
"""
import numpy as np
import pytest
import torch

from triton_client_amd.ops.yolo import YoloPostprocess

CLASSES = [0, 2, 5, 63]


def _pred(B, N, nc, seed=0):
    rng = np.random.default_rng(seed)
    p = np.zeros((B, N, nc + 5), np.float32)
    p[..., :2] = rng.uniform(0, 640, (B, N, 2))
    p[..., 2:4] = rng.uniform(4, 200, (B, N, 2))
    p[..., 4] = rng.beta(0.4, 4, (B, N))
    p[..., 5:] = rng.beta(0.5, 3, (B, N, nc))
    # rows whose best class is excluded but whose second-best allowed class clears the threshold
    p[..., 5 + 1] = np.maximum(p[..., 5 + 1], p[..., 5 + 2] + 0.05)
    hot = rng.uniform(size=(B, N)) < 0.2  # confident rows, top class drawn from {allowed, 1}
    p[..., 4] = np.where(hot, rng.uniform(0.6, 1.0, (B, N)), p[..., 4])
    top = rng.choice(np.array(CLASSES + [1]), size=(B, N))
    bi, ni = np.nonzero(hot)
    p[bi, ni, 5 + top[bi, ni]] = rng.uniform(0.7, 1.0, len(bi))
    return p


def _reference_order_rows(pred_b, conf_thres, classes):
    """Row indices, classes and scores the reference keeps before NMS (single label)."""
    x = pred_b[pred_b[:, 4] > conf_thres]
    rows = np.nonzero(pred_b[:, 4] > conf_thres)[0]
    conf_all = x[:, 5:] * x[:, 4:5]
    j = conf_all.argmax(1)
    conf = conf_all[np.arange(len(j)), j]
    sel = conf > conf_thres
    rows, j, conf = rows[sel], j[sel], conf[sel]
    keep = np.isin(j, classes)
    return rows[keep], j[keep], conf[keep]


def test_class_filter_drops_rows_whose_best_class_is_masked():
    pred = _pred(2, 4000, 80)
    post = YoloPostprocess(80, np.zeros((3, 3, 2), np.float32), conf_thres=0.3, iou_thres=1.01, max_det=4000,
                           classes=CLASSES, device="cpu")
    res = post.postprocess_decoded(pred)
    for b in range(2):
        rows, cls, conf = _reference_order_rows(pred[b], 0.3, CLASSES)
        # iou_thres > 1 keeps every candidate: the kept set is the pre-NMS set
        k = int(res.count[b])
        assert k == len(rows) > 5
        assert sorted(res.cls[b, :k].tolist()) == sorted(cls.tolist())
        np.testing.assert_allclose(np.sort(res.score[b, :k].numpy()), np.sort(conf.astype(np.float32)), rtol=1e-6)
    # the old behaviour (argmax among allowed classes only) would keep more rows here
    x = pred[0][pred[0][:, 4] > 0.3]
    cc = x[:, 5:] * x[:, 4:5]
    masked = np.where(np.isin(np.arange(80), CLASSES)[None], cc, -1.0)
    assert int((masked.max(1) > 0.3).sum()) > int(res.count[0])


@pytest.mark.gpu
def test_filter_decoded_class_order_gpu(cuda):
    pred = _pred(2, 4000, 80, seed=1)
    kw = dict(conf_thres=0.3, iou_thres=1.01, max_det=4000, classes=CLASSES)
    anchors = np.zeros((3, 3, 2), np.float32)
    c = YoloPostprocess(80, anchors, device="cpu", **kw).postprocess_decoded(pred)
    g = YoloPostprocess(80, anchors, device=cuda, **kw).filter_decoded(torch.from_numpy(pred).to(cuda))
    torch.cuda.synchronize()
    for b in range(2):
        rows, cls, _ = _reference_order_rows(pred[b], 0.3, CLASSES)
        k = int(g.count[b])
        assert k == int(c.count[b]) == len(rows)
        assert sorted(g.cls[b, :k].cpu().tolist()) == sorted(cls.tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("img", [416, 608])
def test_decode_odd_total_matches_cpu(cuda, img):
    from triton_client_amd.models.yolov5 import STRIDES
    torch.manual_seed(img)
    nc, na = 80, 3
    anchors = torch.tensor([[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119],
                            [116, 90, 156, 198, 373, 326]], dtype=torch.float32)
    post = YoloPostprocess(nc, anchors, (img, img), device=cuda)
    heads = [torch.randn(1, na * (nc + 5), img // s, img // s, device=cuda) * 3 for s in STRIDES]
    assert (post.num_anchors_total * (nc + 5)) % 4 != 0
    got = post.decode(heads)
    want = post.decode_cpu([h.cpu() for h in heads])
    torch.cuda.synchronize()
    assert got.shape == want.shape == (1, post.num_anchors_total, nc + 5)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-5, atol=1e-3)
