"""yolo_detect.hip (YOLOv5 Detect convs + decode + candidate filter in one kernel) against the
unfused chain it replaces (the plan's three 1x1 convs, then yolo.hip tca_yolo_decode_filter):
the logits are computed with the same split operands, K order and product order, so the
candidate sets must be identical, bit for bit."""
import pytest
import torch

from triton_client_amd.ops.yolo import YoloPostprocess
from triton_client_amd.pipelines import CameraPipeline
from triton_client_amd.utils.synthetic import camera_frame


def _cam(cuda, img_hw=(640, 640), B=2, density=80.0):
    c = CameraPipeline(batch=B, src_hw=(720, 1280), img_hw=img_hw, device=cuda)
    for b in range(B):
        c.frames[b].copy_(torch.from_numpy(camera_frame(720, 1280, 3 + b)))
    c.calibrate_detection_density(density)
    return c


def _sorted_cands(cand):
    out = []
    for b in range(cand.count.shape[0]):
        n = min(int(cand.count[b]), cand.key.shape[1])
        k = cand.key[b, :n]
        o = torch.argsort(k)
        out.append((k[o], cand.box[b, :n][o], cand.score[b, :n][o], cand.cls[b, :n][o]))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("img_hw", [(640, 640), (320, 416)])
@pytest.mark.parametrize("classes", [None, "common"])
def test_detect_fused_candidates_identical(cuda, img_hw, classes):
    c = _cam(cuda, img_hw)
    f = c.build_fast()
    if classes == "common":
        # a class filter drops rows whose best class is masked: filter on the classes the random-init
        # heads actually pick (every other one of the most frequent), so both kernels keep candidates
        p0 = YoloPostprocess(c.model.cfg.nc, c.model.anchors.cpu(), img_hw, 0.3, 0.45, 300, device=cuda)
        c.step()
        cand0, _ = p0._filter(f.forward(from_t1=True), False)
        cls0 = torch.cat([cand0.cls[b, :min(int(cand0.count[b]), cand0.cls.shape[1])] for b in range(2)])
        freq = torch.bincount(cls0.long(), minlength=c.model.cfg.nc)
        classes = torch.argsort(freq, descending=True)[:6:2].tolist()
    post = YoloPostprocess(c.model.cfg.nc, c.model.anchors.cpu(), img_hw, 0.3, 0.45, 300, device=cuda,
                           classes=classes)
    assert post.detect_fused_ok(f)
    c.step()  # fills the plan's buffers (o3 / o4 / o5 and the unfused head maps)
    feats = f.forward(from_t1=True, heads=False)
    heads = f.forward(from_t1=True)
    want, _ = post._filter(heads, False)
    want = _sorted_cands(want)
    post.detect_fused(f, feats)
    from triton_client_amd.ops.nms import Candidates
    got = _sorted_cands(Candidates.alloc(post.ws, "yolo_", 2, min(post.num_anchors_total, 1 << 20), 4))
    torch.cuda.synchronize()
    assert sum(int(w[0].numel()) for w in want) > 10
    for g, w in zip(got, want):
        for a, b in zip(g, w):
            assert torch.equal(a, b)


@pytest.mark.gpu
def test_camera_step_detect_fused_same_detections(cuda, monkeypatch):
    import triton_client_amd.models.fast as fast

    c = _cam(cuda, B=4, density=50.0)
    f = c.build_fast()
    assert c.post.detect_fused_ok(f)
    r1 = c.step()
    torch.cuda.synchronize()
    n1, b1, s1, k1 = r1.count.clone(), r1.box.clone(), r1.score.clone(), r1.cls.clone()
    monkeypatch.setattr(fast, "DETECT_FUSED", False)
    assert not c.post.detect_fused_ok(f)
    r2 = c.step()
    torch.cuda.synchronize()
    assert int(n1.min()) > 0 and torch.equal(n1, r2.count)
    for b in range(4):
        n = int(n1[b])
        assert torch.equal(b1[b, :n], r2.box[b, :n])
        assert torch.equal(s1[b, :n], r2.score[b, :n]) and torch.equal(k1[b, :n], r2.cls[b, :n])


@pytest.mark.gpu
def test_detect_fused_not_taken_for_multilabel(cuda):
    c = _cam(cuda, (320, 320), density=20.0)
    f = c.build_fast()
    post = YoloPostprocess(c.model.cfg.nc, c.model.anchors.cpu(), (320, 320), multi_label=True, device=cuda)
    assert not post.detect_fused_ok(f)
