"""Fused K1 + YOLOv5 s2d stem + b1 (csrc/kernels/image.hip yolo_stem_fused_kernel) against the
three-kernel chain it replaces (prep_s2d -> conv_small_halo_x3 -> conv_nhwc_x3): the same
fp32 values are split into the same hi / lo operands and summed in the same K-step order,
so b1's output agrees to fp32 rounding; and the camera step's detections are unchanged."""
import pytest
import torch

from triton_client_amd.ops.conv import NHWC
from triton_client_amd.ops.image import preprocess, yolo_stem_fused
from triton_client_amd.pipelines import CameraPipeline
from triton_client_amd.utils.synthetic import camera_frame


def _pipe(cuda, B, src_hw, img_hw, swap_rb=False):
    cam = CameraPipeline(batch=B, src_hw=src_hw, img_hw=img_hw, device=cuda, swap_rb=swap_rb)
    for b in range(B):
        cam.frames[b].copy_(torch.from_numpy(camera_frame(*src_hw, b)))
    return cam


@pytest.mark.gpu
@pytest.mark.parametrize("src_hw,img_hw,swap", [((720, 1280), (640, 640), False), ((480, 640), (320, 416), True),
                                                 ((375, 1242), (384, 1248), False)])
def test_stem_fused_matches_chain(cuda, src_hw, img_hw, swap):
    B = 3
    cam = _pipe(cuda, B, src_hw, img_hw, swap)
    f = cam.build_fast()
    assert f.stem_fused_ok()
    preprocess(cam.frames, img_hw, cam.mode, "COCO", f.x.t.dtype, "S2D", swap_rb=swap, out=f.x.t)
    t0 = f.b0(f.x, out=f.t0)
    ref = f.b1(t0, out=NHWC(torch.empty_like(f.t1.t)))
    f.t1.t.fill_(float("nan"))
    yolo_stem_fused(cam.frames, img_hw, cam.mode, f.b0, f.b1, f.t1, "COCO", swap_rb=swap)
    torch.cuda.synchronize()
    got, want = f.t1.t.double(), ref.t.double()
    assert torch.isfinite(got).all()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 1e-6, rel
    assert (got - want).abs().max().item() <= 1e-4 * want.abs().max().item()


@pytest.mark.gpu
def test_camera_step_fused_stem_same_detections(cuda, monkeypatch):
    cam = _pipe(cuda, 4, (720, 1280), (640, 640))
    cam.calibrate_detection_density(50.0)
    f = cam.build_fast()
    r1 = cam.step()
    torch.cuda.synchronize()
    n1, b1 = r1.count.clone(), r1.box.clone()
    monkeypatch.setattr(type(f), "stem_fused_ok", lambda self: False)
    r2 = cam.step()
    torch.cuda.synchronize()
    assert torch.equal(n1, r2.count)
    for b in range(4):
        n = int(n1[b])
        assert torch.allclose(b1[b, :n], r2.box[b, :n], atol=1e-3)
