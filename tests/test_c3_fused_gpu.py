"""c3_fused.hip (YOLOv5 C3 blocks with c_ = 32 / 64 as LDS-resident kernels: FULL for one
bottleneck, FIRST / MID / LAST for two or three) against the unfused _C3Plan chain of
fused 1x1 / 3x3 convs it replaces: the same split operands in the same K order, so the
block outputs agree to fp32 rounding; and the camera step's detections are unchanged."""
import pytest
import torch

from triton_client_amd.ops.conv import NHWC
from triton_client_amd.pipelines import CameraPipeline
from triton_client_amd.utils.synthetic import camera_frame

# YOLOv5n's C3 blocks with c_ = 16 / 32 / 64 (b2: c_ 16; b4: two bottlenecks, b6: three; the head
# C3s: one, no shortcut)
BLOCKS = ["b2", "b4", "b6", "h13", "h17", "h20"]


@pytest.fixture(scope="module")
def cam(cuda):
    c = CameraPipeline(batch=2, src_hw=(64, 64), img_hw=(64, 64), device=cuda)
    c.build_fast()
    return c


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [(20, 20), (23, 37), (9, 50)])
@pytest.mark.parametrize("name", BLOCKS)
def test_c3_fused_matches_chain(cuda, cam, monkeypatch, name, hw):
    import triton_client_amd.models.fast as fast

    torch.manual_seed(hw[0] * 7 + len(name))
    B, (H, W) = 2, hw
    blk = getattr(cam.model, name)
    plan = fast._C3Plan(blk, B, H, W, fast._Buffers(cuda, "fp32"), cuda)
    cin, cout = plan.cv12.cin_p, plan.cv3.N
    x = NHWC(torch.randn(B, H, W, cin + 8, device=cuda) * 2, 8, cin)  # channel-offset input slice
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(fast, "C3_FUSED", fused)
        out = NHWC(torch.full((B, H, W, cout + 16), 7.0, device=cuda), 8, cout)
        assert plan.fused2_ok(x, out) == fused
        plan(x, out)
        torch.cuda.synchronize()
        assert (out.t[..., :8] == 7.0).all() and (out.t[..., 8 + cout:] == 7.0).all()
        outs.append(out.t[..., 8:8 + cout].double())
    got, want = outs
    assert torch.isfinite(got).all()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 1e-6, rel
    assert (got - want).abs().max().item() <= 1e-4 * want.abs().max().item()


@pytest.mark.gpu
def test_camera_step_fused_c3_same_detections(cuda, monkeypatch):
    import triton_client_amd.models.fast as fast

    c = CameraPipeline(batch=4, src_hw=(720, 1280), device=cuda)
    for b in range(4):
        c.frames[b].copy_(torch.from_numpy(camera_frame(720, 1280, b)))
    c.calibrate_detection_density(50.0)
    f = c.build_fast()
    assert all(p._fw is not None for p in (f.c3_2, f.c3_4, f.c3_6, f.c3_13, f.c3_17, f.c3_20))
    assert f.c3_8._fw is None and f.c3_23._fw is None  # c_ = 128: the chain
    r1 = c.step()
    torch.cuda.synchronize()
    n1, b1 = r1.count.clone(), r1.box.clone()
    monkeypatch.setattr(fast, "C3_FUSED", False)
    r2 = c.step()
    torch.cuda.synchronize()
    assert torch.equal(n1, r2.count)
    for b in range(4):
        n = int(n1[b])
        assert torch.allclose(b1[b, :n], r2.box[b, :n], atol=1e-3)
