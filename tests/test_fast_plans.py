"""Concat-free fast execution plans == the reference PyTorch modules
(CPU: fp32 buffers, same math; GPU: fp32 split-product and bf16 MFMA kernels
vs an fp64 evaluation, per-output relative-L2 bounds)."""
import dataclasses

import numpy as np
import pytest
import torch

from triton_client_amd.config.lidar import KITTI_PILLARS, PointPillarsConfig
from triton_client_amd.models.common import fuse_model, randomize_bn
from triton_client_amd.models.fast import FastBEV, FastYOLOv5
from triton_client_amd.models.pointpillars import build_pointpillars
from triton_client_amd.models.yolov5 import build_yolov5
from triton_client_amd.ops.conv import NHWC


def _yolo(img=64):
    m = build_yolov5("n", 80, img)
    randomize_bn(m, 1)
    return fuse_model(m.eval())


def test_fast_yolo_cpu_matches_module():
    m = _yolo(64)
    x = torch.rand(2, 3, 64, 64)
    with torch.no_grad():
        ref = m(x)
    f = FastYOLOv5(m, 2, (64, 64), device="cpu")
    f.set_input(x)
    with torch.no_grad():
        outs = f.forward()
    for r, o in zip(ref, outs):
        torch.testing.assert_close(o.nchw(), r, rtol=1e-4, atol=1e-4)


def _small_pp():
    v = dataclasses.replace(KITTI_PILLARS, point_cloud_range=(0.0, -10.24, -3.0, 10.24, 10.24, 1.0))
    cfg = PointPillarsConfig(voxel=v)
    m = build_pointpillars(cfg)
    randomize_bn(m, 2)
    return fuse_model(m.eval())


def test_fast_bev_cpu_matches_module():
    m = _small_pp()
    nx, ny, _ = m.cfg.voxel.grid_size
    canvas = torch.zeros(1, ny, nx, 64)
    canvas[:, ::3, ::2] = torch.rand(1, (ny + 2) // 3, (nx + 1) // 2, 64)
    with torch.no_grad():
        ref = m.bev_forward(canvas.permute(0, 3, 1, 2))
        f = FastBEV(m, 1, device="cpu")
        outs = f.forward(NHWC(canvas))
    for r, o in zip(ref, outs):
        torch.testing.assert_close(o.nchw(), r, rtol=1e-4, atol=1e-4)


def _rel_l2(got: torch.Tensor, ref: torch.Tensor) -> float:
    got, ref = got.double().cpu(), ref.double().cpu()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


# Per-output relative-L2 bounds against an fp64 evaluation of the same fused
# module.  fp32 mode (split-product MFMA, ~2^-17 relative per product, fp32
# activations): measured on MI355X 2e-7 (YOLOv5n heads) and 1.3e-5 (BEV box /
# direction heads); bound 2e-4.  bf16 mode: activations and weights rounded
# to 8 mantissa bits (2^-9 ~ 2e-3 relative) at every layer; measured 1.9e-3
# (YOLOv5n) and 7.3e-3 (BEV); bound 2e-2.  profiles/r2/round_check2_plans.txt.
PLAN_REL_L2 = {"fp32": 2e-4, "bf16": 2e-2}


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_fast_plans_gpu_vs_fp64_module(cuda, precision):
    dt = torch.float32 if precision == "fp32" else torch.bfloat16
    m = _yolo(128)
    x = torch.rand(2, 3, 128, 128)
    with torch.no_grad():
        ref = m.double()(x.double())
    f = FastYOLOv5(m.float(), 2, (128, 128), device=cuda, precision=precision)
    f.set_input(x.to(cuda))
    outs = f.forward()
    torch.cuda.synchronize()
    errs = [_rel_l2(o.nchw(), r) for r, o in zip(ref, outs)]
    print(precision, "yolo rel L2", errs)
    assert max(errs) < PLAN_REL_L2[precision], errs
    pm = _small_pp()
    nx, ny, _ = pm.cfg.voxel.grid_size
    canvas = torch.zeros(2, ny, nx, 64)
    canvas[:, ::3, ::2] = torch.rand(2, (ny + 2) // 3, (nx + 1) // 2, 64)
    with torch.no_grad():
        ref = pm.double().bev_forward(canvas.double().permute(0, 3, 1, 2))
    fb = FastBEV(pm.float(), 2, device=cuda, precision=precision)
    outs = fb.forward(NHWC(canvas.to(cuda, dt)))
    torch.cuda.synchronize()
    errs = [_rel_l2(o.nchw(), r) for r, o in zip(ref, outs)]
    print(precision, "bev rel L2", errs)
    assert max(errs) < PLAN_REL_L2[precision], errs
