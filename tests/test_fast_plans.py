"""Concat-free fast execution plans == the reference PyTorch modules
(CPU: fp32 buffers, same math; GPU: bf16 MFMA kernels vs fp32)."""
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


@pytest.mark.gpu
def test_fast_plans_gpu_vs_fp32(cuda):
    m = _yolo(128)
    x = torch.rand(2, 3, 128, 128)
    with torch.no_grad():
        ref = m(x)
    f = FastYOLOv5(m, 2, (128, 128), device=cuda)
    f.set_input(x.to(cuda))
    outs = f.forward()
    torch.cuda.synchronize()
    for r, o in zip(ref, outs):
        err = (o.nchw().float().cpu() - r).abs().max().item()
        assert err < 0.1 * max(1.0, r.abs().max().item()), err
    pm = _small_pp()
    nx, ny, _ = pm.cfg.voxel.grid_size
    canvas = torch.zeros(2, ny, nx, 64)
    canvas[:, ::3, ::2] = torch.rand(2, (ny + 2) // 3, (nx + 1) // 2, 64)
    with torch.no_grad():
        ref = pm.bev_forward(canvas.permute(0, 3, 1, 2))
    fb = FastBEV(pm, 2, device=cuda)
    outs = fb.forward(NHWC(canvas.to(cuda, torch.bfloat16)))
    torch.cuda.synchronize()
    for r, o in zip(ref, outs):
        err = (o.nchw().float().cpu() - r).abs().max().item()
        assert err < 0.1 * max(1.0, r.abs().max().item()), err
