#!/usr/bin/env python3
"""SECOND-IoU pipeline probe: per-level sparse row counts and per-stage GPU
time (eager, CUDA events) on the bench's synthetic sweeps."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from triton_client_amd.ops.conv import NHWC  # noqa: E402
from triton_client_amd.ops.lidar import pc2_unpack  # noqa: E402
from triton_client_amd.pipelines import SecondPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda")
    spec = LidarSpec(rings=64, azimuth_steps=1875, sensor_height=3.23)
    maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
    p = SecondPipeline(batch=B, max_points=maxp, device=dev, z_offset=1.5)
    for b in range(B):
        c = lidar_sweep(spec, 500 + b % 8)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        p.data[b * p.frame_bytes:b * p.frame_bytes + raw.numel()].copy_(raw)
        p.frame_n[b] = c.shape[0]
    p.calibrate_detection_density(60.0)
    for _ in range(3):
        p.step()
    torch.cuda.synchronize()
    print("level rows:", p.sparse.level_rows(), "caps:", [lv.cap for lv in p.sparse.levels])
    print("sparse workspace GiB: %.2f" % (p.sparse.nbytes / 2**30))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
    names = ["unpack+vox+vfe", "sparse conv", "bev 2d", "proposals", "roi head"]
    tot = np.zeros(len(names))
    n = 10
    for _ in range(n):
        ev[0].record()
        pts, cnt = pc2_unpack(p.ws, p.data, p.frame_off, p.frame_n, p.layout, p.max_points, p.normalize, p.z_offset)
        p.sparse.reset()
        p.vox.assign(pts, cnt)
        p.sparse.encode_from_slots(pts, p.vox)
        p.vox.finish(pts, cnt, gather=False)
        ev[1].record()
        p.sparse.forward()
        ev[2].record()
        cls, box, dir_ = p.fast.forward(NHWC(p.sparse.bev))
        ev[3].record()
        props = p.prop(cls, box, dir_)
        ev[4].record()
        res = p.roi(p.fast.cat.t, props)
        ev[5].record()
        torch.cuda.synchronize()
        tot += [ev[i].elapsed_time(ev[i + 1]) for i in range(5)]
    for k, v in zip(names, tot / n):
        print(f"{k:16s} {v:8.3f} ms")
    print("total %.3f ms per %d sweeps; dets/frame %.1f" % (tot.sum() / n, B, res.count.float().mean().item()))


if __name__ == "__main__":
    main()
