#!/usr/bin/env python3
"""Host-side cost of replaying the camera / LiDAR step graphs (split mode),
and where each branch starts on the GPU when launched in either order."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from triton_client_amd.pipelines import CameraPipeline, GraphRunner, LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep  # noqa: E402

dev = torch.device("cuda")
B = 16
cam = CameraPipeline(batch=B, src_hw=(720, 1280), device=dev)
spec = LidarSpec(rings=64, azimuth_steps=1875, sensor_height=3.23)
mp = ((spec.points_per_sweep + 1023) // 1024) * 1024
lid = LidarPipeline(batch=B, max_points=mp, device=dev, z_offset=1.5)
for b in range(B):
    cam.frames[b].copy_(torch.from_numpy(camera_frame(720, 1280, b)))
    c = lidar_sweep(spec, b)
    raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
    lid.data[b * lid.frame_bytes:b * lid.frame_bytes + raw.numel()].copy_(raw)
    lid.frame_n[b] = c.shape[0]
cam.calibrate_detection_density(100.0)
lid.calibrate_detection_density(2000.0)
cr, lr = GraphRunner(cam.step), GraphRunner(lid.step)
cr(); lr(); torch.cuda.synchronize()
side = torch.cuda.Stream()
for order in ("lid_first", "cam_first"):
    host = {"lid": [], "cam": []}
    ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for k in ("lid", "cam")}
    spans = []
    for it in range(20):
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        side.wait_stream(torch.cuda.current_stream())
        seq = ["lid", "cam"] if order == "lid_first" else ["cam", "lid"]
        for k in seq:
            s = side if k == "lid" else torch.cuda.current_stream()
            with torch.cuda.stream(s):
                ev[k][0].record()
                t = time.perf_counter()
                (lr if k == "lid" else cr)()
                host[k].append((time.perf_counter() - t) * 1e6)
                ev[k][1].record()
        torch.cuda.current_stream().wait_stream(side)
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        torch.cuda.synchronize()
        spans.append((start.elapsed_time(ev["lid"][0]), start.elapsed_time(ev["lid"][1]),
                      start.elapsed_time(ev["cam"][0]), start.elapsed_time(ev["cam"][1]), start.elapsed_time(end)))
    sp = np.median(np.array(spans[5:]), 0)
    print(f"{order}: host replay us lid {np.median(host['lid'][5:]):.0f} cam {np.median(host['cam'][5:]):.0f}; "
          f"GPU ms: lid {sp[0]:.3f}->{sp[1]:.3f} cam {sp[2]:.3f}->{sp[3]:.3f} total {sp[4]:.3f}")
