"""The PointPillars first conv (3x3 stride 2 over the sparse pillar canvas, occupancy-gated reads)
at the headline shape on the bench's synthetic sweeps: µs per stride-2 tile (ops/conv.py
HX3S2_TILES), with the real canvas and its occupancy.

    python tools/bench_s2_occ.py [tiles,comma,separated]
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from triton_client_amd.ops.conv import NHWC  # noqa: E402
from triton_client_amd.pipelines import LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402

tiles = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [120, 123, 124, 125, 126]
B = 32
spec = LidarSpec(sensor_height=3.23)  # bench.py's mounting
lid = LidarPipeline(batch=B, max_points=(spec.points_per_sweep + 1023) // 1024 * 1024, device="cuda")
for b in range(B):
    c = lidar_sweep(spec, b % 8)
    raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
    lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
    lid.frame_n[b] = c.shape[0]
f = lid.build_fast()
lid.step_pre()
canvas = lid.enc.canvas_nhwc()
convs, pp, H, W = f.bb.blocks[0]
cv = convs[0]
ref = None
for t in tiles:
    out = NHWC(torch.empty_like(pp[0].t), pair=True)
    try:
        cv(canvas, out=out, tile=t)
    except Exception as e:  # noqa: BLE001 - a tile that does not take this shape
        print(json.dumps({"tile": t, "error": str(e)[:80]}), flush=True)
        continue
    torch.cuda.synchronize()
    same = None
    if ref is None:
        ref = out.t.clone()
    else:
        same = bool(torch.equal(out.t.view(torch.int32), ref.view(torch.int32)))
    for _ in range(3):
        cv(canvas, out=out, tile=t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 20
    for _ in range(n):
        cv(canvas, out=out, tile=t)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    print(json.dumps({"layer": "pp.b1.down", "tile": t, "us": round(us, 1), "same_as_first": same,
                      "occupied_cells": int(canvas.occ.sum())}), flush=True)
