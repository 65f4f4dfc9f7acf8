"""Standalone time of the PillarVFE + scatter kernel on the headline's LiDAR batch (32 synthetic
64 x 1875 sweeps, bench.py's data), with the pillar statistics that size its work.

Each rep runs the voxeliser front (clear, assign), then the VFE between two HIP events, then the
voxeliser's finish, so the VFE always reads a fresh slot table; only the VFE is timed.

    python tools/bench_vfe.py [--reps 20] [--variant lin|mfma|lin2]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--variant", choices=("lin", "mfma", "lin2"), default="lin")
    a = ap.parse_args()

    import torch

    from triton_client_amd import _native
    from triton_client_amd.ops.lidar import pc2_unpack
    from triton_client_amd.pipelines.lidar import LidarPipeline
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep

    dev = torch.device("cuda")
    spec = LidarSpec(rings=64, azimuth_steps=1875, sensor_height=3.23)
    max_points = ((spec.points_per_sweep + 1023) // 1024) * 1024
    B = a.batch
    lid = LidarPipeline(batch=B, max_points=max_points, device=dev, z_offset=1.5, precision="fp32")
    fb = lid.frame_bytes
    host = torch.zeros(B * fb, dtype=torch.uint8)
    n = torch.zeros(B, dtype=torch.int32)
    for b in range(B):
        c = lidar_sweep(spec, 500 + b % 8)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        host[b * fb:b * fb + raw.numel()].copy_(raw)
        n[b] = c.shape[0]
    lid.data.copy_(host)
    lid.frame_n.copy_(n)
    lid.build_fast()
    _native.call("tca_pillar_vfe_set_variant", {"lin": 0, "mfma": 1, "lin2": 2}[a.variant])
    enc, vox = lid.enc, lid.vox
    times = []
    for i in range(a.reps + 3):
        pts, cnt = pc2_unpack(lid.ws, lid.data, lid.frame_off, lid.frame_n, lid.layout, lid.max_points,
                              lid.normalize, lid.z_offset)
        enc.clear(vox)
        vox.assign(pts, cnt)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        enc.encode_from_slots(pts, vox)
        e1.record()
        if i == 0:
            torch.cuda.synchronize()
            vc = vox.voxel_count.cpu().numpy()
            per = [vox.vcount[b, :vc[b]].cpu().numpy() for b in range(B)]
        vox.finish(pts, cnt, gather=False)
        torch.cuda.synchronize()
        if i >= 3:
            times.append(e0.elapsed_time(e1) * 1e3)
    allp = np.concatenate(per)
    P = lid.cfg.voxel.max_points_per_voxel
    out = {"variant": a.variant, "batch": B, "us_median": round(float(np.median(times)), 1),
           "us_min": round(float(np.min(times)), 1), "pillars_per_frame": round(float(vc.mean()), 1),
           "pillars_total": int(vc.sum()), "points_per_pillar_mean": round(float(np.minimum(allp, P).mean()), 2),
           "points_per_pillar_p90": float(np.percentile(np.minimum(allp, P), 90)),
           "full_pillars_frac": round(float((allp >= P).mean()), 3), "max_voxels": lid.cfg.voxel.max_voxels}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
