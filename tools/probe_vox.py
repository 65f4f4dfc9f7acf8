"""Points-per-pillar distribution of the bench's synthetic sweeps (drives the
voxeliser insert design: the atomicMin carry chain costs O(points x slots) in
dense pillars)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from triton_client_amd.pipelines import LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402


def main():
    dev = torch.device("cuda")
    B = 16
    spec = LidarSpec(rings=64, azimuth_steps=1875, sensor_height=3.23)
    maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
    lid = LidarPipeline(batch=B, max_points=maxp, device=dev, z_offset=1.5)
    fb = lid.frame_bytes
    for b in range(B):
        c = lidar_sweep(spec, 500 + b)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * fb:b * fb + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    from triton_client_amd.ops.lidar import pc2_unpack
    pts, cnt = pc2_unpack(lid.ws, lid.data, lid.frame_off, lid.frame_n, lid.layout, lid.max_points, lid.normalize,
                          lid.z_offset)
    lid.vox.assign(pts, cnt)
    torch.cuda.synchronize()
    out = {}
    allc = []
    for b in range(B):
        nv = int(lid.vox.voxel_count[b].item())
        allc.append(lid.vox.vcount[b, :nv].cpu().numpy())
    c = np.concatenate(allc)
    out.update({"pillars_per_frame": float(len(c) / B), "points_per_frame": float(c.sum() / B),
                "pct_points_in_pillars_gt32": float(c[c > 32].sum() / c.sum()), "pillars_gt32": int((c > 32).sum()),
                "max": int(c.max()), "p50": float(np.percentile(c, 50)), "p90": float(np.percentile(c, 90)),
                "p99": float(np.percentile(c, 99)), "sum_sq": float((c.astype(np.float64) ** 2).sum() / B)})
    lid.vox.finish(pts, cnt, gather=False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
