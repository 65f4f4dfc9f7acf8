"""Stage-by-stage counts of the LiDAR pipeline at bench scale (debug aid)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from triton_client_amd.pipelines import GraphRunner, LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402


def main(B=16, graph=True):
    spec = LidarSpec(sensor_height=3.23)
    maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
    lid = LidarPipeline(batch=B, max_points=maxp, device="cuda", z_offset=1.5)
    for b in range(B):
        c = lidar_sweep(spec, 500 + b % 8)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    d = lid.calibrate_detection_density(2000.0)
    print("shift", d)
    fn = GraphRunner(lid.step) if graph else lid.step
    for it in range(3):
        r = fn()
        torch.cuda.synchronize()
        ws = lid.post.ws
        print(it, "pts", lid.ws.get("pc2_count", (B,), torch.int32).cpu().tolist()[:4],
              "vox", lid.vox.voxel_count.cpu().tolist()[:4],
              "cand", ws.get("anc_count", (B,), torch.int32).cpu().tolist()[:4],
              "sorted", ws.get("anc_nms_nsorted", (B,), torch.int32).cpu().tolist()[:4],
              "out", r.count.cpu().tolist()[:4])
        with torch.no_grad():
            cls, _, _ = lid.model.bev_forward(lid.enc.canvas_nchw())
        m = cls.float().permute(0, 2, 3, 1).reshape(B, -1, 3).max(-1).values
        print("   eager-recount >= thr:", (torch.sigmoid(m) >= 0.1).sum(1).cpu().tolist()[:4],
              "canvas nonzero", int((lid.enc.canvas != 0).any(-1).sum()))


if __name__ == "__main__":
    main(graph="--eager" not in sys.argv)
