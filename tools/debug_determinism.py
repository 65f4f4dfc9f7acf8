"""Run the LiDAR pipeline twice on the same input; report the first stage whose
buffers differ (debug aid for replay determinism)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from triton_client_amd.ops.lidar import pc2_unpack  # noqa: E402
from triton_client_amd.ops.conv import NHWC  # noqa: E402
from triton_client_amd.pipelines import LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402


def snap(lid):
    ws = lid.post.ws
    d = {"pts": lid.ws.get("pc2_points", (lid.B, lid.max_points, 4), torch.float32).clone(),
         "coords": lid.vox.coords.clone(), "vcount_vox": lid.vox.voxel_count.clone(),
         "canvas": lid.enc.canvas.clone(), "hout": lid.fast.hout.t.clone(),
         "cand_count": ws.get("anc_count", (lid.B,), torch.int32).clone(),
         "order": ws.get("anc_nms_order", (lid.B, 4096), torch.int32).clone(),
         "out_box": ws.get("anc_nms_out_box", (lid.B, 500, 7), torch.float32).clone(),
         "out_count": ws.get("anc_nms_out_count", (lid.B,), torch.int32).clone()}
    for i, (convs, pp, H, W) in enumerate(lid.fast.blocks):
        d[f"blk{i}"] = pp[(len(convs) - 1) % 2].t.clone()
    d["cat"] = lid.fast.cat.t.clone()
    return d


def main():
    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    lid = LidarPipeline(batch=2, max_points=32768, device="cuda")
    for b, s in enumerate((3, 4)):
        c = lidar_sweep(spec, s)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    lid.calibrate_detection_density(500.0)
    lid.step()
    torch.cuda.synchronize()
    a = snap(lid)
    lid.step()
    torch.cuda.synchronize()
    b = snap(lid)
    report(a, b, "eager")
    from triton_client_amd.pipelines import GraphRunner
    g = GraphRunner(lid.step)
    g()
    torch.cuda.synchronize()
    c = snap(lid)
    report(a, c, "eager-vs-replay1")
    g()
    torch.cuda.synchronize()
    d = snap(lid)
    report(c, d, "replay1-vs-replay2")
    lid.step()
    torch.cuda.synchronize()
    report(a, snap(lid), "eager-after-graph")


def report(a, b, tag):
    print("==", tag)
    for k in a:
        x, y = a[k], b[k]
        same = torch.equal(x, y)
        extra = ""
        if not same and x.is_floating_point() or (not same and x.dtype == torch.bfloat16):
            extra = f" maxdiff {(x.float() - y.float()).abs().max().item():.3g} ndiff {(x != y).sum().item()}"
        elif not same:
            extra = f" ndiff {(x != y).sum().item()}"
        print(f"{k:12s} identical={same}{extra}", flush=True)


if __name__ == "__main__":
    main()
