"""fp32 fused BEV neck + head (K15) on the PointPillars KITTI shapes at the headline
batch: pair-storage branch inputs (the LiDAR pipeline's form), µs per call.  (The
tiling variants this tool compared were removed in round 4, after
profiles/r4/neck_variants.jsonl; variant 0 is the one tiling.)

    python tools/bench_neck.py [batch] [variants,comma,separated]
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from triton_client_amd.config.lidar import PointPillarsConfig  # noqa: E402
from triton_client_amd.models.common import fuse_model, randomize_bn  # noqa: E402
from triton_client_amd.models.fast import FastBEV  # noqa: E402
from triton_client_amd.models.pointpillars import build_pointpillars  # noqa: E402
from triton_client_amd.ops.conv import NHWC, to_pairs  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    dev = torch.device("cuda")
    m = build_pointpillars(PointPillarsConfig())
    randomize_bn(m, 3)
    m = fuse_model(m.eval())
    fb = FastBEV(m, B, device=dev, precision="fp32", pair=True)
    neck = fb.neck
    ny, nx = m.cfg.voxel.grid_size[1], m.cfg.voxel.grid_size[0]
    H, W = ny // 2, nx // 2
    g = torch.Generator().manual_seed(0)
    xs = [NHWC(to_pairs(torch.randn(B, H // s, W // s, c, generator=g)).to(dev), pair=True)
          for s, c in zip(neck.strides, (64, 128, 256))]
    res = {}
    outs = {}
    for v in variants:
        neck.variant = v
        out = NHWC(torch.empty(B, H, W, neck.nh, device=dev))
        for _ in range(3):
            neck(xs, out)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            neck(xs, out)
        torch.cuda.synchronize()
        res[v] = round((time.perf_counter() - t) / 10 * 1e6, 1)
        outs[v] = out.t.clone()
    ref = outs[variants[0]]
    same = {v: bool(torch.equal(o, ref)) for v, o in outs.items()}
    print(json.dumps({"batch": B, "H": H, "W": W, "us_by_variant": res, "bit_identical": same}))


if __name__ == "__main__":
    main()
