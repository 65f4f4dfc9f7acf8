"""Fused MFMA NHWC conv vs PyTorch/MIOpen (conv + bias + act) on the
detectors' real layer shapes, batch 16, bf16.  Prints one JSON line per shape."""
import json
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, ".")
from triton_client_amd.ops.conv import NHWC, FusedConv  # noqa: E402

SHAPES = [
    # name, B, H, W, cin, cout, k, s, act   (PointPillars KITTI 496x432 canvas, then YOLOv5n @640)
    ("pp.b1.down", 16, 496, 432, 64, 64, 3, 2, 1),
    ("pp.b1.conv", 16, 248, 216, 64, 64, 3, 1, 1),
    ("pp.b2.down", 16, 248, 216, 64, 128, 3, 2, 1),
    ("pp.b2.conv", 16, 124, 108, 128, 128, 3, 1, 1),
    ("pp.b3.down", 16, 124, 108, 128, 256, 3, 2, 1),
    ("pp.b3.conv", 16, 62, 54, 256, 256, 3, 1, 1),
    ("pp.head", 16, 248, 216, 384, 72, 1, 1, 0),
    ("pp.de1", 16, 248, 216, 64, 128, 1, 1, 1),
    ("y.stem_s2d", 16, 320, 320, 16, 16, 3, 1, 2),
    ("y.b1", 16, 320, 320, 16, 32, 3, 2, 2),
    ("y.c3.3x3", 16, 160, 160, 16, 16, 3, 1, 2),
    ("y.b3", 16, 160, 160, 32, 64, 3, 2, 2),
    ("y.c3.1x1", 16, 80, 80, 64, 32, 1, 1, 2),
    ("y.b5", 16, 80, 80, 64, 128, 3, 2, 2),
    ("y.b7", 16, 40, 40, 128, 256, 3, 2, 2),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    dev = torch.device("cuda")
    tiles = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 5, 6, 7, 20, 22, 24, 25, 31, 41, 42]
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for name, B, H, W, ci, co, k, s, act in SHAPES:
        if only and not any(name.startswith(o) for o in only):
            continue
        conv = nn.Conv2d(ci, co, k, s, k // 2, bias=True).to(dev)
        fc = FusedConv(conv, act=act, device=dev)
        x = torch.randn(B, H, W, ci, device=dev, dtype=torch.bfloat16)
        xin = NHWC(x)
        out = fc(xin)
        cm = conv.to(torch.bfloat16).to(memory_format=torch.channels_last)
        xc = x.permute(0, 3, 1, 2)
        actf = {0: lambda t: t, 1: F.relu, 2: F.silu}[act]
        ref = actf(cm(xc))
        err = (out.nchw().float() - ref.float()).abs().max().item()
        scale = ref.float().abs().max().item()
        Ho, Wo = out.shape[1], out.shape[2]
        flops = 2.0 * B * Ho * Wo * co * ci * k * k
        t_ref = timeit(lambda: actf(cm(xc)))
        best = None
        res = {}
        for t in tiles:
            try:
                us = timeit(lambda: fc(xin, out=out, tile=t))
            except Exception as e:  # noqa
                continue
            fc(xin, out=out, tile=t)
            e_t = (out.nchw().float() - ref.float()).abs().max().item()
            if e_t > 0.05 * max(scale, 1.0):
                res[t] = f"WRONG err={e_t:.3g} {us:.1f}us"
                continue
            res[t] = round(us, 1)
            if best is None or us < best[1]:
                best = (t, us)
        if best is None:
            print(json.dumps({"layer": name, "miopen_us": round(t_ref, 1), "fused_us_by_tile": res}), flush=True)
            continue
        print(json.dumps({"layer": name, "miopen_us": round(t_ref, 1), "fused_us_by_tile": res,
                          "best_tile": best[0], "speedup": round(t_ref / best[1], 2),
                          "fused_tflops": round(flops / best[1] / 1e6, 1), "max_err": err, "ref_scale": scale}),
              flush=True)


if __name__ == "__main__":
    main()
