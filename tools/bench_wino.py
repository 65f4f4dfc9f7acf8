#!/usr/bin/env python3
"""hx3 (direct, conv_hx3.hip) vs wino (F(2,3), conv_wino.hip) on the PointPillars backbone's
stride-1 layer shapes at batch 32 (pair storage in and out, ReLU): us per call, TFLOP/s of the
direct conv's work (x3 split products), one JSON line per shape."""
import copy
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from triton_client_amd.ops.conv import NHWC, FusedConv, to_pairs  # noqa: E402


def main():
    dev = torch.device("cuda")
    B = int(os.environ.get("B", 32))
    shapes = [(248, 216, 64), (124, 108, 128), (62, 54, 256)]
    only = os.environ.get("SHAPE")  # e.g. SHAPE=1: the 128-channel layer only
    tiles = [int(t) for t in os.environ.get("TILES", "110,130,131,132,133,134").split(",")]
    for (H, W, c) in ([shapes[int(only)]] if only else shapes):
        torch.manual_seed(0)
        conv = nn.Conv2d(c, c, 3, 1, 1, bias=True)
        fc = FusedConv(copy.deepcopy(conv), act=1, device=dev, precision="fp32")
        xr = torch.relu(torch.randn(B, H, W, c))
        x = NHWC(to_pairs(xr).to(dev), pair=True)
        x32 = NHWC(xr.to(dev), pair=False)  # fp32 storage (the chain inside a block)
        o32 = NHWC(torch.empty(B, H, W, c, device=dev), pair=False)
        outs = {t: NHWC(torch.empty(B, H, W, c, device=dev), pair=True) for t in (110, 130)}
        if os.environ.get("F32"):  # fp32 storage in and out for every wino tile (PMC runs)
            x, outs[130] = x32, o32
        res = {"shape": [B, H, W, c]}
        for t in tiles:
            if t in (131, 132) and c % 128:
                continue
            o = outs[110 if t == 110 else 130]
            for _ in range(3):
                fc(x, out=o, tile=t)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                fc(x, out=o, tile=t)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            flops = 2.0 * B * H * W * c * c * 9 * 3
            res[str(t)] = {"us": round(us, 1), "tflops_x3": round(flops / us / 1e6, 1)}
            if t == 130:  # fp32 storage in and out
                for _ in range(3):
                    fc(x32, out=o32, tile=t)
                e0.record()
                for _ in range(n):
                    fc(x32, out=o32, tile=t)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / n
                res["130_fp32io"] = {"us": round(us, 1), "tflops_x3": round(flops / us / 1e6, 1)}
        if 110 in tiles and any(t >= 130 for t in tiles):
            d = (outs[110].nchw() - outs[130].nchw()).norm() / outs[110].nchw().norm()
            res["rel_l2_wino_vs_hx3"] = float(d)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
