"""fp32-mode fused conv (split-product MFMA) tiles vs MIOpen fp32 on the
detectors' layer shapes at the headline batch (32).  One JSON line per shape:
µs per tile, useful fp32 TFLOP/s, and the bf16-MFMA utilisation the 3 split
products imply (3 x FLOPs / 2.5 PF).

    python tools/bench_conv_x3.py [tiles,comma,separated] [layer-prefixes] [--pair]

--pair: input and output in pair storage (ops/conv.py to_pairs), the BEV
chain's fp32-mode format.
"""
import json
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, ".")
from triton_client_amd.ops.conv import NHWC, FusedConv, to_pairs  # noqa: E402

PAIR = "--pair" in sys.argv
if PAIR:
    sys.argv.remove("--pair")

B = 32
SHAPES = [
    ("pp.b1.down", B, 496, 432, 64, 64, 3, 2, 1),
    ("pp.b1.conv", B, 248, 216, 64, 64, 3, 1, 1),
    ("pp.b2.down", B, 248, 216, 64, 128, 3, 2, 1),
    ("pp.b2.conv", B, 124, 108, 128, 128, 3, 1, 1),
    ("pp.b3.down", B, 124, 108, 128, 256, 3, 2, 1),
    ("pp.b3.conv", B, 62, 54, 256, 256, 3, 1, 1),
    ("y.stem_s2d", B, 320, 320, 16, 16, 3, 1, 2),
    ("y.b1", B, 320, 320, 16, 32, 3, 2, 2),
    ("y.c3.3x3", B, 160, 160, 16, 16, 3, 1, 2),
    ("y.b3", B, 160, 160, 32, 64, 3, 2, 2),
    ("y.c3b.1x1", B, 80, 80, 64, 32, 1, 1, 2),
    ("y.c3b.3x3", B, 80, 80, 32, 32, 3, 1, 2),
    ("y.b5", B, 80, 80, 64, 128, 3, 2, 2),
    ("y.c3c.1x1", B, 40, 40, 128, 64, 1, 1, 2),
    ("y.c3c.3x3", B, 40, 40, 64, 64, 3, 1, 2),
    ("y.b7", B, 40, 40, 128, 256, 3, 2, 2),
    # the c_ = 128 C3 blocks (b8 / h23, unfused) and the SPPF / neck 1x1s at 20 x 20, the PAN downsamples
    ("y.c3d.cv12", B, 20, 20, 256, 256, 1, 1, 2),
    ("y.c3d.m1", B, 20, 20, 128, 128, 1, 1, 2),
    ("y.c3d.m2", B, 20, 20, 128, 128, 3, 1, 2),
    ("y.sp1", B, 20, 20, 256, 128, 1, 1, 2),
    ("y.sp2", B, 20, 20, 512, 256, 1, 1, 2),
    ("y.h19", B, 80, 80, 64, 64, 3, 2, 2),
    ("y.h22", B, 40, 40, 128, 128, 3, 2, 2),
    # Detect heads (1x1, 255 -> 256 outputs, no activation): short K, output-write bound
    ("y.det80", B, 80, 80, 64, 256, 1, 1, 0),
    ("y.det40", B, 40, 40, 128, 256, 1, 1, 0),
    ("y.det20", B, 20, 20, 256, 256, 1, 1, 0),
]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    dev = torch.device("cuda")
    tiles = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 and sys.argv[1] else [0]
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for name, b, H, W, ci, co, k, s, act in SHAPES:
        if only and not any(name.startswith(o) for o in only):
            continue
        torch.manual_seed(0)
        conv = nn.Conv2d(ci, co, k, s, k // 2, bias=True).to(dev)
        fc = FusedConv(conv, act=act, device=dev, precision="fp32")
        x = torch.randn(b, H, W, ci, device=dev)
        xin = NHWC(to_pairs(x), pair=True) if PAIR else NHWC(x)
        out = fc(xin, out=NHWC(torch.empty(b, *fc.out_hw(H, W), fc.N, device=dev), pair=PAIR))
        cm = conv.to(memory_format=torch.channels_last)
        xc = x.permute(0, 3, 1, 2)
        actf = {0: lambda t: t, 1: F.relu, 2: F.silu}[act]
        with torch.no_grad():
            ref = actf(cm(xc))
            t_ref = timeit(lambda: actf(cm(xc)))
        Ho, Wo = out.shape[1], out.shape[2]
        flops = 2.0 * b * Ho * Wo * co * ci * k * k
        res, best = {}, None
        for t in tiles:
            try:
                us = timeit(lambda: fc(xin, out=out, tile=t))
            except Exception:  # noqa: BLE001  (tile outside the shape's contract)
                continue
            fc(xin, out=out, tile=t)
            e = ((out.nchw() - ref).norm() / ref.norm()).item()
            if e > 1e-4:
                res[t] = f"WRONG rel={e:.3g} {us:.1f}us"
                continue
            res[t] = round(us, 1)
            if best is None or us < best[1]:
                best = (t, us, e)
        line = {"layer": name, "batch": b, "miopen_fp32_us": round(t_ref, 1), "us_by_tile": res}
        if best:
            line.update(best_tile=best[0], best_us=round(best[1], 1), rel_l2=float(f"{best[2]:.2e}"),
                        fp32_tflops=round(flops / best[1] / 1e6, 1),
                        bf16_mfma_util=round(3 * flops / best[1] / 1e6 / 2500, 3),
                        speedup_vs_miopen=round(t_ref / best[1], 2))
        print(json.dumps(line), flush=True)
        del x, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
