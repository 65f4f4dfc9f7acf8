"""Run one fused-conv layer shape / tile a few times (a target for rocprofv3 --pmc).

    python tools/conv_once.py <layer> <tile> <precision fp32|bf16|fp32p> [iters] [batch]
layer names as in tools/bench_conv_x3.py; fp32p = fp32 mode with pair-storage
input and output."""
import sys

import torch
import torch.nn as nn

sys.path.insert(0, ".")
from triton_client_amd.ops.conv import NHWC, FusedConv, to_pairs  # noqa: E402
from tools.bench_conv_x3 import SHAPES  # noqa: E402


def main():
    name, tile, prec = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    shp = next(s for s in SHAPES if s[0] == name)
    _, b, H, W, ci, co, k, s, act = shp
    if len(sys.argv) > 5:
        b = int(sys.argv[5])
    dev = torch.device("cuda")
    pair = prec == "fp32p"
    conv = nn.Conv2d(ci, co, k, s, k // 2, bias=True).to(dev)
    fc = FusedConv(conv, act=act, device=dev, precision="fp32" if pair else prec)
    x = torch.randn(b, H, W, ci, device=dev, dtype=fc.dtype)
    xin = NHWC(to_pairs(x), pair=True) if pair else NHWC(x)
    out = fc(xin, out=NHWC(torch.empty(b, *fc.out_hw(H, W), fc.N, device=dev, dtype=fc.dtype), pair=pair),
             tile=tile)
    for _ in range(iters):
        fc(xin, out=out, tile=tile)
    torch.cuda.synchronize()
    print("done", name, tile, prec)


if __name__ == "__main__":
    main()
