"""hx3 numerics probe: single-tap weights, chunk counts, tiles -> relative error table."""
import sys

import torch
import torch.nn as nn

sys.path.insert(0, ".")
from triton_client_amd.ops.conv import NHWC, FusedConv, to_pairs  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
for cin, cout in ((32, 128), (64, 128), (32, 64)):
    B, H, W = 1, 8, 16
    x = torch.randn(B, H, W, cin)
    for tap in list(range(9)) + ["all"]:
        conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
        with torch.no_grad():
            if tap != "all":
                m = torch.zeros(3, 3)
                m[tap // 3, tap % 3] = 1
                conv.weight.mul_(m)
        fc = FusedConv(conv, act=0, device=dev, precision="fp32")
        ref = conv(x.permute(0, 3, 1, 2)).detach()
        row = []
        for t in (90, 111, 112, 113, 114):
            if t in (111, 112) and cout % 128:
                row.append("   -  ")
                continue
            out = NHWC(torch.zeros(B, H, W, cout, device=dev), pair=True)
            try:
                fc(NHWC(to_pairs(x).to(dev), pair=True), out=out, tile=t)
                torch.cuda.synchronize()
                e = ((out.nchw().cpu() - ref).norm() / ref.norm()).item()
                row.append(f"{e:6.1e}")
            except Exception as ex:  # noqa: BLE001
                row.append(f"ERR {type(ex).__name__}")
        print(f"cin {cin:3d} cout {cout:3d} tap {tap}: " + " ".join(row), flush=True)
# one output pixel's error pattern for tap all, tile 111
cin, cout = 32, 128
conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
fc = FusedConv(conv, act=0, device=dev, precision="fp32")
x = torch.randn(1, 8, 16, cin)
ref = conv(x.permute(0, 3, 1, 2)).detach()
out = NHWC(torch.zeros(1, 8, 16, cout, device=dev), pair=True)
fc(NHWC(to_pairs(x).to(dev), pair=True), out=out, tile=111)
torch.cuda.synchronize()
err = (out.nchw().cpu() - ref).abs()
print("err by y (max over c, x):", [round(v, 3) for v in err.amax((0, 1, 3)).tolist()])
print("err by x (max over c, y):", [round(v, 3) for v in err.amax((0, 1, 2)).tolist()])
print("err by c group of 16:", [round(v, 3) for v in err.amax((0, 2, 3)).view(-1, 16).amax(1).tolist()])
