"""Probe: forward latency of the detector models through PyTorch-ROCm (MIOpen)
at several batch sizes, dtypes and memory formats, eager vs hipGraph.
Used to decide which convolutions need the hand-written MFMA path."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from triton_client_amd.models.common import fuse_model  # noqa: E402
from triton_client_amd.models.yolov5 import build_yolov5  # noqa: E402
from triton_client_amd.models.pointpillars import build_pointpillars  # noqa: E402


def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def graphed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g.replay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,16,32")
    args = ap.parse_args()
    dev = "cuda"
    res = []
    y = fuse_model(build_yolov5("n").eval()).to(dev)
    pp = fuse_model(build_pointpillars().eval()).to(dev)
    for dtype in (torch.bfloat16, torch.float16):
        for cl in (True, False):
            mf = torch.channels_last if cl else torch.contiguous_format
            ym = y.to(dtype=dtype, memory_format=mf)
            pm = pp.to(dtype=dtype, memory_format=mf)
            for b in [int(x) for x in args.batches.split(",")]:
                x = torch.randn(b, 3, 640, 640, device=dev, dtype=dtype).contiguous(memory_format=mf)
                c = torch.randn(b, 64, 496, 432, device=dev, dtype=dtype).contiguous(memory_format=mf)
                with torch.no_grad():
                    fy = lambda: ym(x)  # noqa
                    fp = lambda: pm.bev_forward(c)  # noqa
                    ty = bench(fy)
                    tp = bench(fp)
                    try:
                        ty_g = bench(graphed(fy))
                        tp_g = bench(graphed(fp))
                    except Exception as e:  # noqa
                        ty_g = tp_g = float("nan")
                        print("graph failed", e)
                r = dict(dtype=str(dtype), channels_last=cl, batch=b, yolo_ms=ty, yolo_graph_ms=ty_g,
                         pp_ms=tp, pp_graph_ms=tp_g)
                print(json.dumps(r), flush=True)
                res.append(r)


if __name__ == "__main__":
    main()
