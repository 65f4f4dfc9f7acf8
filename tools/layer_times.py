"""Per-layer device time of the fused camera / BEV plans (eager, event-timed).

    python tools/layer_times.py [--branch camera|lidar] [--batch 32] [--reps 5]

Every FusedConv call (and the maxpool / upsample / fused C3 / stem kernels) of one
forward is bracketed by HIP events on the current stream; the table lists, per call
site, the mean time, the conv geometry (Cin -> N, k, stride, output H x W), the
storage (pair / fp32) and the dense-equivalent FLOP rate (2 * MACs * 3 split
products, fp32 mode) — the input to deciding which layer to fuse or retile.
Prints one JSON line (and a text table to stderr).
"""
import argparse
import json
import sys
import time
from collections import defaultdict

sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--branch", choices=["camera", "lidar"], default="camera")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()

    import numpy as np
    import torch

    from triton_client_amd.ops import conv as convmod
    from triton_client_amd.pipelines import CameraPipeline, LidarPipeline
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    dev = torch.device("cuda")
    rec = defaultdict(list)
    order = []
    on = {"v": False}

    def timed(label_fn, fn):
        def wrap(*args, **kw):
            if not on["v"]:
                return fn(*args, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn(*args, **kw)
            e1.record()
            key = label_fn(*args, **kw)
            if key not in rec:
                order.append(key)
            rec[key].append((e0, e1))
            return out
        return wrap

    counter = defaultdict(int)

    def conv_label(self, x, out=None, res=None, **kw):
        B, H, W, _ = x.shape
        Ho, Wo = self.out_hw(H, W) if hasattr(self, "out_hw") else (H, W)
        site = id(self)
        return ("conv", site, self.cin, self.N, self.k, self.s, Ho, Wo, bool(x.pair), bool(out.pair) if out else False,
                res is not None)

    orig_call = convmod.FusedConv.__call__
    convmod.FusedConv.__call__ = timed(conv_label, orig_call)
    for name in ("maxpool_nhwc", "upsample2x_nhwc", "sppf_pools"):
        f = getattr(convmod, name)
        setattr(convmod, name, timed(lambda x, out, *r, _n=name, **k: (_n, x.shape[1], x.shape[2], x.c), f))
    import triton_client_amd.models.fast as fast
    for name in ("maxpool_nhwc", "upsample2x_nhwc", "sppf_pools"):
        setattr(fast, name, getattr(convmod, name))
    fast._C3Plan.__call__ = timed(lambda self, x, out: ("c3", id(self), x.c, self.c_, x.shape[1], x.shape[2],
                                                        self.fused2_ok(x, out)),
                                            fast._C3Plan.__call__)

    B = a.batch
    if a.branch == "camera":
        p = CameraPipeline(batch=B, src_hw=(720, 1280), device=dev)
        for b in range(B):
            p.frames[b].copy_(torch.from_numpy(camera_frame(720, 1280, b % 8)))
        p.calibrate_detection_density(100.0)
    else:
        spec = LidarSpec(sensor_height=3.23)
        maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
        p = LidarPipeline(batch=B, max_points=maxp, device=dev)
        for b in range(B):
            c = lidar_sweep(spec, b % 8)
            raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
            p.data[b * p.frame_bytes: b * p.frame_bytes + raw.numel()].copy_(raw)
            p.frame_n[b] = c.shape[0]
        p.calibrate_detection_density(2000.0)
    p.step()
    torch.cuda.synchronize()
    step_ms = []
    for r in range(a.reps):
        on["v"] = r > 0
        t0 = time.perf_counter()
        p.step()
        torch.cuda.synchronize()
        step_ms.append(1e3 * (time.perf_counter() - t0))
    rows = []
    total = 0.0
    for key in order:
        ts = [e0.elapsed_time(e1) * 1e3 for e0, e1 in rec[key]]
        us = sum(ts) / len(ts)
        if key[0] != "c3":  # a C3's own time includes its convs
            total += us
        row = {"op": key[0], "us": round(us, 1)}
        if key[0] == "conv":
            _, _, cin, n, k, s, ho, wo, pin, pout, res = key
            fl = 2.0 * B * ho * wo * n * cin * k * k * 3
            row.update(cin=cin, n=n, k=k, s=s, out_hw=[ho, wo], pair_in=pin, pair_out=pout, res=res,
                       tflops_x3=round(fl / (us * 1e-6) / 1e12, 1))
        elif key[0] == "c3":
            row.update(cin=key[2], c_=key[3], hw=[key[4], key[5]], fused=key[6])
        else:
            row.update(hw=[key[1], key[2]], c=key[3])
        rows.append(row)
    print(f"{'op':6s} {'us':>8s}  detail", file=sys.stderr)
    for r in sorted(rows, key=lambda r: -r["us"]):
        print(f"{r['op']:6s} {r['us']:8.1f}  {json.dumps({k: v for k, v in r.items() if k not in ('op', 'us')})}",
              file=sys.stderr)
    print(json.dumps({"branch": a.branch, "batch": B, "eager_step_ms": [round(v, 3) for v in step_ms],
                      "layer_sum_us": round(total, 1), "layers": rows}))


if __name__ == "__main__":
    main()
