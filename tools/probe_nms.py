"""Probe the LiDAR NMS stage on the bench's real candidate distribution:
per-frame candidate counts, circumcircle / AABB pair counts, and per-kernel
times of topk / mask (several grids) / reduce.  One JSON line per measurement."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from triton_client_amd import _native  # noqa: E402
from triton_client_amd.pipelines import LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    dev = torch.device("cuda")
    B = 16
    spec = LidarSpec(rings=64, azimuth_steps=1875, sensor_height=3.23)
    maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
    lid = LidarPipeline(batch=B, max_points=maxp, device=dev, z_offset=1.5)
    fb = lid.frame_bytes
    for b in range(B):
        c = lidar_sweep(spec, 500 + b)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * fb:b * fb + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    lid.calibrate_detection_density(2000.0)
    res = lid.step()
    torch.cuda.synchronize()
    post = lid.post
    ws = post.ws
    cfg = post.cfg
    cand = {k: ws._bufs["anc_" + k] for k in ("box", "score", "cls", "key", "count")}
    order, nsorted, mask = ws._bufs["anc_nms_order"], ws._bufs["anc_nms_nsorted"], \
        ws._bufs["anc_nms_mask"]
    cap = cand["box"].shape[1]
    pre_max = order.shape[1]
    n = nsorted.cpu().numpy()
    kept = res.count.cpu().numpy() if hasattr(res, "count") else None
    print(json.dumps({"count": cand["count"].cpu().tolist(), "nsorted": n.tolist(),
                      "kept": None if kept is None else kept.tolist(), "pre_max": pre_max, "cap": cap}))
    # pair statistics on frame 0
    o = order[0, : n[0]].long()
    bx = cand["box"][0, o].float()
    r = 0.5 * torch.sqrt(bx[:, 3] ** 2 + bx[:, 4] ** 2)
    d2 = (bx[:, None, 0] - bx[None, :, 0]) ** 2 + (bx[:, None, 1] - bx[None, :, 1]) ** 2
    circ = (d2 <= (r[:, None] + r[None, :]) ** 2).triu(1).sum().item()
    print(json.dumps({"frame0_n": int(n[0]), "circle_pairs": circ, "all_pairs": int(n[0] * (n[0] - 1) // 2)}))
    s = 0
    words = (pre_max + 63) // 64
    P = _native.ptr
    t_topk = timeit(lambda: _native.call("tca_topk_sort", P(cand["key"]), P(cand["count"]), B, cap, pre_max,
                                         P(order), P(nsorted), s))
    res_t = {"topk_us": round(t_topk, 1)}
    for g in (64, 128, 256, 512, 1024, 2048):
        res_t[f"mask_g{g}_us"] = round(timeit(lambda: _native.call(
            "tca_nms_mask", 1, P(cand["box"]), 7, P(cand["cls"]), P(order), P(nsorted), B, cap, pre_max,
            float(cfg.nms_thresh), 1, P(mask), g, s)), 1)
    # v2 mask (prep + tile kernel) vs v1 on the upper-triangle words
    _native.call("tca_nms_mask", 1, P(cand["box"]), 7, P(cand["cls"]), P(order), P(nsorted), B, cap, pre_max,
                 float(cfg.nms_thresh), 1, P(mask), 2048, s)
    m1 = mask.clone()
    soa = torch.zeros(B, 9, (pre_max + 3) // 4 * 4, device=dev)
    mask.zero_()
    res_t["mask_rot_us"] = round(timeit(lambda: _native.call(
        "tca_nms_mask_rot", P(cand["box"]), 7, P(cand["cls"]), P(order), P(nsorted), B, cap, pre_max,
        float(cfg.nms_thresh), 1, P(soa), P(mask), s)), 1)
    torch.cuda.synchronize()
    bad = 0
    for b in range(B):
        nb = (int(n[b]) + 63) // 64
        for rb in range(nb):
            rows = slice(rb * 64, min(int(n[b]), rb * 64 + 64))
            bad += int((m1[b, rows, rb:nb] != mask[b, rows, rb:nb]).sum().item())
    res_t["mask_mismatch_words"] = bad
    out = [torch.empty(B, cfg.nms_post_max, 7, device=dev), torch.empty(B, cfg.nms_post_max, device=dev),
           torch.empty(B, cfg.nms_post_max, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)]
    res_t["reduce_us"] = round(timeit(lambda: _native.call(
        "tca_nms_reduce", P(order), P(nsorted), P(mask), B, pre_max, P(cand["box"]), 7, P(cand["score"]),
        P(cand["cls"]), cap, cfg.nms_post_max, None, P(out[0]), P(out[1]), P(out[2]), P(out[3]), s)), 1)
    res_t["words"] = words
    print(json.dumps(res_t))


if __name__ == "__main__":
    main()
