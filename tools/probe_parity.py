"""Diagnose end-to-end detection parity of the camera pipeline: where do the
GPU pipeline and the fp32 module + CPU postprocess diverge?  (tools only)"""
import copy
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from triton_client_amd.ops.golden import box_iou_np, preprocess_image  # noqa: E402
from triton_client_amd.ops.image import space_to_depth2  # noqa: E402
from triton_client_amd.pipelines import CameraPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import camera_frame  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


def main(precision="fp32"):
    dev = torch.device("cuda")
    B = 2
    cam = CameraPipeline(batch=B, src_hw=(360, 640), device=dev, precision=precision)
    frames = [camera_frame(360, 640, 10 + b) for b in range(B)]
    for b in range(B):
        cam.frames[b].copy_(torch.from_numpy(frames[b]))
    cam.calibrate_detection_density(100.0)
    got = cam.step()
    torch.cuda.synchronize()
    f = cam.fast
    x = torch.from_numpy(np.stack([preprocess_image(fr, (640, 640), "letterbox") for fr in frames]))
    xs = space_to_depth2(x.permute(0, 2, 3, 1).contiguous())
    print("input S2D rel", rel(f.x.t.float().cpu(), xs), "maxabs", (f.x.t.float().cpu() - xs).abs().max().item())
    model = copy.deepcopy(cam.model).float().to(memory_format=torch.contiguous_format)
    with torch.no_grad():
        heads = model(x.to(dev))
        heads64 = copy.deepcopy(model).double()(x.to(dev).double())
    C = cam.post.na * (cam.post.nc + 5)
    for i, (h, h64, d) in enumerate(zip(heads, heads64, f.dout)):
        g = d.t[..., :C].permute(0, 3, 1, 2).float()
        print(f"head {i}: fast vs f64 rel {rel(g, h64):.3e}  module32 vs f64 rel {rel(h, h64):.3e}  "
              f"maxabs fast-f64 {(g.double() - h64).abs().max().item():.3e}")
    ref = cam.post.cpu([h.float().cpu() for h in heads], cam.xform)
    ref_fast = cam.post.cpu([d.t[..., :C].permute(0, 3, 1, 2).float().cpu() for d in f.dout], cam.xform)
    for b in range(B):
        for name, r in (("module", ref), ("fast-heads-cpu-post", ref_fast)):
            n_r, n_g = int(r.count[b]), int(got.count[b])
            rb, gb = np.asarray(r.box[b, :n_r]), got.box[b, :n_g].cpu().numpy()
            iou = box_iou_np(rb, gb) * (np.asarray(r.cls[b, :n_r])[:, None] == got.cls[b, :n_g].cpu().numpy()[None])
            best = iou.max(1)
            print(f"frame {b} vs {name}: n_ref {n_r} n_gpu {n_g} matched@0.99 {(best > 0.99).mean():.3f} "
                  f"@0.9 {(best > 0.9).mean():.3f}")
            bad = np.nonzero(best <= 0.99)[0][:5]
            for i in bad:
                j = iou[i].argmax()
                print("   ref", rb[i].round(3), float(r.score[b, i]), int(r.cls[b, i]), " gpu", gb[j].round(3),
                      float(got.score[b, j]), int(got.cls[b, j]), "iou", round(float(iou[i, j]), 4))


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["fp32"]))
