"""Debug: is the BEV backbone output deterministic/correct at bench scale?"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from triton_client_amd.models.common import fuse_model  # noqa: E402
from triton_client_amd.models.pointpillars import build_pointpillars  # noqa: E402
from triton_client_amd.pipelines import LidarPipeline  # noqa: E402
from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep  # noqa: E402


def stats(name, t):
    t = t.float()
    print(f"{name}: shape {tuple(t.shape)} finite {bool(torch.isfinite(t).all())} min {t.min().item():.3g} "
          f"max {t.max().item():.3g} mean {t.mean().item():.3g}", flush=True)


def main():
    for B in (1, 2, 16):
        spec = LidarSpec(sensor_height=3.23)
        maxp = ((spec.points_per_sweep + 1023) // 1024) * 1024
        lid = LidarPipeline(batch=B, max_points=maxp, device="cuda", z_offset=1.5)
        for b in range(B):
            c = lidar_sweep(spec, 500 + b % 8)
            raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
            lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
            lid.frame_n[b] = c.shape[0]
        lid.step()
        torch.cuda.synchronize()
        canvas = lid.enc.canvas_nchw()
        stats(f"B={B} canvas", canvas)
        with torch.no_grad():
            o1 = lid.model.bev_forward(canvas)
            o2 = lid.model.bev_forward(canvas)
            torch.cuda.synchronize()
            for k, (a, b_) in enumerate(zip(o1, o2)):
                stats(f"  head{k}", a)
                print("   deterministic:", torch.equal(a, b_), flush=True)
            # reference: fp32 NCHW on the GPU and on the CPU for frame 0
            ref = fuse_model(build_pointpillars().eval())
            ref.head.conv_cls.bias.data.copy_(lid.model.head.conv_cls.bias.float())
            c0 = canvas[:1].float().contiguous()
            r_gpu = ref.cuda().bev_forward(c0)
            r_cpu = ref.cpu().bev_forward(c0.cpu())
            for k in range(3):
                d_bf = (o1[k][:1].float().cpu() - r_cpu[k]).abs().max().item()
                d_f32 = (r_gpu[k].cpu() - r_cpu[k]).abs().max().item()
                print(f"   head{k}: |bf16 CL gpu - fp32 cpu| = {d_bf:.4g}  |fp32 gpu - fp32 cpu| = {d_f32:.4g}"
                      f"  ref scale {r_cpu[k].abs().max().item():.4g}", flush=True)
            # backbone stages, bf16 CL vs cpu fp32
            x_b, x_c = canvas[:1], c0.cpu()
            for i, (blk_b, blk_c) in enumerate(zip(lid.model.backbone.blocks, ref.backbone.blocks)):
                x_b = blk_b(x_b)
                x_c = blk_c(x_c)
                print(f"   block{i}: diff {(x_b.float().cpu() - x_c).abs().max().item():.4g} scale {x_c.abs().max().item():.4g}")
                u_b = lid.model.backbone.deblocks[i](x_b)
                u_c = ref.backbone.deblocks[i](x_c)
                print(f"   deblock{i}: diff {(u_b.float().cpu() - u_c).abs().max().item():.4g} scale {u_c.abs().max().item():.4g}"
                      f" layout_cl={u_b.is_contiguous(memory_format=torch.channels_last)}")
        del lid
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
