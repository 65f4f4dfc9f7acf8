#!/usr/bin/env python3
"""Upper-bound probes for the headline step (diagnostic only; the results are NOT measurements of
the framework: the skipped stages run on the previous batch's stale buffers).

How much would the headline gain if a stage cost nothing?  ``WHATIF`` names the stage removed from
the captured step; everything else is ``bench.py`` unchanged (same flags).

  WHATIF=novox   the LiDAR unpack + voxeliser chain (pc2_unpack, canvas clear, assign, finish):
                 only the PillarVFE scatter runs, over the slots of the warm-up batches
  WHATIF=nofront the whole LiDAR front (voxeliser + PillarVFE): the BEV blocks read a stale canvas
  WHATIF=nopost  the LiDAR anchor decode + rotated NMS: the step returns the warm-up batches' result
  WHATIF=noneck  the fused neck + head: the decode + NMS read the warm-up batches' head maps

    WHATIF=novox python tools/whatif_bench.py --steps 30 --warmup 5
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.chdir(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from triton_client_amd.pipelines import lidar as lidar_mod

    mode = os.environ.get("WHATIF", "")
    warm = int(os.environ.get("WHATIF_FULL_CALLS", "4"))  # eager warm-up calls that still run everything

    @torch.no_grad()
    def step_pre(self):
        from triton_client_amd.ops.lidar import pc2_unpack
        n = getattr(self, "_whatif_calls", 0)
        self._whatif_calls = n + 1
        if n < warm:  # LidarPipeline.step_pre, keeping the point buffer for the probe calls
            if self.use_fast and self.fast is None:
                self.build_fast()
            pts, cnt = pc2_unpack(self.ws, self.data, self.frame_off, self.frame_n, self.layout, self.max_points,
                                  self.normalize, self.z_offset)
            self._whatif_pts = pts
            self.enc.clear(self.vox)
            self.vox.assign(pts, cnt)
            canvas = self.enc.encode_from_slots(pts, self.vox)
            self.vox.finish(pts, cnt, gather=False)
            return canvas
        if mode == "novox":
            return self.enc.encode_from_slots(self._whatif_pts, self.vox)
        return self.enc.canvas_nchw()  # nofront

    @torch.no_grad()
    def step_back(self):
        n = getattr(self, "_whatif_back", 0)
        self._whatif_back = n + 1
        if n < warm:  # LidarPipeline.step_back
            head = self._head if self._blocks is None else self.fast.forward_neck(self._blocks)
            self._whatif_res = self.post(*head)
            return self._whatif_res
        if mode == "nopost":
            if self._blocks is not None:
                self.fast.forward_neck(self._blocks)
            return self._whatif_res
        return self.post(*self.fast.head_maps())  # noneck

    if mode in ("novox", "nofront"):
        lidar_mod.LidarPipeline.step_pre = step_pre
    elif mode in ("nopost", "noneck"):
        lidar_mod.LidarPipeline.step_back = step_back
    elif mode:
        raise SystemExit(f"WHATIF={mode!r}: novox, nofront, nopost or noneck")
    import bench
    bench.main()


if __name__ == "__main__":
    main()
