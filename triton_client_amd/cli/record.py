"""Synthetic sensor bags for replay / evaluation (no datasets are reachable):
camera frames (JPEG CompressedImage or raw Image), LiDAR sweeps (PointCloud2)
and, for evaluation, ground-truth Detection2DArray boxes drawn into the frames."""
from __future__ import annotations

import argparse
import sys

import numpy as np


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("out")
    p.add_argument("--frames", type=int, default=20)
    p.add_argument("--camera-topic", default="/camera/color/image_raw")
    p.add_argument("--lidar-topic", default="/ai_test_field/sensors/os_cloud_node/points")
    p.add_argument("--gt-topic", default="/camera/color/Detection2DArray")
    p.add_argument("--cam", default="720x1280")
    p.add_argument("--raw", action="store_true", help="raw rgb8 Image instead of JPEG")
    p.add_argument("--no-camera", action="store_true")
    p.add_argument("--lidar", action="store_true")
    p.add_argument("--rings", type=int, default=64)
    p.add_argument("--columns", type=int, default=1875)
    p.add_argument("--gt", action="store_true", help="also write synthetic ground-truth boxes")
    a = p.parse_args(argv)
    from ..inference.ros_inference import detections_to_msg
    from ..ros import Bag, compat, msgs
    from ..utils.draw import draw_rect
    from ..utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    H, W = (int(v) for v in a.cam.split("x"))
    spec = LidarSpec(rings=a.rings, azimuth_steps=a.columns, sensor_height=3.23)
    rng = np.random.default_rng(0)
    with Bag(a.out, "w") as bag:
        for s in range(a.frames):
            t = msgs.Time.from_sec(1.0 + 0.1 * s)
            if not a.no_camera:
                img = camera_frame(H, W, s)
                hdr = msgs.Header(seq=s, stamp=t, frame_id="camera")
                if a.gt:
                    n = int(rng.integers(1, 6))
                    g = np.zeros((n, 6), np.float32)
                    for k in range(n):
                        w, h = rng.uniform(0.05, 0.3) * W, rng.uniform(0.05, 0.3) * H
                        x, y = rng.uniform(0, W - w), rng.uniform(0, H - h)
                        g[k] = [x, y, x + w, y + h, 1.0, rng.integers(0, 2)]
                        img[int(y):int(y + h), int(x):int(x + w)] = (60, 180, 60) if g[k, 5] else (160, 80, 40)
                        draw_rect(img, x, y, x + w, y + h, (255, 255, 255), 1)
                    gm = detections_to_msg(g, msgs.Header(seq=s, stamp=t, frame_id="camera"))
                    bag.write(a.gt_topic, gm, t)
                if a.raw:
                    m = compat.numpy_to_imgmsg(img, "rgb8", header=hdr)
                else:
                    m = msgs.CompressedImage(header=hdr, format="rgb8; jpeg compressed bgr8",
                                             data=compat.jpeg_encode(img))
                bag.write(a.camera_topic, m, t)
            if a.lidar:
                pts = lidar_sweep(spec, s)
                raw = np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4)
                bag.write(a.lidar_topic, compat.create_cloud_xyzi(raw, msgs.Header(seq=s, stamp=t, frame_id="lidar")),
                          t)
    print(f"wrote {a.frames} frames to {a.out}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
