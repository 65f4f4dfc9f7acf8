"""Bag utilities (reference ``tools/bag_stitch.py``, ``tools/pc_extractor.py``).

    python -m triton_client_amd.cli.bagtools info BAG
    python -m triton_client_amd.cli.bagtools stitch SRC DST [-n 500] [--topics T ...]
    python -m triton_client_amd.cli.bagtools extract-pc BAG OUT_DIR [--topic T] [--bev] [--scene]
"""
from __future__ import annotations

import argparse
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("info")
    p.add_argument("bag")
    p = sub.add_parser("stitch", help="copy the first N messages (reference bag_stitch.py: 500)")
    p.add_argument("src")
    p.add_argument("dst")
    p.add_argument("-n", type=int, default=500)
    p.add_argument("--topics", nargs="*", default=None)
    p = sub.add_parser("extract-pc", help="PointCloud2 messages → NNNNNN.npy [N, 4] (x, y, z, intensity)")
    p.add_argument("bag")
    p.add_argument("out")
    p.add_argument("--topic", default=None, help="default: every PointCloud2 topic")
    p.add_argument("--bev", action="store_true", help="also write a bird's-eye-view PNG per cloud")
    p.add_argument("--scene", action="store_true",
                   help="also write a 3D scene view PNG per cloud (the reference's Open3D draw_scenes, headless)")
    a = ap.parse_args(argv)
    from ..ros import Bag, msgs
    from ..ros.bag import stitch

    if a.cmd == "info":
        with Bag(a.bag) as b:
            info = b.get_type_and_topic_info()
            n = b.get_message_count()
        print(f"{a.bag}: {n} messages")
        for topic, d in sorted(info.items()):
            print(f"  {topic:50s} {d['type']:40s} {d['count']}")
        return 0
    if a.cmd == "stitch":
        n = stitch(a.src, a.dst, a.n, a.topics)
        print(f"wrote {n} messages to {a.dst}")
        return 0
    import numpy as np

    from ..ros.compat import cloud_to_numpy
    from ..utils.visualize import draw_scenes, render_bev

    os.makedirs(a.out, exist_ok=True)
    k = 0
    with Bag(a.bag) as b:
        for topic, m, _ in b.read_messages(topics=[a.topic] if a.topic else None):
            if not isinstance(m, msgs.PointCloud2):
                continue
            pts = cloud_to_numpy(m)
            np.save(os.path.join(a.out, f"{k:06d}.npy"), pts)
            if a.bev:
                render_bev(pts, path=os.path.join(a.out, f"{k:06d}.png"))
            if a.scene:
                draw_scenes(pts, path=os.path.join(a.out, f"{k:06d}_scene.png"))
            k += 1
    print(f"extracted {k} clouds to {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
