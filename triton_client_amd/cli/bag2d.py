"""Offline 2D bag replay (reference ``bag2d.py``): bag → annotated PNGs (+ output bag)."""
from __future__ import annotations

import argparse
import os
import sys

from .common import DATA, add_framework_flags, add_reference_flags, load_params, setup_logging
from .engines import engine_2d, export_if_asked, maybe_data_parallel


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    add_reference_flags(p, "YOLOv5n")
    add_framework_flags(p, os.path.join(DATA, "client_parameter.yaml"))
    p.add_argument("--bag", required=True, help="input bag")
    p.add_argument("--out", default="./output_data", help="PNG output directory ('' to skip)")
    p.add_argument("--out-bag", default=None, help="write input + annotated image + detections here")
    p.add_argument("--start-seq", type=int, default=0, help="resume after this many frames")
    p.add_argument("--max-frames", type=int, default=None)
    return p.parse_args(argv)


def main(argv=None) -> int:
    flags = parse_args(argv)
    setup_logging(flags.verbose)
    from ..inference import BagInference2D

    params = load_params(flags.params, flags.server)
    engine, channel, client = engine_2d(flags, params)
    info = None
    if flags.engine == "local":
        engine, info = maybe_data_parallel(engine)
        if info is not None and not info.is_main:  # worker rank: serve shards until rank 0 is done
            engine.serve()
            from ..parallel.dp import shutdown
            shutdown(info)
            return 0
    drv = BagInference2D(channel, client, engine=engine, params=params, bagfile=flags.bag, out_dir=flags.out or None,
                         out_bag=flags.out_bag, batch=max(1, flags.frames_per_step), save_png=bool(flags.out),
                         start_seq=flags.start_seq, max_frames=flags.max_frames)
    n = drv.start_inference()
    export_if_asked(flags, engine)
    if info is not None:
        engine.close()
        from ..parallel.dp import shutdown
        shutdown(info)
    fps = n / drv.elapsed if drv.elapsed > 0 else 0.0
    print(f"processed {n} frames in {drv.elapsed:.2f}s ({fps:.1f} FPS)", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
