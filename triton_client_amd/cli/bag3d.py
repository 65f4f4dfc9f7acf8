"""Offline 3D bag replay (reference ``bag3d.py``): bag → <bag>_output.bag with boxes."""
from __future__ import annotations

import argparse
import os
import sys

from .common import DATA, add_framework_flags, add_reference_flags, labels_arg, load_params, setup_logging
from .engines import engine_3d, export_if_asked, maybe_data_parallel


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    add_reference_flags(p, "pointpillar_kitti")
    add_framework_flags(p, os.path.join(DATA, "client_parameter_3d.yaml"), three_d=True)
    p.add_argument("--bag", required=True, help="input bag")
    p.add_argument("--out-bag", default="", help="output bag (default <bag>_output.bag, 'none' to skip)")
    p.add_argument("--start-seq", type=int, default=0)
    p.add_argument("--max-frames", type=int, default=None)
    return p.parse_args(argv)


def main(argv=None) -> int:
    flags = parse_args(argv)
    setup_logging(flags.verbose)
    from ..inference import BagInference3D

    params = load_params(flags.params, flags.server)
    engine, channel, client = engine_3d(flags, params)
    info = None
    if flags.engine == "local":
        engine, info = maybe_data_parallel(engine, three_d=True)
        if info is not None and not info.is_main:  # worker rank: serve shards until rank 0 is done
            engine.serve()
            from ..parallel.dp import shutdown
            shutdown(info)
            return 0
    drv = BagInference3D(channel, client, engine=engine, params=params, bagfile=flags.bag,
                         out_bag=None if flags.out_bag == "none" else flags.out_bag,
                         batch=max(1, flags.frames_per_step), start_seq=flags.start_seq,
                         max_frames=flags.max_frames, verbose=flags.verbose, jsk=not flags.detection3d,
                         labels=labels_arg(flags.labels), score_thresh=flags.score_thresh)
    n = drv.start_inference()
    export_if_asked(flags, engine)
    if info is not None:
        engine.close()
        from ..parallel.dp import shutdown
        shutdown(info)
    fps = n / drv.elapsed if drv.elapsed > 0 else 0.0
    print(f"processed {n} clouds in {drv.elapsed:.2f}s ({fps:.1f} FPS)", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
