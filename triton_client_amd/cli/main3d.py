"""3D live inference (reference ``main3d.py``): PointCloud2 topic → 3D boxes."""
from __future__ import annotations

import argparse
import os
import sys

from .common import DATA, add_framework_flags, add_reference_flags, labels_arg, load_params, play_bag, setup_logging
from .engines import engine_3d, export_if_asked, maybe_data_parallel


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    add_reference_flags(p, "pointpillar_kitti")
    add_framework_flags(p, os.path.join(DATA, "client_parameter_3d.yaml"), three_d=True)
    return p.parse_args(argv)


def main(argv=None) -> int:
    flags = parse_args(argv)
    setup_logging(flags.verbose)
    from ..inference import RosInference3D
    from ..ros import compat, default_bus

    compat.init_node("ros_infer_3d")
    params = load_params(flags.params, flags.server)
    engine, channel, client = engine_3d(flags, params)
    info = None
    if flags.engine == "local":  # under torchrun: shard every micro-batch over the node's GPUs
        engine, info = maybe_data_parallel(engine, three_d=True)
        if info is not None and not info.is_main:
            engine.serve()
            from ..parallel.dp import shutdown
            shutdown(info)
            return 0
    bus = default_bus() if (flags.play or not compat.HAVE_ROSPY) else None
    drv = RosInference3D(channel, client, engine=engine, params=params, bus=bus, jsk=not flags.detection3d,
                         labels=labels_arg(flags.labels), score_thresh=flags.score_thresh,
                         queue_size=None if flags.play else 50,
                       batch=flags.live_batch, workers=flags.live_workers)
    if flags.play:
        play_bag(flags.play, bus, topics=[params["sub_topic"]])
    drv.start_inference(spin=True, timeout=flags.spin_timeout)
    drv.stop()
    if hasattr(engine, "release_transport"):  # a remote client's shared-memory regions
        engine.release_transport()
    export_if_asked(flags, engine)
    if info is not None:
        engine.close()
        from ..parallel.dp import shutdown
        shutdown(info)
    print(f"processed {drv.frames} clouds", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
