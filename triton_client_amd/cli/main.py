"""2D live inference (reference ``main.py``): camera topic → detections."""
from __future__ import annotations

import argparse
import os
import sys

from .common import (DATA, add_framework_flags, add_reference_flags, image_files, load_params, play_bag,
                     setup_logging)
from .engines import engine_2d, export_if_asked, maybe_data_parallel


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__)
    add_reference_flags(p, "YOLOv5n")
    add_framework_flags(p, os.path.join(DATA, "client_parameter.yaml"))
    return p.parse_args(argv)


def main(argv=None) -> int:
    flags = parse_args(argv)
    setup_logging(flags.verbose)
    from ..inference import RosInference
    from ..ros import compat, default_bus

    compat.init_node("ros_infer_2D")
    params = load_params(flags.params, flags.server)
    engine, channel, client = engine_2d(flags, params)
    info = None
    if flags.engine == "local":  # under torchrun: shard every micro-batch over the node's GPUs
        engine, info = maybe_data_parallel(engine)
        if info is not None and not info.is_main:
            engine.serve()
            from ..parallel.dp import shutdown
            shutdown(info)
            return 0
    metrics = None
    if flags.metrics_port:
        from ..utils.metrics import ClientMetrics
        metrics = ClientMetrics(flags.metrics_port)
    bus = default_bus() if (flags.play or flags.image_src == "local" or not compat.HAVE_ROSPY) else None
    drv = RosInference(channel, client, engine=engine, params=params, bus=bus, metrics=metrics,
                       queue_size=None if flags.play or flags.image_src == "local" else 1,
                       batch=flags.live_batch, workers=flags.live_workers)
    if flags.image_src == "local":
        rc = _run_local_images(drv, flags, params)
        export_if_asked(flags, engine)
        if info is not None:
            engine.close()
            from ..parallel.dp import shutdown
            shutdown(info)
        return rc
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
    print(f"processed {drv.frames} frames", file=sys.stderr)
    return 0


def _run_local_images(drv, flags, params) -> int:
    """-i local: run the image files in --images and write annotated PNGs next to them."""
    import numpy as np
    from PIL import Image

    from ..ros import msgs

    if not flags.images:
        raise SystemExit("-i local needs --images DIR")
    files = image_files(flags.images)
    out_dir = os.path.join(flags.images, "detections")
    os.makedirs(out_dir, exist_ok=True)
    step = max(1, flags.frames_per_step)
    from ..ros import compat
    for s in range(0, len(files), step):
        batch = []
        for k, f in enumerate(files[s:s + step]):
            img = np.asarray(Image.open(f).convert("RGB"))
            batch.append(compat.numpy_to_imgmsg(img, header=msgs.Header(seq=s + k, frame_id=os.path.basename(f))))
        for m, (im, _, d) in zip(batch, drv.process(batch)):
            Image.fromarray(compat.imgmsg_to_numpy(im)).save(os.path.join(out_dir, m.header.frame_id + ".png"))
            print(f"{m.header.frame_id}: {len(d)} detections")
    return 0


if __name__ == "__main__":
    sys.exit(main())
