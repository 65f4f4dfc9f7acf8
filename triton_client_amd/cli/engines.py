"""Engine construction from CLI flags (local MI355X pipeline or remote server)."""
from __future__ import annotations

import os

from .common import DATA, make_channel, make_client, rpc_mode


def yolo_spec(model_name: str, classes: int):
    """(variant, nc, img, names file) of a known YOLO deployment name."""
    n = model_name.lower()
    if "crop" in n or "weed" in n:  # examples/YOLOv5/config.pbtxt: 512, 2 classes
        return "n", 2, 512, os.path.join(DATA, "crop.names")
    variant = "n"
    for v in ("n", "s", "m", "l", "x"):
        if n.startswith("yolov5" + v):
            variant = v
    return variant, classes, 640, os.path.join(DATA, "coco.names")


def engine_2d(flags, params, letterbox=None, conf_thres=None):
    """→ (engine, channel, client)."""
    lb = flags.letterbox if letterbox is None else letterbox
    conf = flags.conf_thres if conf_thres is None else conf_thres
    if flags.engine == "local":
        from ..inference import LocalDetector2D
        from ..clients.postprocess.base_postprocess import Postprocess

        variant, nc, img, names = yolo_spec(flags.model_name, flags.classes)
        eng = LocalDetector2D(variant, nc, img, batch=max(1, flags.frames_per_step), letterbox=lb, conf_thres=conf,
                              device=flags.device, weights=flags.weights,
                              names=Postprocess.load_class_names(names) if os.path.exists(names) else None)
        return eng, None, None
    from ..inference import RemoteDetector2D

    ch = make_channel(params, flags)
    client = make_client(flags, ch)
    eng = RemoteDetector2D(ch, client, letterbox=lb, conf_thres=conf, mode=rpc_mode(flags), wire=flags.wire,
                           scaling=flags.scaling if flags.scaling != "COCO" else None,
                           device=flags.device if flags.device != "auto" else "cpu")
    return eng, ch, client


def lidar_family(model_name: str) -> str:
    """Model family of a served 3D model name (the reference's ``-m`` values:
    ``second_iou`` by default in .vscode/launch.json, ``pointpillar_kitti``)."""
    n = model_name.lower()
    if "second" in n:
        return "second_iou"
    if "centerpoint" in n or "nusc" in n:
        return "centerpoint"
    return "pointpillars"


def engine_3d(flags, params):
    if flags.engine == "local":
        from ..inference import LocalDetector3D

        eng = LocalDetector3D(batch=max(1, flags.frames_per_step), device=flags.device, weights=flags.weights,
                              z_offset=flags.z_offset, family=lidar_family(flags.model_name))
        return eng, None, None
    from ..inference import RemoteDetector3D

    ch = make_channel(params, flags)
    client = make_client(flags, ch)
    eng = RemoteDetector3D(ch, client, z_offset=flags.z_offset, mode=rpc_mode(flags), wire=flags.wire)
    return eng, ch, client


def maybe_data_parallel(engine, three_d: bool = False):
    """Under torchrun (WORLD_SIZE > 1) wrap a *local* engine so rank 0's frames
    are sharded over every GPU (RCCL scatter/gather).  Returns (engine, info);
    non-main ranks must call ``engine.serve()`` instead of running a driver."""
    import os

    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return engine, None
    from ..parallel.dp import DataParallelDetector2D, DataParallelDetector3D, init_distributed

    info = init_distributed()
    if hasattr(engine, "calibrate_synthetic"):
        engine.calibrate_synthetic()
    if hasattr(engine, "model"):
        from ..models.common import broadcast_parameters

        broadcast_parameters(engine.model)  # every replica runs rank 0's weights
    # rank-failure detection: heartbeats over the c10d store; a dead rank's
    # shards are re-split over the survivors (TCA_DP_HEARTBEAT=0 disables)
    monitor = None
    if os.environ.get("TCA_DP_HEARTBEAT", "1") != "0":
        from ..parallel.dp import HealthMonitor

        monitor = HealthMonitor(info, timeout=float(os.environ.get("TCA_DP_HEARTBEAT_TIMEOUT", "5")))
    box_dim = 9 if getattr(engine, "family", "") == "centerpoint" else 7
    wrap = (DataParallelDetector3D(engine, info, box_dim=box_dim, monitor=monitor) if three_d
            else DataParallelDetector2D(engine, info, monitor=monitor))
    return wrap, info
