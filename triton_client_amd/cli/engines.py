"""Engine construction from CLI flags (local MI355X pipeline or remote server)."""
from __future__ import annotations

import os

from .common import DATA, make_channel, make_client, resolve_device, rpc_mode


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


def camera_spec(model_name: str, classes: int):
    """Local camera engine for a served 2D model name (the reference's ``-m``):
    (family, YOLOv5 variant, nc, model input (H, W), names file).  The names follow
    the reference's model repository: YOLOv5* / weed_detector / *CROP
    (``examples/YOLOv5/config.pbtxt``), YOLOv4 (``examples/YOLOv4/config.pbtxt``),
    ``test_model`` = RetinaNet (``examples/RetinaNet_detectron/config.pbtxt``,
    input [3, 640, 480]), *retina* / *fcos* / *detectron* (Detectron2, the 1333x800
    class).  An unknown name raises instead of running another network."""
    n = model_name.lower()
    coco = os.path.join(DATA, "coco.names")
    if "yolov4" in n:
        return "yolov4", "n", classes, (512, 512), coco
    if n.startswith("yolov5") or "weed_detector" == n or "crop" in n or n.startswith("yolo"):
        variant, nc, img, names = yolo_spec(model_name, classes)
        return "yolov5", variant, nc, (img, img), names
    if n == "test_model":
        return "retinanet", "n", classes, (640, 480), coco
    if "fcos" in n or "retina" in n or "detectron" in n:
        fam = "fcos" if "fcos" in n else "retinanet"
        if "weed" in n:  # main.py:75 -m fcos_weed_detector: weeds, maize
            return fam, "n", 2, (800, 1344), os.path.join(DATA, "crop.names")
        return fam, "n", classes, (800, 1344), coco
    raise ValueError(f"-m {model_name!r}: no local camera engine for this model name (YOLOv5*, weed_detector, "
                     "YOLOv4, test_model, *retina*, *fcos*); use --engine remote to serve it elsewhere")


def engine_2d(flags, params, letterbox=None, conf_thres=None):
    """→ (engine, channel, client)."""
    lb = flags.letterbox if letterbox is None else letterbox
    conf = flags.conf_thres if conf_thres is None else conf_thres
    if flags.engine == "local":
        from ..inference import LocalDetector2D
        from ..clients.postprocess.base_postprocess import Postprocess

        family, variant, nc, img, names = camera_spec(flags.model_name, flags.classes)
        if family == "yolov4" and conf_thres is None and flags.conf_thres == 0.3:
            conf = 0.4  # tools/utils.py:166-233 post-processing (conf 0.4, NMS 0.6)
        eng = LocalDetector2D(variant, nc, img, batch=max(1, flags.frames_per_step), letterbox=lb, conf_thres=conf,
                              iou_thres=0.6 if family == "yolov4" else 0.45, device=flags.device,
                              weights=flags.weights, family=family,
                              names=Postprocess.load_class_names(names) if os.path.exists(names) else None)
        return eng, None, None
    from ..inference import RemoteDetector2D

    ch = make_channel(params, flags)
    client = make_client(flags, ch)
    eng = RemoteDetector2D(ch, client, letterbox=lb, conf_thres=conf, mode=rpc_mode(flags), wire=flags.wire,
                           scaling=flags.scaling if flags.scaling != "COCO" else None,
                           device=resolve_device(flags.device))
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
    eng = RemoteDetector3D(ch, client, z_offset=flags.z_offset, mode=rpc_mode(flags), wire=flags.wire,
                           device=resolve_device(flags.device))
    return eng, ch, client


def export_if_asked(flags, engine) -> None:
    """``--export-weights``: the local engine's fused, calibrated model as a checkpoint
    (rank 0 under data parallelism; the replicas hold the same weights)."""
    path = getattr(flags, "export_weights", None)
    if not path or flags.engine != "local":
        return
    from ..inference.engines import export_weights

    export_weights(getattr(engine, "local", engine).model, path)


def maybe_data_parallel(engine, three_d: bool = False):
    """Under torchrun (WORLD_SIZE > 1) wrap a *local* engine so rank 0's frames
    are sharded over every GPU (RCCL scatter/gather).  Returns (engine, info);
    non-main ranks must call ``engine.serve()`` instead of running a driver."""
    import os

    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return engine, None
    from ..parallel.dp import DataParallelDetector2D, DataParallelDetector3D, init_distributed

    info = init_distributed()
    # random-init weights: rank 0 calibrates the head prior on the node batch's first frame
    # (what one GPU does) and broadcasts the result; the gather checks that the replicas agree
    # rank-failure detection: heartbeats over the c10d store; a dead rank's
    # shards are re-split over the survivors (TCA_DP_HEARTBEAT=0 disables)
    monitor = None
    if os.environ.get("TCA_DP_HEARTBEAT", "1") != "0":
        from ..parallel.dp import HealthMonitor

        monitor = HealthMonitor(info, timeout=float(os.environ.get("TCA_DP_HEARTBEAT_TIMEOUT", "5")))
    box_dim = 9 if getattr(engine, "family", "") == "centerpoint" else 7
    comm = native_comm(info)
    wrap = (DataParallelDetector3D(engine, info, box_dim=box_dim, monitor=monitor, comm=comm) if three_d
            else DataParallelDetector2D(engine, info, monitor=monitor, comm=comm))
    return wrap, info


_COMM = {}


def native_comm(info):
    """The C++ RCCL communicator for the DP detection gather (one per process, shared
    by the 2D and 3D detectors), or None under the gloo rehearsal / on CPU.  Every
    rank takes the same decision (an all-reduce of the outcome)."""
    import torch.distributed as dist

    if info.world <= 1 or info.device.type != "cuda" or dist.get_backend() != "nccl":
        return None
    if "comm" not in _COMM:
        import torch

        from ..parallel.rccl import NativeComm
        try:
            comm = NativeComm.from_info(info)
        except Exception:  # noqa: BLE001 - the process group's own RCCL path still serves
            comm = None
        ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32, device=info.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        _COMM["comm"] = comm if int(ok.item()) else None
    return _COMM["comm"]
