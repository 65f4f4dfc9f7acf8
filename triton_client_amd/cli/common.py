"""Shared command-line surface of the entry points.

The reference's flags are kept with the same names and defaults
(``main.py:51-113``; identical in ``main3d.py``, ``bag2d.py``,
``bag3d.py``): ``-v``, ``-a/--async``, ``--streaming``, ``-m``, ``-x``,
``-b``, ``-c``, ``-s``, ``-i``.  Additions are listed in ``--help``:

* the engine — ``remote`` (a KServe/Triton server, as in the reference) or
  ``local`` (in-process MI355X pipeline);
* the client parameter file.  The reference read it through the rosparam
  ``client_parameter_file`` (``main.py:119-121``);
* the bag paths.  The reference hard-coded them;
* ``--client``, which picks the client by model family.  The reference
  always used YOLOv5 (A1).
"""
from __future__ import annotations

import argparse
import logging
import os
from typing import Optional

import yaml

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "data")


def add_reference_flags(p: argparse.ArgumentParser, default_model: str = "YOLOv5n") -> None:
    p.add_argument("-v", "--verbose", action="store_true", default=False, help="Enable verbose output")
    p.add_argument("-a", "--async", dest="async_set", action="store_true", default=False,
                   help="Use asynchronous inference API")
    p.add_argument("--streaming", action="store_true", default=False, help="Use streaming inference API")
    p.add_argument("-m", "--model-name", type=str, default=default_model, help="Name of model")
    p.add_argument("-x", "--model-version", type=str, default="",
                   help="Version of model. Default is to use latest version.")
    p.add_argument("-b", "--batch-size", type=int, default=1, help="Batch size. Default is 1.")
    p.add_argument("-c", "--classes", type=int, default=80, help="Number of class results to report.")
    p.add_argument("-s", "--scaling", type=str, choices=["NONE", "INCEPTION", "VGG", "COCO"], default="COCO",
                   help="Type of scaling to apply to image pixels.")
    p.add_argument("-i", "--image-src", type=str, choices=["ros", "local"], default="ros",
                   help="Source of input: the ROS topic (or a replayed bag) or local image files")


def add_framework_flags(p: argparse.ArgumentParser, params_default: str, three_d: bool = False) -> None:
    g = p.add_argument_group("triton_client_amd")
    g.add_argument("--params", default=params_default, help="client parameter YAML (grpc_channel, topics)")
    g.add_argument("--engine", choices=["remote", "local"], default="remote",
                   help="remote: KServe/Triton server at grpc_channel; local: in-process MI355X pipeline")
    g.add_argument("--client", choices=["auto", "yolov5", "fcos", "pointpillars"], default="auto",
                   help="model-family client (auto: from the model's config)")
    g.add_argument("--server", default=None, help="override grpc_channel host:port")
    g.add_argument("--device", default="auto",
                   help="where the engine runs: the local pipeline, or the remote client's decode / preprocess / "
                        "postprocess HIP kernels (auto: the first GPU if there is one; cuda:N; cpu)")
    g.add_argument("--frames-per-step", type=int, default=8, help="micro-batch for bag replay / local engine")
    g.add_argument("--live-batch", type=int, default=1,
                   help="live topic: run up to N pending frames per engine call (latest-wins window, "
                        "re-published in header.seq order); 1 = the reference's one frame per callback")
    g.add_argument("--live-workers", type=int, default=1,
                   help="live topic: micro-batches in flight (host work of one overlaps another's GPU work)")
    g.add_argument("--wire", choices=["raw", "proto", "shm", "devshm"], default="raw",
                   help="raw: C++ zero-copy KServe codec; proto: reference-style protobuf request; shm: KServe "
                        "system shared memory (server on the same host; tensors stay in a /dev/shm region); "
                        "devshm: KServe device shared memory (server on the same GPU node; the model input and "
                        "outputs stay in a GPU allocation the server maps by HIP IPC handle -- needs --device cuda)")
    g.add_argument("--timeout", type=float, default=None, help="per-RPC deadline (s); default none")
    g.add_argument("--retries", type=int, default=2, help="retries on UNAVAILABLE/DEADLINE_EXCEEDED")
    g.add_argument("--weights", default=None, help="state_dict for the local engine: path, file://, http(s):// or s3:// URI (loaded with torch.load weights_only)")
    g.add_argument("--export-weights", default=None,
                   help="local engine: after the run, save its fused, calibrated weights here (reload with --weights "
                        "to reproduce them exactly, e.g. on every rank or host of a deployment)")
    g.add_argument("--play", default=None, help="replay this bag onto the in-process topic bus (no rospy)")
    g.add_argument("--spin-timeout", type=float, default=None, help="stop spinning after N seconds")
    g.add_argument("--metrics-port", type=int, default=None, help="Prometheus exporter port for client metrics")
    if three_d:
        g.add_argument("--detection3d", action="store_true", help="publish vision_msgs/Detection3DArray, not jsk")
        g.add_argument("--labels", default="2", help="labels to publish (comma list, 'all'); reference: 2")
        g.add_argument("--score-thresh", type=float, default=0.5, help="publish threshold (reference 0.5)")
        g.add_argument("--z-offset", type=float, default=1.5, help="z added before voxelising (reference 1.5)")
    else:
        g.add_argument("--letterbox", action="store_true", help="letterbox instead of the reference's stretch")
        g.add_argument("--conf-thres", type=float, default=0.3, help="reference: 0.3")
        g.add_argument("--images", default=None, help="directory of images for -i local")


def load_params(path: Optional[str], server: Optional[str] = None) -> dict:
    from ..ros import compat

    path = compat.get_param("client_parameter_file", path) or path
    with open(path) as f:
        params = yaml.safe_load(f)
    if server:
        params["grpc_channel"] = server
    return params


def setup_logging(verbose: bool) -> None:
    logging.basicConfig(level=logging.DEBUG if verbose else logging.INFO,
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")


def make_channel(params: dict, flags):
    from ..channel.grpc_channel import GRPCChannel

    return GRPCChannel(params, flags, timeout_s=getattr(flags, "timeout", None), retries=getattr(flags, "retries", 2))


def resolve_device(flag: Optional[str]) -> str:
    """``--device``: "auto" is the first visible GPU when there is one, else the CPU
    (config 1, the CPU-only client); anything else is taken as given."""
    if flag in (None, "", "auto"):
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"
    return flag


def make_client(flags, channel=None):
    """The model-family client, its pre/postprocess on ``--device`` (the remote
    engine's HIP path on a GPU client)."""
    from ..clients import FCOS_client, Pointpillars_client, Yolov5client, client_for_model

    dev = resolve_device(getattr(flags, "device", "cpu"))
    c = getattr(flags, "client", "auto")
    if c == "yolov5":
        return Yolov5client(dev)
    if c == "fcos":
        return FCOS_client(dev)
    if c == "pointpillars":
        return Pointpillars_client(dev)
    cfg = None
    if channel is not None:
        cr = channel.get_metadata().get("config_response")
        cfg = getattr(cr, "config", cr)
    return client_for_model(flags.model_name, cfg, dev)


def rpc_mode(flags) -> str:
    return "stream" if flags.streaming else "async" if flags.async_set else "sync"


def labels_arg(s: str):
    return None if s in ("all", "", "none") else tuple(int(v) for v in s.split(","))


def play_bag(path: str, bus, topics=None, rate: Optional[float] = None, shutdown: bool = True):
    """rosbag-play equivalent onto the in-process bus (background thread)."""
    import threading
    import time

    from ..ros.bag import Bag

    def run():
        t_prev = None
        with Bag(path) as bag:
            for topic, msg, t in bag.read_messages(topics=topics):
                if rate and t_prev is not None:
                    time.sleep(max(0.0, (t.to_sec() - t_prev) / rate))
                t_prev = t.to_sec()
                bus.publish(topic, msg)
        bus.wait_idle(600)
        if shutdown:
            bus.shutdown_event.set()

    th = threading.Thread(target=run, daemon=True, name="bag-play")
    th.start()
    return th


def image_files(d: str):
    exts = (".png", ".jpg", ".jpeg", ".bmp")
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.lower().endswith(exts))
