#!/usr/bin/env python3
"""Served-path throughput: the reference's architecture (client → KServe-v2
gRPC → server → client), with this framework's zero-copy served path.

Client (``inference/engines.py`` RemoteDetector2D/3D, ``--device cuda``):
camera frame → pinned → GPU K1 preprocess → pinned staging → C++ encoder
writes the request bytes directly (one host copy of the tensor); LiDAR
PointCloud2 bytes → GPU unpack + spconv-order voxeliser → pinned staging →
C++ encoder.  Requests go as a window of gRPC futures (``-a``).
Server (``server/kserve_server.py`` ModelInferBytes): the C++ codec parses
the request bytes into views, the model copies them once into pinned
staging → DMA → captured GPU pipeline → pinned output staging → the C++
encoder writes the response.  Client parses the response into views.

Camera and LiDAR clients run concurrently (two threads: the reference runs
them as two ROS nodes) against one in-process server on 127.0.0.1; one
frame pair = one camera frame + one LiDAR sweep.  Prints one JSON line with
frame pairs/s and per-stage milliseconds; ``--reference`` also runs
tools/reference_equivalent.py's per-frame protocol for the ratio.

    python tools/served_bench.py --frames 64 [--window 8] [--device cuda]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--window", type=int, default=8, help="requests in flight per client")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--cam", default="720x1280")
    ap.add_argument("--rings", type=int, default=64)
    ap.add_argument("--columns", type=int, default=1875)
    ap.add_argument("--workers", type=int, default=32, help="server threads")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--wire", default="raw", choices=("raw", "shm", "devshm"),
                    help="raw: tensors in the gRPC messages (C++ codec); shm: KServe system shared memory; "
                         "devshm: device shared memory (GPU buffers shared by HIP IPC handle, Triton's CUDA shm)")
    ap.add_argument("--server-process", action="store_true",
                    help="run the server as its own process (the deployed topology: no GIL shared with the clients)")
    ap.add_argument("--client-procs", type=int, default=0,
                    help="P > 0: P camera + P LiDAR client processes (the reference runs each sensor client as its "
                         "own ROS node), each streaming --frames frames; implies --server-process")
    ap.add_argument("--burst", action="store_true",
                    help="drain the window every --window frames (the previous protocol) instead of a sliding window")
    ap.add_argument("--role", default=None, choices=("camera", "lidar"), help=argparse.SUPPRESS)
    ap.add_argument("--target", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--seed", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--server-procs", type=int, default=1, help="server processes sharing the port (--procs)")
    ap.add_argument("--model-procs", action="store_true",
                    help="one server process per model, each on its own port (camera clients -> the YOLOv5 "
                         "server, LiDAR clients -> the PointPillars server): two GILs, and each model's dynamic "
                         "batcher still sees all of its requests")
    ap.add_argument("--client-hw-queues", type=int, default=0,
                    help="multi-process runs: GPU_MAX_HW_QUEUES of each client process (0: HIP's default); fewer "
                         "queues per client leave more of the hardware scheduler's mapped queues to the server")
    ap.add_argument("--server-profile", default=None, metavar="JSON",
                    help="multi-process runs: the server's stage clock (TCA_SERVER_PROFILE) written here")
    a = ap.parse_args(argv)
    if a.role is not None:
        return client_proc(a)
    if a.client_procs > 0:
        return multi_proc(a)

    import torch

    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov5client, client_for_model
    from triton_client_amd.inference.engines import RemoteDetector2D, RemoteDetector3D
    from triton_client_amd.ros import compat
    from triton_client_amd.server import KServeServer, ModelRepository
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    H0, W0 = (int(v) for v in a.cam.split("x"))
    proc = repo = srv = None
    if a.server_process:
        import socket
        import subprocess

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        target = f"127.0.0.1:{port}"
        proc = subprocess.Popen([sys.executable, "-m", "triton_client_amd.server", "--host", "127.0.0.1", "--port",
                                 str(port), "--workers", str(a.workers), "--metrics-port", "0", "--device", a.device,
                                 "--models", "YOLOv5nCOCO,pointpillar_kitti"])
    else:
        repo = ModelRepository(a.device)
        repo.load("YOLOv5nCOCO")
        repo.load("pointpillar_kitti")
        srv = KServeServer(repo, "127.0.0.1:0", max_workers=a.workers).start()
        target = srv.target

    def channel(model):
        flags = SimpleNamespace(model_name=model, model_version="", batch_size=64, verbose=False)
        ch = GRPCChannel({"grpc_channel": target}, flags, wait_ready_s=300.0) if proc else \
            GRPCChannel({"grpc_channel": target}, flags)
        return ch

    ch2, ch3 = channel("YOLOv5nCOCO"), channel("pointpillar_kitti")
    cr3 = ch3.get_metadata()["config_response"]
    det2 = RemoteDetector2D(ch2, Yolov5client(), letterbox=False, conf_thres=0.3, mode="async", wire=a.wire,
                            device=a.device)
    det3 = RemoteDetector3D(ch3, client_for_model("pointpillar_kitti", getattr(cr3, "config", cr3)), z_offset=1.5,
                            mode="async", wire=a.wire, device=a.device)
    det2.window = det3.window = a.window
    n = a.frames + a.warmup
    frames = [camera_frame(H0, W0, s) for s in range(8)]
    spec = LidarSpec(rings=a.rings, azimuth_steps=a.columns, sensor_height=3.23)
    clouds = [compat.create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, 500 + s).tobytes(), np.float32).reshape(-1, 4))
              for s in range(8)]

    def run(det, items, count, out):
        out.append(stream_frames(det, items, count, a.window, a.burst))

    # warm-up (graph capture, calibration, connection setup), then timed
    run(det2, frames, a.warmup, [])
    run(det3, clouds, a.warmup, [])
    det2.timer, det3.timer = {}, {}
    r2, r3 = [], []
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(det2, frames, a.frames, r2)),
          threading.Thread(target=run, args=(det3, clouds, a.frames, r3))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    stats = {}
    for m in ("YOLOv5nCOCO", "pointpillar_kitti"):  # from the server (either topology) over the stats RPC
        ms_ = ch2.model_statistics(m).model_stats[0]
        stats[m] = SimpleNamespace(compute_ns=ms_.inference_stats.compute_infer.ns, inference_count=ms_.inference_count,
                                   execution_count=ms_.execution_count)
    for d in (det2, det3):
        if hasattr(d, "close_shm"):
            d.close_shm()
    if srv is not None:
        srv.stop()
    if proc is not None:
        proc.terminate()
        proc.wait(30)

    def ms(timer):
        return {k: round(1e3 * float(np.sum(v)) / a.frames, 3) for k, v in timer.items()}

    n2 = float(np.mean([len(d) for res in r2 for d in res]))
    n3 = float(np.mean([len(d["pred_scores"]) for res in r3 for d in res]))
    line = {"metric": "served-path frame pairs/s (camera + LiDAR over KServe gRPC, localhost)",
            "value": round(a.frames / wall, 2), "unit": "frame pairs/s", "frames": a.frames, "window": a.window,
            "wall_s": round(wall, 3), "device": a.device,
            "client_ms_per_frame": {"camera": ms(det2.timer), "lidar": ms(det3.timer)},
            "server_compute_ms_per_request": {m: round(s.compute_ns / max(1, s.inference_count) / 1e6, 3)
                                              for m, s in stats.items()},
            "server_requests_per_execution": {m: round(s.inference_count / max(1, s.execution_count), 2)
                                              for m, s in stats.items()},
            "topology": "server process + client process" if proc else "one process", "wire": a.wire,
            "window_mode": "burst" if a.burst else "sliding",
            "avg_dets_per_frame": {"2d": round(n2, 1), "3d": round(n3, 1)},
            "path": ("GPU preprocess/voxelise -> pinned shared-memory slot (KServe system shared memory) -> "
                     "gRPC message with region references -> server view of the region -> pinned -> GPU model -> "
                     "2D output written into the client's region / 3D outputs in the message") if a.wire == "shm" else
                    ("GPU preprocess/voxelise -> pinned staging -> C++ KServe encoder -> gRPC -> C++ parse -> pinned "
                     "-> GPU model -> pinned -> C++ encoder -> gRPC -> zero-copy response views")}
    print(json.dumps(line), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(line) + "\n")
    return 0


def stream_frames(det, items, count, window, burst=False):
    """Send ``count`` frames (cycling over ``items``) through ``det``: one
    detect() call, so its window of in-flight requests stays full (a sensor
    stream), or with ``burst`` one call per ``window`` frames."""
    if not burst:
        return det.detect([items[i % len(items)] for i in range(count)])
    res, done = [], 0
    while done < count:
        k = min(window, count - done)
        res += det.detect([items[(done + i) % len(items)] for i in range(k)])
        done += k
    return res


def _sensor_data(a, seed0=0):
    from triton_client_amd.ros import compat
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    H0, W0 = (int(v) for v in a.cam.split("x"))
    frames = [camera_frame(H0, W0, seed0 + s) for s in range(8)]
    spec = LidarSpec(rings=a.rings, azimuth_steps=a.columns, sensor_height=3.23)
    clouds = [compat.create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, seed0 + 500 + s).tobytes(), np.float32)
                                       .reshape(-1, 4)) for s in range(8)]
    return frames, clouds


def _detector(a, target, role, wait_ready_s=300.0):
    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov5client, client_for_model
    from triton_client_amd.inference.engines import RemoteDetector2D, RemoteDetector3D

    model = "YOLOv5nCOCO" if role == "camera" else "pointpillar_kitti"
    flags = SimpleNamespace(model_name=model, model_version="", batch_size=64, verbose=False)
    ch = GRPCChannel({"grpc_channel": target}, flags, wait_ready_s=wait_ready_s)
    if role == "camera":
        det = RemoteDetector2D(ch, Yolov5client(), letterbox=False, conf_thres=0.3, mode="async", wire=a.wire,
                               device=a.device)
    else:
        cr3 = ch.get_metadata()["config_response"]
        det = RemoteDetector3D(ch, client_for_model(model, getattr(cr3, "config", cr3)), z_offset=1.5,
                               mode="async", wire=a.wire, device=a.device)
    det.window = a.window
    return ch, det


def client_proc(a) -> int:
    """One sensor client process: warm up, report READY, wait for GO on stdin,
    stream --frames frames, report its stage times and detection counts."""
    frames, clouds = _sensor_data(a, 1000 * a.seed)
    ch, det = _detector(a, a.target, a.role)
    items = frames if a.role == "camera" else clouds
    stream_frames(det, items, a.warmup, a.window, a.burst)
    det.timer = {}
    print("READY", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    res = stream_frames(det, items, a.frames, a.window, a.burst)
    wall = time.perf_counter() - t0
    if hasattr(det, "close_shm"):
        det.close_shm()
    n = float(np.mean([len(d) if a.role == "camera" else len(d["pred_scores"]) for d in res]))
    print(json.dumps({"role": a.role, "wall_s": wall, "frames": len(res), "dets": n,
                      "ms": {k: 1e3 * float(np.sum(v)) / a.frames for k, v in det.timer.items()}}), flush=True)
    return 0


def multi_proc(a) -> int:
    """Server process + P camera and P LiDAR client processes; the clock runs
    from GO to the last client's last response."""
    import socket
    import subprocess

    def free_port():
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            return sk.getsockname()[1]

    here = os.path.abspath(__file__)
    models = {"camera": "YOLOv5nCOCO", "lidar": "pointpillar_kitti"}
    groups = [list(models.values())] if not a.model_procs else [[m] for m in models.values()]
    servers, targets = [], {}
    for i, g in enumerate(groups):
        port = free_port()
        env = dict(os.environ)
        if a.server_profile:
            prof = os.path.abspath(a.server_profile)
            env["TCA_SERVER_PROFILE"] = prof if len(groups) == 1 else prof.replace(".json", f"_{g[0]}.json")
        servers.append(subprocess.Popen(
            [sys.executable, "-X", "faulthandler", "-m", "triton_client_amd.server", "--host", "127.0.0.1", "--port",
             str(port), "--workers", str(a.workers), "--metrics-port", "0", "--device", a.device,
             "--models", ",".join(g), "--procs", str(a.server_procs)],
            cwd=os.path.dirname(os.path.dirname(here)), env=env))
        for m in g:
            targets[m] = f"127.0.0.1:{port}"
    common = ["--frames", str(a.frames), "--warmup", str(a.warmup), "--window", str(a.window), "--device", a.device,
              "--cam", a.cam, "--rings", str(a.rings), "--columns", str(a.columns), "--wire", a.wire] + \
        (["--burst"] if a.burst else [])
    clients = []
    cenv = dict(os.environ, **({"GPU_MAX_HW_QUEUES": str(a.client_hw_queues)} if a.client_hw_queues > 0 else {}))
    try:
        for p in range(a.client_procs):
            for role in ("camera", "lidar"):
                clients.append(subprocess.Popen([sys.executable, here, "--role", role, "--seed", str(p), "--target",
                                                 targets[models[role]]] + common,
                                                stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                                env=cenv))
        for c in clients:
            line = c.stdout.readline()
            if line.strip() != "READY":
                raise RuntimeError(f"client failed before READY: {line!r} "
                                   f"(server exit codes {[s.poll() for s in servers]})")
        import psutil

        procs = [psutil.Process(s.pid) for s in servers] + [psutil.Process(c.pid) for c in clients]

        def cpu_s():  # user + system seconds of the server (and its children) and the clients
            tot = 0.0
            for p in procs:
                try:
                    for q in [p] + p.children(recursive=True):
                        t = q.cpu_times()
                        tot += t.user + t.system
                except psutil.NoSuchProcess:
                    pass
            return tot
        c0 = cpu_s()
        t0 = time.perf_counter()
        for c in clients:
            c.stdin.write("GO\n")
            c.stdin.flush()
        outs = [json.loads(c.stdout.readline()) for c in clients]
        wall = time.perf_counter() - t0
        cpu_cores = (cpu_s() - c0) / wall
        try:
            cpu_avail = len(os.sched_getaffinity(0))
        except AttributeError:
            cpu_avail = os.cpu_count()
        for c in clients:
            if c.wait(60) != 0:
                raise RuntimeError("a client process failed")
        from triton_client_amd.channel.grpc_channel import GRPCChannel

        rpe = {}
        for m in models.values():
            ch = GRPCChannel({"grpc_channel": targets[m]}, SimpleNamespace(model_name=m, model_version="",
                                                                           batch_size=64, verbose=False))
            st = ch.model_statistics(m).model_stats[0]
            rpe[m] = round(st.inference_count / max(1, st.execution_count), 2)
    finally:
        for c in clients:
            if c.poll() is None:
                c.kill()
        for server in servers:
            server.terminate()
        for server in servers:
            try:
                server.wait(30)
            except subprocess.TimeoutExpired:  # e.g. under a tracer that flushes at exit: the results stand
                server.kill()
                server.wait(30)

    def mean_ms(role):
        rs = [o for o in outs if o["role"] == role]
        return {k: round(float(np.mean([o["ms"][k] for o in rs])), 3) for k in rs[0]["ms"]}

    pairs = a.client_procs * a.frames
    line = {"metric": "served-path frame pairs/s (camera + LiDAR over KServe gRPC, localhost)",
            "value": round(pairs / wall, 2), "unit": "frame pairs/s", "frames": pairs, "window": a.window,
            "wall_s": round(wall, 3), "device": a.device,
            "client_ms_per_frame": {"camera": mean_ms("camera"), "lidar": mean_ms("lidar")},
            "client_wall_s": {o["role"] + str(i // 2): round(o["wall_s"], 3) for i, o in enumerate(outs)},
            "server_requests_per_execution": rpe,
            "host_cpu_cores_busy": round(cpu_cores, 2), "host_cpus_in_affinity": cpu_avail,
            "topology": ((f"one server process per model ({a.server_procs} each)" if a.model_procs else
                          f"{a.server_procs} server process{'es' if a.server_procs > 1 else ''}") +
                         f" + {a.client_procs} camera and {a.client_procs} LiDAR client processes"),
            "wire": a.wire, "window_mode": "burst" if a.burst else "sliding", "server_workers": a.workers,
            "client_hw_queues": a.client_hw_queues or None,
            "path": {"raw": "tensors inside the gRPC messages (C++ codec both ends)",
                     "shm": "GPU preprocess -> page-locked /dev/shm slot -> region references in the message -> "
                            "server DMA from / into the client's slot",
                     "devshm": "GPU preprocess into the client's device buffer (HIP IPC handle registered with the "
                               "server) -> region references in the message -> server copies device to device, "
                               "writes the 2D output into the client's device buffer; only detections cross PCIe"
                     }[a.wire],
            "avg_dets_per_frame": {"2d": round(float(np.mean([o["dets"] for o in outs if o["role"] == "camera"])), 1),
                                   "3d": round(float(np.mean([o["dets"] for o in outs if o["role"] == "lidar"])), 1)}}
    print(json.dumps(line), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(line) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
