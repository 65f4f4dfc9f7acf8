"""Live-driver GPU bench: the reference's actual loop, message in -> message published.

The reference's product is the subscriber callback: CompressedImage -> decode ->
preprocess -> ModelInfer -> NMS -> draw -> publish ``Image``
(``communicator/ros_inference.py:117-175``), and PointCloud2 -> ``read_points`` ->
voxelise -> ModelInfer -> filter -> jsk ``BoundingBoxArray`` -> publish
(``communicator/ros_inference3d.py:120-213``).  ``bench.py`` times the device step
from raw pinned bytes to device detections; this tool times the drivers
(:class:`RosInference` / :class:`RosInference3D`) with the local GPU engines over
the in-process topic bus, including JPEG decode, micro-batching, the ordered
re-publisher, GPU annotation and building the published messages.

    python tools/driver_bench.py [--camera N] [--lidar N] [--batch B] [--workers W] [--gpus N]

``--gpus N`` (N > 1) runs the drivers data-parallel the way ``torchrun main.py
--engine local`` does (``parallel/ring_dp.py``): rank 0 subscribes and publishes, the
node batch goes through the shared host ring, every rank decodes / detects its shard
on its own GPU.  Launched without torchrun it starts ``torch.distributed.run`` as a
child process; ``TCA_DIST_BACKEND=gloo`` rehearses N ranks on one GPU.

Messages are published paced so the latest-wins windows never drop (every
message is detected and published); throughput = messages / wall time from the
first publish to the last published result.  Prints one JSON line.
"""
import argparse
import io
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, ".")


class _Stages:
    """ClientMetrics stand-in: per-stage sums (StageTimer calls .stage / .frame)."""

    def __init__(self):
        self.sum, self.n, self.lock = {}, {}, threading.Lock()

    def stage(self, name, seconds):
        with self.lock:
            self.sum[name] = self.sum.get(name, 0.0) + seconds
            self.n[name] = self.n.get(name, 0) + 1

    def frame(self, n=1):
        pass

    def bytes(self, n):
        pass

    def summary(self):
        return {k: {"calls": self.n[k], "ms_per_call": round(1e3 * v / self.n[k], 3)} for k, v in self.sum.items()}


def _run(bus, pub_topic, out_topic, out_type, messages, window, timeout):
    from triton_client_amd.ros import compat

    got = []
    done = threading.Event()

    def on_out(m):
        got.append(time.perf_counter())
        if len(got) >= len(messages):
            done.set()
    sub = compat.Subscriber(out_topic, out_type, on_out, bus=bus)
    pub = compat.Publisher(pub_topic, type(messages[0]), bus=bus)
    t0 = time.perf_counter()
    for i, m in enumerate(messages):
        while i - len(got) >= window:  # pace: never more than `window` messages in flight
            time.sleep(0.0002)
        pub.publish(m)
    ok = done.wait(timeout)
    t1 = time.perf_counter()
    sub.unregister()
    return len(got), (t1 - t0), ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--camera", type=int, default=512, help="CompressedImage messages (0: skip)")
    ap.add_argument("--lidar", type=int, default=512, help="PointCloud2 messages (0: skip)")
    ap.add_argument("--batch", type=int, default=32, help="micro-batch per engine call")
    ap.add_argument("--workers", type=int, default=2, help="driver worker threads (host || device overlap)")
    ap.add_argument("--hw", default="720,1280")
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--gpus", type=int, default=1, help="data-parallel ranks (one process per GPU)")
    ap.add_argument("--engine", choices=["local", "remote"], default="local",
                    help="remote: the reference's architecture -- the drivers are KServe clients (RemoteDetector2D / "
                         "3D with their HIP pre/post on this GPU, main.py's default) of a server process started here "
                         "with YOLOv5nCOCO + pointpillar_kitti on the same GPU")
    ap.add_argument("--mode", choices=["sync", "async"], default="sync",
                    help="remote: RPC mode (sync = the reference's blocking ModelInfer; async = -a)")
    ap.add_argument("--wire", choices=["raw", "proto", "shm", "devshm"], default="raw",
                    help="remote: request codec / transport (shm, devshm: shared-memory regions, server on this node)")
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:  # self-launch (a child: nothing has touched the GPU)
        import socket
        import subprocess
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", __file__] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    from PIL import Image

    from triton_client_amd.inference.engines import LocalDetector2D, LocalDetector3D
    from triton_client_amd.inference.ros_inference import RosInference
    from triton_client_amd.inference.ros_inference3d import RosInference3D
    from triton_client_amd.ros import compat, msgs
    from triton_client_amd.ros.bus import TopicBus
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    from triton_client_amd.cli.engines import maybe_data_parallel

    H, W = (int(v) for v in a.hw.split(","))
    if a.engine == "remote":
        return _remote(a, H, W)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.device == "cuda" and world > 1:
        a.device = f"cuda:{int(os.environ.get('LOCAL_RANK', '0')) % max(1, torch.cuda.device_count())}"
    os.environ.setdefault("TCA_DP_HEARTBEAT", "0")
    # every rank builds both engines (and their DP wrappers) in the same order
    eng2, info = maybe_data_parallel(LocalDetector2D(batch=a.batch, device=a.device, letterbox=True)) \
        if a.camera else (None, None)
    eng3, info3 = maybe_data_parallel(LocalDetector3D(batch=a.batch, device=a.device), three_d=True) \
        if a.lidar else (None, None)
    info = info or info3
    if info is not None and not info.is_main:  # worker rank: serve shards until rank 0 is done
        for e in (eng2, eng3):
            if e is not None:
                e.serve()
        from triton_client_amd.parallel.dp import shutdown
        shutdown(info)
        return
    out = {"tool": "driver_bench", "batch": a.batch, "workers": a.workers, "gpus": world,
           "device": torch.cuda.get_device_name(0) if a.device.startswith("cuda") else a.device}
    bus = TopicBus()
    window = 2 * a.batch * a.workers
    if a.camera:
        jpegs = []
        for s in range(8):
            buf = io.BytesIO()
            Image.fromarray(camera_frame(H, W, s)).save(buf, format="JPEG", quality=90)
            jpegs.append(buf.getvalue())
        # header.seq strictly increasing over warm-up + run: the re-publisher drops a seq that is
        # not newer than the last one it published
        warm = 2 * a.batch
        msgs_in = [msgs.CompressedImage(header=msgs.Header(seq=i + 1, frame_id="cam"), format="jpeg",
                                        data=jpegs[i % 8]) for i in range(warm + a.camera)]
        st = _Stages()
        drv = RosInference(engine=eng2, params={"sub_topic": "/cam", "pub_topic": "/cam_out"}, bus=bus,
                           batch=a.batch, workers=a.workers, metrics=st, queue_size=window)
        drv.start_inference(spin=False)
        _run(bus, "/cam", "/cam_out", msgs.Image, msgs_in[:warm], window, a.timeout)  # warm-up + graphs
        st.sum.clear(), st.n.clear()
        n, dt, ok = _run(bus, "/cam", "/cam_out", msgs.Image, msgs_in[warm:], window, a.timeout)
        drv.stop()
        if info is not None:
            eng2.close()
        out["camera"] = {"messages": n, "complete": ok, "seconds": round(dt, 3), "msgs_per_s": round(n / dt, 1),
                         "input": f"CompressedImage JPEG {W}x{H} q90", "output": "annotated Image + Detection2DArray",
                         "stages": st.summary()}
    if a.lidar:
        spec = LidarSpec(sensor_height=3.23)
        clouds = [compat.create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, s).tobytes(), np.float32).reshape(-1, 4))
                  for s in range(8)]
        warm = 2 * a.batch
        msgs_in = []
        for i in range(warm + a.lidar):
            c = clouds[i % 8]
            msgs_in.append(msgs.PointCloud2(header=msgs.Header(seq=i + 1, frame_id="os"), height=c.height,
                                            width=c.width, fields=c.fields, is_bigendian=False,
                                            point_step=c.point_step, row_step=c.row_step, data=c.data,
                                            is_dense=True))
        st = _Stages()
        drv = RosInference3D(engine=eng3, params={"sub_topic": "/pc", "pub_topic": "/pc_out"}, bus=bus,
                             batch=a.batch, workers=a.workers, metrics=st, queue_size=window)
        drv.start_inference(spin=False)
        _run(bus, "/pc", "/pc_out", msgs.BoundingBoxArray, msgs_in[:warm], window, a.timeout)
        st.sum.clear(), st.n.clear()
        n, dt, ok = _run(bus, "/pc", "/pc_out", msgs.BoundingBoxArray, msgs_in[warm:], window, a.timeout)
        drv.stop()
        if info is not None:
            eng3.close()
        out["lidar"] = {"messages": n, "complete": ok, "seconds": round(dt, 3), "msgs_per_s": round(n / dt, 1),
                        "input": f"PointCloud2 {clouds[0].width} points x {clouds[0].point_step} B",
                        "output": "jsk BoundingBoxArray (label 2, score > 0.5)", "stages": st.summary()}
    bus.close()
    print(json.dumps(out), flush=True)
    if info is not None:
        from triton_client_amd.parallel.dp import shutdown
        shutdown(info)


def _camera_messages(H, W, n):
    from PIL import Image

    from triton_client_amd.ros import msgs
    from triton_client_amd.utils.synthetic import camera_frame

    jpegs = []
    for s in range(8):
        buf = io.BytesIO()
        Image.fromarray(camera_frame(H, W, s)).save(buf, format="JPEG", quality=90)
        jpegs.append(buf.getvalue())
    return [msgs.CompressedImage(header=msgs.Header(seq=i + 1, frame_id="cam"), format="jpeg", data=jpegs[i % 8])
            for i in range(n)]


def _cloud_messages(n):
    from triton_client_amd.ros import compat, msgs
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep

    spec = LidarSpec(sensor_height=3.23)
    clouds = [compat.create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, s).tobytes(), np.float32).reshape(-1, 4))
              for s in range(8)]
    out = []
    for i in range(n):
        c = clouds[i % 8]
        out.append(msgs.PointCloud2(header=msgs.Header(seq=i + 1, frame_id="os"), height=c.height, width=c.width,
                                    fields=c.fields, is_bigendian=False, point_step=c.point_step, row_step=c.row_step,
                                    data=c.data, is_dense=True))
    return out


def _remote(a, H, W):
    """--engine remote: a KServe server process on this GPU; the drivers as its clients
    (RemoteDetector2D / RemoteDetector3D on the GPU: main.py / main3d.py's default path)."""
    import socket
    import subprocess
    from types import SimpleNamespace

    import torch

    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import client_for_model
    from triton_client_amd.inference.engines import RemoteDetector2D, RemoteDetector3D
    from triton_client_amd.inference.ros_inference import RosInference
    from triton_client_amd.inference.ros_inference3d import RosInference3D
    from triton_client_amd.ros import msgs
    from triton_client_amd.ros.bus import TopicBus

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    target = f"127.0.0.1:{port}"
    proc = subprocess.Popen([sys.executable, "-m", "triton_client_amd.server", "--host", "127.0.0.1", "--port",
                             str(port), "--metrics-port", "0", "--models", "YOLOv5nCOCO,pointpillar_kitti"])
    out = {"tool": "driver_bench", "engine": "remote", "mode": a.mode, "wire": a.wire, "batch": a.batch,
           "workers": a.workers, "device": torch.cuda.get_device_name(0) if a.device.startswith("cuda") else a.device,
           "server": "separate process, same GPU: YOLOv5nCOCO + pointpillar_kitti (fp32)"}
    try:
        def channel(model):
            f = SimpleNamespace(model_name=model, model_version="", batch_size=1, verbose=False)
            return GRPCChannel({"grpc_channel": target}, f, wait_ready_s=600.0)

        bus = TopicBus()
        window = 2 * a.batch * a.workers
        if a.camera:
            ch = channel("YOLOv5nCOCO")
            cr = ch.get_metadata()["config_response"]
            client = client_for_model("YOLOv5nCOCO", getattr(cr, "config", cr), a.device)
            eng = RemoteDetector2D(ch, client, letterbox=False, conf_thres=0.3, mode=a.mode, wire=a.wire,
                                   device=a.device)
            warm = 2 * a.batch
            ms = _camera_messages(H, W, warm + a.camera)
            st = _Stages()
            drv = RosInference(None, client, engine=eng, params={"sub_topic": "/cam", "pub_topic": "/cam_out"},
                               bus=bus, batch=a.batch, workers=a.workers, metrics=st, queue_size=window)
            drv.start_inference(spin=False)
            _run(bus, "/cam", "/cam_out", msgs.Image, ms[:warm], window, a.timeout)
            st.sum.clear(), st.n.clear()
            n, dt, ok = _run(bus, "/cam", "/cam_out", msgs.Image, ms[warm:], window, a.timeout)
            drv.stop()
            live = eng.live()
            eng.release_transport()
            out["camera"] = {"messages": n, "complete": ok, "seconds": round(dt, 3), "msgs_per_s": round(n / dt, 1),
                             "device_path": live is not None and live.stats["frames"] > 0,
                             "input": f"CompressedImage JPEG {W}x{H} q90", "output": "annotated Image + Detection2DArray",
                             "stages": st.summary()}
            ch.close()
        if a.lidar:
            ch = channel("pointpillar_kitti")
            cr = ch.get_metadata()["config_response"]
            client = client_for_model("pointpillar_kitti", getattr(cr, "config", cr), a.device)
            eng = RemoteDetector3D(ch, client, z_offset=1.5, mode=a.mode, wire=a.wire, device=a.device)
            warm = 2 * a.batch
            ms = _cloud_messages(warm + a.lidar)
            st = _Stages()
            drv = RosInference3D(None, client, engine=eng, params={"sub_topic": "/pc", "pub_topic": "/pc_out"},
                                 bus=bus, batch=a.batch, workers=a.workers, metrics=st, queue_size=window)
            drv.start_inference(spin=False)
            _run(bus, "/pc", "/pc_out", msgs.BoundingBoxArray, ms[:warm], window, a.timeout)
            st.sum.clear(), st.n.clear()
            n, dt, ok = _run(bus, "/pc", "/pc_out", msgs.BoundingBoxArray, ms[warm:], window, a.timeout)
            drv.stop()
            eng.release_transport()
            out["lidar"] = {"messages": n, "complete": ok, "seconds": round(dt, 3), "msgs_per_s": round(n / dt, 1),
                            "device_voxeliser": str(getattr(eng.pre, "device", "cpu")),
                            "input": f"PointCloud2 {ms[0].width} points x {ms[0].point_step} B",
                            "output": "jsk BoundingBoxArray (label 2, score > 0.5)", "stages": st.summary()}
            ch.close()
        bus.close()
        print(json.dumps(out), flush=True)
    finally:
        proc.terminate()
        try:
            proc.wait(60)
        except subprocess.TimeoutExpired:
            proc.kill()


if __name__ == "__main__":
    main()
