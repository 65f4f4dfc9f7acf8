"""Two-rank gloo rehearsal of the ring DP detectors on one GPU, with progress
lines and a traceback dump of every rank after --dump seconds (diagnostics for a
hang: which call each rank is in).

    python tools/dp_debug.py [--dump 100] [--three-d]
"""
import argparse
import os
import socket
import sys
import time

sys.path.insert(0, ".")


def log(rank, msg):
    print(f"[{time.strftime('%H:%M:%S')}] rank{rank}: {msg}", flush=True)


def worker(rank, world, port, dump, three_d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(dump, exit=True, file=sys.stdout)
    import numpy as np
    import torch

    from triton_client_amd.inference.engines import LocalDetector2D, LocalDetector3D
    from triton_client_amd.parallel.dp import DataParallelDetector2D, DataParallelDetector3D, init_distributed
    from triton_client_amd.ros.compat import create_cloud_xyzi
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

    log(rank, f"affinity before init: {len(os.sched_getaffinity(0))} cpus")
    info = init_distributed("gloo")
    log(rank, f"init done, affinity {len(os.sched_getaffinity(0))} cpus")
    if three_d:
        det = LocalDetector3D(batch=2, device=info.device, max_points=32768)
    else:
        det = LocalDetector2D(batch=2, device=info.device)
    # no per-rank calibration: rank 0 calibrates on its first frame and broadcasts
    dp = (DataParallelDetector3D if three_d else DataParallelDetector2D)(det, info)
    log(rank, f"ring {dp.ring.name} attached")
    if info.is_main:
        if three_d:
            spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
            items = [create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, 200 + i).tobytes(), np.float32)
                                       .reshape(-1, 4)) for i in range(3)]
        else:
            items = [camera_frame(360, 640, 100 + i) for i in range(5)]
        t0 = time.perf_counter()
        got = dp.detect(items)
        log(rank, f"detect done in {time.perf_counter() - t0:.1f}s: {[len(g) for g in got]}")
        dp.close()
        log(rank, "closed")
    else:
        n = dp.serve()
        log(rank, f"served {n}")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    os._exit(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", type=int, default=100)
    ap.add_argument("--three-d", action="store_true")
    a = ap.parse_args()
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, 2, port, a.dump, a.three_d)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(a.dump + 30)
    codes = [p.exitcode for p in ps]
    print("exit codes", codes, flush=True)
    sys.exit(0 if codes == [0, 0] else 1)


if __name__ == "__main__":
    main()
