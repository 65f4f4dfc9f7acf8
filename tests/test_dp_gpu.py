"""Device-resident data parallelism on a GPU box: two ranks share the one
card over host-staged gloo (RCCL refuses two ranks on one device).  The node
batch goes through the shared host ring and each rank runs its shard on its
live device path — the engine's host API (numpy frames in) raises if it is
called on a worker — and rank 0's gathered detections must be bit-identical
to a single-rank run on the same frames (same weights, same kernels)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(240, exit=True)
    try:
        import torch

        from triton_client_amd.inference.engines import LocalDetector2D, LocalDetector3D
        from triton_client_amd.parallel.dp import DataParallelDetector2D, DataParallelDetector3D, init_distributed
        from triton_client_amd.ros.compat import create_cloud_xyzi
        from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

        info = init_distributed("gloo")
        d2 = LocalDetector2D(batch=2, device=info.device)
        d3 = LocalDetector3D(batch=2, device=info.device, max_points=32768)
        # no per-rank calibration: rank 0 calibrates on the first frame and broadcasts
        if rank != 0:
            def no_host(*a, **k):
                raise AssertionError("worker rank used the host detect() path")
            d2.detect = no_host
            d3.detect = no_host
        dp2 = DataParallelDetector2D(d2, info, max_det=300)
        dp3 = DataParallelDetector3D(d3, info, max_out=500)
        spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
        if info.is_main:
            frames = [camera_frame(360, 640, 100 + i) for i in range(5)]
            clouds = [create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, 200 + i).tobytes(), np.float32).reshape(-1, 4))
                      for i in range(3)]
            got2 = dp2.detect(frames)
            dp2.close()  # the two detectors share the p2p channel: rank 1 moves on to dp3.serve()
            got3 = dp3.detect(clouds)
            dp3.close()
            want2 = d2.detect(frames)
            want3 = d3.detect(clouds)
            assert all(len(w) > 0 for w in want2) and all(len(w["pred_scores"]) > 0 for w in want3)
            for g, w in zip(got2, want2):
                np.testing.assert_array_equal(g, w)
            for g, w in zip(got3, want3):
                for k in ("pred_boxes", "pred_scores", "pred_labels"):
                    np.testing.assert_array_equal(g[k], w[k])
            q.put((0, "ok"))
        else:
            n2 = dp2.serve()
            n3 = dp3.serve()
            q.put((rank, f"served {n2} {n3}"))
        torch.cuda.synchronize()
        q.close()
        q.join_thread()
        os._exit(0)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


def test_dp_device_resident_two_ranks(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res == {0: "ok", 1: "served 1 1"}, res


def _family_worker(rank, world, port, q, family):
    """Every reference family on the device-resident DP path: rank 0's gathered
    detections vs a single-rank run of the same engine on the same inputs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import faulthandler
    faulthandler.dump_traceback_later(280, exit=True)
    try:
        import torch

        from triton_client_amd.inference.engines import LocalDetector2D, LocalDetector3D
        from triton_client_amd.parallel.dp import DataParallelDetector2D, DataParallelDetector3D, init_distributed
        from triton_client_amd.ros.compat import create_cloud_xyzi
        from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

        info = init_distributed("gloo")
        three_d = family in ("centerpoint", "second_iou")
        if three_d:
            det = LocalDetector3D(batch=2, device=info.device, max_points=65536, family=family)
            dp = DataParallelDetector3D(det, info, max_out=500, box_dim=det.box_dim)
        else:
            det = LocalDetector2D(batch=2, device=info.device, family=family, img=(640, 480) if family != "yolov4"
                                  else 512, nc=80)
            dp = DataParallelDetector2D(det, info, max_det=300)
        if rank != 0:
            def no_host(*a, **k):
                raise AssertionError("worker rank used the host detect() path")
            det.detect = no_host
        if info.is_main:
            if three_d:
                spec = LidarSpec(rings=32, azimuth_steps=1800, sensor_height=1.8)
                items = [create_cloud_xyzi(np.frombuffer(lidar_sweep(spec, 300 + i).tobytes(), np.float32)
                                           .reshape(-1, 4)) for i in range(3)]
            else:
                items = [camera_frame(360, 640, 400 + i) for i in range(3)]
            got = dp.detect(items)
            dp.close()
            want = det.detect(items)
            for g, w in zip(got, want):  # bit-identical to the single-rank run
                if three_d:
                    assert len(w["pred_scores"]) > 0 and g["pred_boxes"].shape[1] == det.box_dim
                    for k in ("pred_boxes", "pred_scores", "pred_labels"):
                        np.testing.assert_array_equal(g[k], w[k])
                else:
                    assert len(w) > 0
                    np.testing.assert_array_equal(g, w)
            q.put((0, "ok"))
        else:
            q.put((rank, f"served {dp.serve()}"))
        torch.cuda.synchronize()
        q.close()
        q.join_thread()
        os._exit(0)
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
        q.close()
        q.join_thread()
        os._exit(1)


@pytest.mark.parametrize("family", ["centerpoint", "second_iou", "retinanet", "fcos", "yolov4"])
def test_dp_families_two_ranks(cuda, family):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_family_worker, args=(r, 2, port, q, family)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res == {0: "ok", 1: "served 1"}, res
