#!/usr/bin/env python3
"""Reference-equivalent end-to-end FPS (SURVEY §6 protocol).

The reference publishes no throughput numbers, so the denominator for
``bench.py``'s ``vs_baseline`` is measured: the same synthetic frame pair
(a 1280x720 RGB camera frame plus a 64x1875 LiDAR sweep) is pushed through a
CPU re-implementation of the reference client's per-frame behaviour.  Each
frame is one blocking KServe ``ModelInfer`` to the same in-process server,
which runs the models on the GPU when there is one, as the reference's
Triton server did.

The behaviour reproduced per frame pair comes from SURVEY §3.1/§3.2.  It is
re-implemented here, not copied.

2D (``communicator/ros_inference.py:117-175``):

1. Stretch resize to 640x640.  ``torch.nn.functional.interpolate`` on the
   CPU stands in for ``cv2.resize``; both are native bilinear.
2. HWC→CHW, fp32, /255, add a batch dim (``yolov5_preprocess.py:20-24``).
3. Clear and refill the reusable protobuf request with ``tobytes()``, then a
   blocking ModelInfer (``ros_inference.py:143-147``).
4. Decode the response with one ``struct.unpack_from`` per element into an
   object array (``base_postprocess.py:15-25``).
5. Filter candidates on that object array: ``obj > conf``, ``cls *= obj``,
   best class, threshold (``yolov5_postprocess.py:41-92``).
6. Class-offset greedy NMS at IoU 0.45 keeping at most 300.  A vectorised
   NumPy greedy NMS stands in for torchvision's C++ NMS.
7. Rescale the boxes and draw them on the frame.

3D (``communicator/ros_inference3d.py:120-213``):

1. ``read_points(skip_nans=True)`` as a Python generator of
   ``struct.unpack_from`` records, built into an array with ``np.array(list(...))``.
2. intensity /= max, z += 1.5.
3. Voxelise.  The vectorised NumPy voxeliser stands in for spconv's C++
   ``VoxelGenerator``.
4. Three ``tobytes`` inputs, then a blocking ModelInfer.
5. Decode each of the 3 outputs with a per-element struct loop.
6. Keep label 2 with score > 0.5 and build a BoundingBoxArray.

Usage: ``python tools/reference_equivalent.py --frames 5 [--device cuda]``.
The tool prints one JSON line with per-stage milliseconds and the FPS of a
camera + LiDAR frame pair.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def struct_decode_float(raw: bytes) -> np.ndarray:
    """Reference-style per-element float decode into an object array."""
    n = len(raw) // 4
    out = np.empty(n, dtype=object)
    for i in range(n):
        out[i] = struct.unpack_from("f", raw, 4 * i)[0]
    return out


def struct_decode_int64(raw: bytes) -> np.ndarray:
    n = len(raw) // 8
    out = np.empty(n, dtype=object)
    for i in range(n):
        out[i] = struct.unpack_from("q", raw, 8 * i)[0]
    return out


def read_points_generator(data: bytes, n: int, step: int, offs, fmt="f"):
    for i in range(n):
        base = i * step
        vals = tuple(struct.unpack_from(fmt, data, base + o)[0] for o in offs)
        if any(v != v for v in vals):  # skip NaNs
            continue
        yield vals


def greedy_nms(boxes, scores, thr, max_det):
    order = np.argsort(-scores, kind="stable")
    x1, y1, x2, y2 = boxes.T
    area = (x2 - x1) * (y2 - y1)
    keep = []
    while order.size and len(keep) < max_det:
        i = order[0]
        keep.append(i)
        r = order[1:]
        w = np.clip(np.minimum(x2[i], x2[r]) - np.maximum(x1[i], x1[r]), 0, None)
        h = np.clip(np.minimum(y2[i], y2[r]) - np.maximum(y1[i], y1[r]), 0, None)
        inter = w * h
        iou = inter / (area[i] + area[r] - inter)
        order = r[iou <= thr]
    return np.asarray(keep, np.int64)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--cam", default="720x1280")
    ap.add_argument("--rings", type=int, default=64)
    ap.add_argument("--columns", type=int, default=1875)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)

    from triton_client_amd.channel.grpc_channel import GRPCInferenceServiceStub
    from triton_client_amd.clients.detector_3d_client import PointpillarPreprocess, voxel_config_from_model
    from triton_client_amd.proto import service_pb2 as pb
    from triton_client_amd.ros import compat, msgs
    from triton_client_amd.server import KServeServer, ModelRepository
    from triton_client_amd.utils.draw import draw_rect
    from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep
    import grpc

    H0, W0 = (int(v) for v in a.cam.split("x"))
    repo = ModelRepository(a.device)
    repo.load("YOLOv5nCOCO")
    repo.load("pointpillar_kitti")
    srv = KServeServer(repo, "127.0.0.1:0").start()
    ch = grpc.insecure_channel(srv.target, options=[("grpc.max_send_message_length", 1 << 30),
                                                     ("grpc.max_receive_message_length", 1 << 30)])
    stub = GRPCInferenceServiceStub(ch)
    cfg3 = stub.ModelConfig(pb.ModelConfigRequest(name="pointpillar_kitti")).config
    pre3 = PointpillarPreprocess(voxel_config_from_model(cfg3), "cpu")
    req2 = pb.ModelInferRequest(model_name="YOLOv5nCOCO")
    inp2 = pb.ModelInferRequest.InferInputTensor(name="images", datatype="FP32", shape=[1, 3, 640, 640])
    req2.outputs.add(name="output")
    spec = LidarSpec(rings=a.rings, azimuth_steps=a.columns, sensor_height=3.23)
    frames = [camera_frame(H0, W0, s) for s in range(a.frames + a.warmup)]
    clouds = []
    for s in range(a.frames + a.warmup):
        pts = lidar_sweep(spec, 500 + s)
        clouds.append(compat.create_cloud_xyzi(np.frombuffer(pts.tobytes(), np.float32).reshape(-1, 4)))

    stages = {}

    def tick(name, t0):
        stages[name] = stages.get(name, 0.0) + time.perf_counter() - t0
        return time.perf_counter()

    def frame_pair(img, cloud):
        # ---------------- 2D
        t = time.perf_counter()
        x = torch.from_numpy(img).permute(2, 0, 1)[None].float()
        x = torch.nn.functional.interpolate(x, size=(640, 640), mode="bilinear", align_corners=False)
        rs = x[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8).numpy()
        t = tick("2d_resize", t)
        arr = rs.transpose(2, 0, 1).astype(np.float32)[None] / 255.0
        t = tick("2d_image_adjust", t)
        req2.ClearField("inputs")
        req2.ClearField("raw_input_contents")
        req2.inputs.extend([inp2])
        req2.raw_input_contents.extend([arr.astype(np.float32).tobytes()])
        resp = stub.ModelInfer(req2)
        t = tick("2d_rpc", t)
        out = struct_decode_float(resp.raw_output_contents[0]).reshape(tuple(resp.outputs[0].shape))
        t = tick("2d_struct_decode", t)
        p = out[0]
        cand = p[p[:, 4] > 0.3]
        cand[:, 5:] *= cand[:, 4:5]
        c = cand.astype(np.float64)
        boxes = np.stack([c[:, 0] - c[:, 2] / 2, c[:, 1] - c[:, 3] / 2, c[:, 0] + c[:, 2] / 2,
                          c[:, 1] + c[:, 3] / 2], 1) if len(c) else np.zeros((0, 4))
        conf = c[:, 5:].max(1) if len(c) else np.zeros((0,))
        j = c[:, 5:].argmax(1) if len(c) else np.zeros((0,), np.int64)
        m = conf > 0.3
        boxes, conf, j = boxes[m], conf[m], j[m]
        keep = greedy_nms(boxes + j[:, None] * 4096.0, conf, 0.45, 300)
        t = tick("2d_filter_nms", t)
        canvas = img.copy()
        for k in keep:
            b = boxes[k]
            draw_rect(canvas, b[0] * W0 / 640, b[1] * H0 / 640, b[2] * W0 / 640, b[3] * H0 / 640, (255, 0, 0), 2)
        compat.numpy_to_imgmsg(canvas, "rgb8")
        t = tick("2d_draw_publish", t)
        # ---------------- 3D
        pts = np.array(list(read_points_generator(cloud.data, cloud.width, cloud.point_step, (0, 4, 8, 12))),
                       np.float32)
        t = tick("3d_read_points", t)
        pts[:, 3] /= max(pts[:, 3].max(), 1e-12)
        pts[:, 2] += 1.5
        d = pre3.filter_pc(pts)
        t = tick("3d_voxelize", t)
        req3 = pb.ModelInferRequest(model_name="pointpillar_kitti")
        for name, dt, v in (("voxels", "FP32", d["voxels"].astype(np.float32)),
                            ("voxel_coords", "INT32", d["voxel_coords"].astype(np.int32)),
                            ("voxel_num_points", "INT32", d["voxel_num_points"].astype(np.int32))):
            req3.inputs.add(name=name, datatype=dt, shape=list(v.shape))
            req3.raw_input_contents.append(v.tobytes())
        resp3 = stub.ModelInfer(req3)
        t = tick("3d_rpc", t)
        bx = struct_decode_float(resp3.raw_output_contents[0]).reshape(-1, 7)
        sc = struct_decode_float(resp3.raw_output_contents[1])
        lb = struct_decode_int64(resp3.raw_output_contents[2])
        t = tick("3d_struct_decode", t)
        idx = [i for i in range(len(lb)) if lb[i] == 2 and sc[i] > 0.5]
        arrm = msgs.BoundingBoxArray()
        for i in idx:
            b = bx[i]
            arrm.boxes.append(msgs.BoundingBox(pose=msgs.Pose(msgs.Point(b[0], b[1], b[2] - 1.5),
                                                              compat.yaw2quaternion(float(b[6]))),
                                               dimensions=msgs.Vector3(b[4], b[3], b[5])))
        tick("3d_boxes_publish", t)

    for i in range(a.warmup):
        frame_pair(frames[i], clouds[i])
    stages.clear()
    t0 = time.perf_counter()
    for i in range(a.warmup, a.warmup + a.frames):
        frame_pair(frames[i], clouds[i])
    el = time.perf_counter() - t0
    srv.stop()
    res = {"metric": "reference-equivalent end-to-end FPS (camera+LiDAR frame pair, batch 1, sync RPC)",
           "fps": round(a.frames / el, 4), "ms_per_frame_pair": round(el / a.frames * 1e3, 1),
           "stages_ms": {k: round(v / a.frames * 1e3, 2) for k, v in stages.items()},
           "server_device": str(repo.get("YOLOv5nCOCO").device), "frames": a.frames,
           "cam": a.cam, "lidar": f"{a.rings}x{a.columns}"}
    line = json.dumps(res)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
