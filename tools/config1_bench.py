#!/usr/bin/env python3
"""BASELINE config 1: YOLOv5n 640x640, single JPEG per request over gRPC to a
localhost CPU-only server (plumbing, no GPU).

The reference's camera node (``communicator/ros_inference.py:117-175``) takes
one ``CompressedImage``, decodes it (``cv2.imdecode``), resizes to 640x640,
sends one blocking ModelInfer to Triton and runs NMS on the reply.  Config 1
is that loop against a CPU-only Triton on the same host.  This tool times it
end to end with this framework on a GPU-less host:

* client: JPEG -> RGB (libjpeg via PIL; ``--decoder native`` uses the C++
  entropy decoder + the NumPy pixel stage instead), CPU letterbox /
  normalise, raw KServe request encoded by the C++ codec, blocking RPC,
  CPU decode / filter / NMS (``inference/engines.py`` RemoteDetector2D,
  ``device="cpu"``, ``mode="sync"``);
* server: ``KServeServer`` with ``ModelRepository("cpu")`` — YOLOv5n fp32 on
  the host CPU through PyTorch.

Prints one JSON line: frames/s and mean per-stage milliseconds.
    python tools/config1_bench.py --frames 50 [--threads 8]
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _ReferenceClient:
    """The reference camera node's per-frame 2D work after decode
    (``communicator/ros_inference.py:132-175``), via tools/reference_equivalent.py's helpers."""

    def __init__(self, target, W0, H0):
        import grpc

        from triton_client_amd.channel.grpc_channel import GRPCInferenceServiceStub
        from triton_client_amd.proto import service_pb2 as pb

        self.pb, self.W0, self.H0 = pb, W0, H0
        self.ch = grpc.insecure_channel(target, options=[("grpc.max_send_message_length", 1 << 30),
                                                         ("grpc.max_receive_message_length", 1 << 30)])
        self.stub = GRPCInferenceServiceStub(self.ch)
        self.req = pb.ModelInferRequest(model_name="YOLOv5nCOCO")
        self.inp = pb.ModelInferRequest.InferInputTensor(name="images", datatype="FP32", shape=[1, 3, 640, 640])
        self.req.outputs.add(name="output")

    def detect(self, frames):
        import torch

        from tools.reference_equivalent import greedy_nms, struct_decode_float

        img = frames[0]
        x = torch.from_numpy(img).permute(2, 0, 1)[None].float()
        x = torch.nn.functional.interpolate(x, size=(640, 640), mode="bilinear", align_corners=False)
        rs = x[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8).numpy()
        arr = rs.transpose(2, 0, 1).astype(np.float32)[None] / 255.0
        self.req.ClearField("inputs")
        self.req.ClearField("raw_input_contents")
        self.req.inputs.extend([self.inp])
        self.req.raw_input_contents.extend([arr.tobytes()])
        resp = self.stub.ModelInfer(self.req)
        out = struct_decode_float(resp.raw_output_contents[0]).reshape(tuple(resp.outputs[0].shape))
        p = out[0]
        cand = p[p[:, 4] > 0.3]
        cand[:, 5:] *= cand[:, 4:5]
        c = cand.astype(np.float64)
        if not len(c):
            return [np.zeros((0, 6))]
        boxes = np.stack([c[:, 0] - c[:, 2] / 2, c[:, 1] - c[:, 3] / 2, c[:, 0] + c[:, 2] / 2,
                          c[:, 1] + c[:, 3] / 2], 1)
        conf, j = c[:, 5:].max(1), c[:, 5:].argmax(1)
        m = conf > 0.3
        keep = greedy_nms(boxes[m] + j[m][:, None] * 4096.0, conf[m], 0.45, 300)
        return [np.concatenate([boxes[m][keep], conf[m][keep, None], j[m][keep, None]], 1)]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cam", default="720x1280")
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--threads", type=int, default=0, help="torch CPU threads for the server model (0: default)")
    ap.add_argument("--decoder", choices=["pil", "native"], default="pil")
    ap.add_argument("--protocol", choices=["framework", "reference"], default="framework",
                    help="reference: the reference client's per-frame 2D path against the same server (PIL decode "
                         "standing in for cv2.imdecode, stretch resize, tobytes request, per-element struct decode, "
                         "NumPy NMS; tools/reference_equivalent.py)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)

    import torch
    from PIL import Image

    from triton_client_amd.channel.grpc_channel import GRPCChannel
    from triton_client_amd.clients import Yolov5client
    from triton_client_amd.inference.engines import RemoteDetector2D
    from triton_client_amd.ops import jpeg as J
    from triton_client_amd.server import KServeServer, ModelRepository
    from triton_client_amd.utils.synthetic import camera_frame

    if a.threads:
        torch.set_num_threads(a.threads)
    H0, W0 = (int(v) for v in a.cam.split("x"))
    jpegs = []
    for s in range(8):
        buf = io.BytesIO()
        Image.fromarray(camera_frame(H0, W0, s)).save(buf, format="JPEG", quality=a.quality)
        jpegs.append(buf.getvalue())

    def decode(data):
        if a.decoder == "pil":
            return J.decode_pil(data)
        c, q, g = J.decode_coefficients(data)
        return J.reconstruct_numpy(c, q, g)

    repo = ModelRepository("cpu")
    repo.load("YOLOv5nCOCO")
    srv = KServeServer(repo, "127.0.0.1:0", max_workers=2).start()
    flags = SimpleNamespace(model_name="YOLOv5nCOCO", model_version="", batch_size=1, verbose=False)
    ch = GRPCChannel({"grpc_channel": srv.target}, flags)
    if a.protocol == "reference":
        det = _ReferenceClient(srv.target, W0, H0)
    else:
        det = RemoteDetector2D(ch, Yolov5client(), letterbox=True, conf_thres=0.3, mode="sync", wire="raw",
                               device="cpu")
    t_dec, t_det, ndet = [], [], []
    for i in range(a.warmup + a.frames):
        t0 = time.perf_counter()
        rgb = decode(jpegs[i % len(jpegs)])
        t1 = time.perf_counter()
        out = det.detect([rgb])
        t2 = time.perf_counter()
        if i >= a.warmup:
            t_dec.append(t1 - t0)
            t_det.append(t2 - t1)
            ndet.append(len(out[0]))
    srv.stop()
    st = repo.get("YOLOv5nCOCO").stats
    server_ms = st.compute_ns / max(1, st.inference_count) / 1e6
    total = float(np.sum(t_dec) + np.sum(t_det))
    line = {"metric": "config 1: YOLOv5n-640 single JPEG over gRPC to localhost CPU-only server",
            "value": round(a.frames / total, 2), "unit": "frames/s", "frames": a.frames,
            "ms_per_frame": round(1e3 * total / a.frames, 2),
            "stages_ms": {"jpeg_decode": round(1e3 * float(np.mean(t_dec)), 2),
                          "client_pre_rpc_post": round(1e3 * float(np.mean(t_det)), 2),
                          "server_compute": round(server_ms, 2)},
            "protocol": a.protocol, "decoder": a.decoder, "jpeg_bytes": int(np.mean([len(j) for j in jpegs])),
            "torch_threads": torch.get_num_threads(), "avg_dets": float(np.mean(ndet)),
            "device": "cpu", "model_init": "random (seeded), head prior calibrated on synthetic frames"}
    print(json.dumps(line), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(line) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
