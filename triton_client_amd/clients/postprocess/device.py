"""Response tensors -> the GPU, for the remote client's device postprocess.

The reference decodes every ``ModelInfer`` response on the CPU and runs
``torchvision.ops.nms`` there (``clients/postprocess/yolov5_postprocess.py:28-125``,
called at ``communicator/ros_inference.py:148``).  On a GPU client the
response's raw output bytes are instead gathered by C++ threads (no GIL) into a
page-locked batch slot and moved to the device by one H2D DMA; the filter
(K3, ``tca_yolo_filter_decoded``) and the sort + bitmask NMS (K4) run there and
only the kept rows come back.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...ops.nms import NmsResult


class ResponseUpload:
    """Batches of same-shaped host arrays (views of response bytes) -> one device
    tensor [n, *shape].  Two pinned slots rotate; a slot is rewritten only after
    the H2D that read it has completed."""

    def __init__(self, device, slots: int = 2, threads: int = 8):
        self.device = torch.device(device)
        self.nslots, self.threads = slots, threads
        self._pin: List[Optional[torch.Tensor]] = [None] * slots
        self._ev: List[Optional[torch.cuda.Event]] = [None] * slots
        self._k = 0
        self._lock = threading.Lock()

    def __call__(self, arrays: Sequence[np.ndarray], dtype=np.float32, stream=None) -> torch.Tensor:
        from ...inference.live import gather_copy

        if not arrays:
            raise ValueError("no arrays to upload")
        shape = tuple(arrays[0].shape)
        for a in arrays:
            if tuple(a.shape) != shape or a.dtype != dtype:
                raise ValueError(f"response tensors differ: {tuple(a.shape)} {a.dtype} vs {shape} {np.dtype(dtype)}")
        n, nb = len(arrays), int(np.prod(shape)) * np.dtype(dtype).itemsize
        tdt = torch.from_numpy(np.zeros(1, dtype)).dtype
        with self._lock:
            k = self._k
            self._k = (k + 1) % self.nslots
            if self._ev[k] is not None:
                self._ev[k].synchronize()
            pin = self._pin[k]
            if pin is None or pin.numel() < n * nb:
                pin = self._pin[k] = torch.empty((max(n * nb, 1 << 20),), dtype=torch.uint8).pin_memory()
            gather_copy([pin.data_ptr() + i * nb for i in range(n)], [np.ascontiguousarray(a) for a in arrays],
                        [nb] * n, self.threads)
            s = stream or torch.cuda.current_stream(self.device)
            with torch.cuda.stream(s):
                dev = torch.empty((n * nb,), dtype=torch.uint8, device=self.device)
                dev.copy_(pin[:n * nb], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s)
            self._ev[k] = ev
        return dev.view(tdt).view(n, *shape)


def pack_host_detections(per_image: Sequence[np.ndarray], device, max_out: Optional[int] = None) -> NmsResult:
    """Host detections [n_i, 6] (x1, y1, x2, y2, conf, cls) -> a device NmsResult
    (for families whose server returns final boxes, e.g. Detectron2 FCOS/RetinaNet:
    the boxes still have to reach the frames the GPU annotates)."""
    B = len(per_image)
    K = max_out or max([len(d) for d in per_image] + [1])
    box = np.zeros((B, K, 4), np.float32)
    score = np.zeros((B, K), np.float32)
    cls = np.zeros((B, K), np.int32)
    cnt = np.zeros((B,), np.int32)
    for b, d in enumerate(per_image):
        d = np.asarray(d, np.float32).reshape(-1, 6)[:K]
        k = len(d)
        box[b, :k], score[b, :k], cls[b, :k], cnt[b] = d[:, :4], d[:, 4], d[:, 5].astype(np.int32), k
    dev = torch.device(device)
    return NmsResult(*[torch.from_numpy(a).to(dev, non_blocking=False) for a in (box, score, cls, cnt)])
