"""YOLOv4 (CSPDarknet53 + SPP + PANet, 3 YOLO heads), the model behind the
reference's ``examples/YOLOv4/config.pbtxt`` (input ``input`` [3, 512, 512];
outputs ``confs`` [1, 16128, 80], ``boxes`` [1, 16128, 1, 4]).

* Decode: ``tools/yolo_layer.py:148-288`` (``yolo_forward_dynamic``).  Per
  anchor, x = (sigmoid(tx)·sxy − ½(sxy−1) + gx)/W and w = exp(tw)·(anchor/stride)/W,
  giving normalised x1y1x2y2.  conf = sigmoid(cls)·sigmoid(obj).  Rows are
  anchor-major (a, y, x) per level, levels at strides 8 / 16 / 32.  On the GPU
  this is HIP kernel K5 (``csrc/kernels/yolo.hip``).
* Post-processing: ``tools/utils.py:166-233``.  max / argmax over classes,
  conf > 0.4 (``utils/postprocess.py:205``), greedy NMS 0.6 per class.

The network is described once as a darknet-style layer graph
(:data:`YOLOV4_SPEC`: conv / route / add / maxpool / upsample).
:class:`YOLOv4` evaluates it as a PyTorch module (the CPU reference).
:class:`~.fast.FastGraph` runs the same graph on the fused NHWC convs, with
every route (concat) written in place.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .common import ConvBNAct, kaiming_init

ANCHORS = (12, 16, 19, 36, 40, 28, 36, 75, 76, 55, 72, 146, 142, 110, 192, 243, 459, 401)  # tools/utils.py:168
MASKS = ((0, 1, 2), (3, 4, 5), (6, 7, 8))
STRIDES = (8, 16, 32)


def _spec(nc: int = 80):
    L: List[Tuple[str, str, dict]] = []

    def conv(n, src, c, k, s=1, act="mish", bn=True):
        L.append((n, "conv", dict(src=src, c=c, k=k, s=s, act=act, bn=bn)))

    def route(n, srcs):
        L.append((n, "route", dict(srcs=list(srcs))))

    def add(n, a, b):
        L.append((n, "add", dict(a=a, b=b)))

    # DownSample1
    conv("d1c1", "input", 32, 3)
    conv("d1c2", "d1c1", 64, 3, 2)
    conv("d1c3", "d1c2", 64, 1)
    conv("d1c4", "d1c2", 64, 1)
    conv("d1c5", "d1c4", 32, 1)
    conv("d1c6", "d1c5", 64, 3)
    add("d1a", "d1c6", "d1c4")
    conv("d1c7", "d1a", 64, 1)
    route("d1r", ["d1c7", "d1c3"])
    conv("d1c8", "d1r", 64, 1)
    prev = "d1c8"
    for i, (c, n) in enumerate(((64, 2), (128, 8), (256, 8), (512, 4)), start=2):
        p = f"d{i}"
        conv(f"{p}c1", prev, 2 * c, 3, 2)
        conv(f"{p}c2", f"{p}c1", c, 1)
        conv(f"{p}c3", f"{p}c1", c, 1)
        x = f"{p}c3"
        for j in range(n):
            conv(f"{p}r{j}a", x, c, 1)
            conv(f"{p}r{j}b", f"{p}r{j}a", c, 3)
            add(f"{p}r{j}", f"{p}r{j}b", x)
            x = f"{p}r{j}"
        conv(f"{p}c4", x, c, 1)
        route(f"{p}r", [f"{p}c4", f"{p}c2"])
        conv(f"{p}c5", f"{p}r", 2 * c, 1)
        prev = f"{p}c5"
    # Neck (leaky)
    lk = "leaky"
    conv("n1", "d5c5", 512, 1, act=lk)
    conv("n2", "n1", 1024, 3, act=lk)
    conv("n3", "n2", 512, 1, act=lk)
    L.append(("mp5", "maxpool", dict(src="n3", k=5)))
    L.append(("mp9", "maxpool", dict(src="n3", k=9)))
    L.append(("mp13", "maxpool", dict(src="n3", k=13)))
    route("spp", ["mp13", "mp9", "mp5", "n3"])
    conv("n4", "spp", 512, 1, act=lk)
    conv("n5", "n4", 1024, 3, act=lk)
    conv("n6", "n5", 512, 1, act=lk)
    conv("n7", "n6", 256, 1, act=lk)
    L.append(("n7u", "upsample", dict(src="n7")))
    conv("n8", "d4c5", 256, 1, act=lk)
    route("n8r", ["n8", "n7u"])
    conv("n9", "n8r", 256, 1, act=lk)
    conv("n10", "n9", 512, 3, act=lk)
    conv("n11", "n10", 256, 1, act=lk)
    conv("n12", "n11", 512, 3, act=lk)
    conv("n13", "n12", 256, 1, act=lk)
    conv("n14", "n13", 128, 1, act=lk)
    L.append(("n14u", "upsample", dict(src="n14")))
    conv("n15", "d3c5", 128, 1, act=lk)
    route("n15r", ["n15", "n14u"])
    conv("n16", "n15r", 128, 1, act=lk)
    conv("n17", "n16", 256, 3, act=lk)
    conv("n18", "n17", 128, 1, act=lk)
    conv("n19", "n18", 256, 3, act=lk)
    conv("n20", "n19", 128, 1, act=lk)
    # Head
    no = 3 * (5 + nc)
    conv("h1", "n20", 256, 3, act=lk)
    conv("out0", "h1", no, 1, act="linear", bn=False)
    conv("h3", "n20", 256, 3, 2, act=lk)
    route("h3r", ["h3", "n13"])
    conv("h4", "h3r", 256, 1, act=lk)
    conv("h5", "h4", 512, 3, act=lk)
    conv("h6", "h5", 256, 1, act=lk)
    conv("h7", "h6", 512, 3, act=lk)
    conv("h8", "h7", 256, 1, act=lk)
    conv("h9", "h8", 512, 3, act=lk)
    conv("out1", "h9", no, 1, act="linear", bn=False)
    conv("h11", "h8", 512, 3, 2, act=lk)
    route("h11r", ["h11", "n6"])
    conv("h12", "h11r", 512, 1, act=lk)
    conv("h13", "h12", 1024, 3, act=lk)
    conv("h14", "h13", 512, 1, act=lk)
    conv("h15", "h14", 1024, 3, act=lk)
    conv("h16", "h15", 512, 1, act=lk)
    conv("h17", "h16", 1024, 3, act=lk)
    conv("out2", "h17", no, 1, act="linear", bn=False)
    return L


YOLOV4_OUTPUTS = ("out0", "out1", "out2")


@dataclass
class YoloV4Config:
    nc: int = 80
    img: Tuple[int, int] = (512, 512)
    conf_thres: float = 0.4   # utils/postprocess.py:205
    nms_thres: float = 0.6    # utils/postprocess.py:206
    scale_x_y: float = 1.0    # tools/yolo_layer.py:311

    def num_predictions(self) -> int:
        return sum(3 * (self.img[0] // s) * (self.img[1] // s) for s in STRIDES)


class YOLOv4(nn.Module):
    def __init__(self, cfg: Optional[YoloV4Config] = None):
        super().__init__()
        self.cfg = cfg or YoloV4Config()
        self.spec = _spec(self.cfg.nc)
        self.layers = nn.ModuleDict()
        ch = {"input": 3}
        for name, op, a in self.spec:
            if op == "conv":
                self.layers[name] = ConvBNAct(ch[a["src"]], a["c"], a["k"], a["s"], a["k"] // 2, act=a["act"],
                                              bn=a["bn"], bias=not a["bn"])
                ch[name] = a["c"]
            elif op == "route":
                ch[name] = sum(ch[s] for s in a["srcs"])
            elif op == "add":
                ch[name] = ch[a["a"]]
            else:
                ch[name] = ch[a["src"]]
        self.channels = ch
        kaiming_init(self)

    def forward(self, x) -> List[torch.Tensor]:
        v: Dict[str, torch.Tensor] = {"input": x}
        for name, op, a in self.spec:
            if op == "conv":
                v[name] = self.layers[name](v[a["src"]])
            elif op == "route":
                v[name] = torch.cat([v[s] for s in a["srcs"]], 1)
            elif op == "add":
                v[name] = v[a["a"]] + v[a["b"]]
            elif op == "maxpool":
                v[name] = F.max_pool2d(v[a["src"]], a["k"], 1, a["k"] // 2)
            elif op == "upsample":
                v[name] = F.interpolate(v[a["src"]], scale_factor=2.0, mode="nearest")
        return [v[n] for n in YOLOV4_OUTPUTS]


def build_yolov4(nc: int = 80, img=512, seed: int = 0) -> YOLOv4:
    torch.manual_seed(seed)
    img = (img, img) if isinstance(img, int) else tuple(img)
    return YOLOv4(YoloV4Config(nc=nc, img=img))


def decode_reference(heads: Sequence[torch.Tensor], nc: int, scale_x_y: float = 1.0):
    """fp32 ``yolo_forward_dynamic`` over the three heads → (boxes [B, N, 1, 4]
    normalised x1y1x2y2, confs [B, N, nc])."""
    boxes_all, confs_all = [], []
    for lvl, out in enumerate(heads):
        out = out.float()
        B, _, H, W = out.shape
        s = STRIDES[lvl]
        o = out.view(B, 3, 5 + nc, H, W)
        anc = torch.tensor([ANCHORS[2 * m: 2 * m + 2] for m in MASKS[lvl]], dtype=torch.float32) / s  # [3, 2]
        gy, gx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32),
                                indexing="ij")
        bx = (torch.sigmoid(o[:, :, 0]) * scale_x_y - 0.5 * (scale_x_y - 1) + gx) / W
        by = (torch.sigmoid(o[:, :, 1]) * scale_x_y - 0.5 * (scale_x_y - 1) + gy) / H
        bw = torch.exp(o[:, :, 2]) * anc[:, 0].view(1, 3, 1, 1) / W
        bh = torch.exp(o[:, :, 3]) * anc[:, 1].view(1, 3, 1, 1) / H
        x1, y1 = bx - bw * 0.5, by - bh * 0.5
        boxes = torch.stack([x1, y1, x1 + bw, y1 + bh], -1).reshape(B, 3 * H * W, 1, 4)
        conf = torch.sigmoid(o[:, :, 5:]) * torch.sigmoid(o[:, :, 4:5])  # [B, 3, nc, H, W]
        confs = conf.permute(0, 1, 3, 4, 2).reshape(B, 3 * H * W, nc)
        boxes_all.append(boxes)
        confs_all.append(confs)
    return torch.cat(boxes_all, 1), torch.cat(confs_all, 1)


def post_processing(boxes: np.ndarray, confs: np.ndarray, conf_thresh: float = 0.4, nms_thresh: float = 0.6):
    """``tools/utils.py:166-233`` semantics → per image [n, 6] (x1, y1, x2, y2
    normalised, conf, cls), classes in ascending order, per-class greedy NMS."""
    from ..clients.postprocess.base_postprocess import Postprocess

    box_array = np.asarray(boxes)[:, :, 0]
    confs = np.asarray(confs)
    max_conf, max_id = confs.max(2), confs.argmax(2)
    out = []
    for i in range(box_array.shape[0]):
        keep_i = max_conf[i] > conf_thresh
        b, c, k = box_array[i, keep_i], max_conf[i, keep_i], max_id[i, keep_i]
        rows = []
        for j in range(confs.shape[2]):
            sel = k == j
            if not sel.any():
                continue
            keep = Postprocess.nms_cpu(b[sel], c[sel], nms_thresh)
            for q in keep:
                rows.append([*b[sel][q], c[sel][q], j])
        out.append(np.asarray(rows, np.float32).reshape(-1, 6))
    return out
