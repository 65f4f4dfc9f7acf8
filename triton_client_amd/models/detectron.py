"""Detectron2 one-stage detectors: RetinaNet / FCOS on ResNet-50 + FPN.

The reference serves these as TorchScript through Triton's libtorch backend
(``examples/RetinaNet_detectron/config.pbtxt``; FCOS / RetinaNet clients
``clients/detectron_client.py``, ``clients/postprocess/detectron_postprocess.py:26-38``).
The networks follow Detectron2's defaults (``config/detectron.py``):

* ResNet-50.  FrozenBN is folded.  The stride is in the first 1×1 of each
  bottleneck (MSRA).  Each block's output is relu(main + shortcut), run with
  the conv epilogue's post-residual activation.
* FPN with P3–P5 from res3–res5 (lateral 1×1, nearest 2× top-down add, 3×3
  output).  RetinaNet takes P6/P7 from res5 (LastLevelP6P7 on C5); FCOS takes
  them from P5.
* RetinaNet head: 4×(conv3×3+ReLU) towers, cls A·C, box A·4, shared over
  levels.  FCOS head: 4×(conv3×3+GN(32)+ReLU) towers, cls C, ltrb 4,
  centerness 1.
* Decode: sigmoid(cls) (FCOS: sqrt(cls·ctr)) > threshold, per-level top 1000,
  box decode, class-aware NMS, keep 100.  On the GPU this is K-R / K-F plus a
  segment merge and K4.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config.detectron import DetectronConfig
from .common import ConvBNAct, kaiming_init


class Bottleneck(nn.Module):
    def __init__(self, c_in: int, c_b: int, c_out: int, stride: int, stride_in_1x1: bool = True):
        super().__init__()
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = ConvBNAct(c_in, c_b, 1, s1, 0, act="relu")
        self.conv2 = ConvBNAct(c_b, c_b, 3, s3, 1, act="relu")
        self.conv3 = ConvBNAct(c_b, c_out, 1, 1, 0, act="none")
        self.shortcut = ConvBNAct(c_in, c_out, 1, stride, 0, act="none") if (c_in != c_out or stride != 1) else None

    def forward(self, x):
        sc = self.shortcut(x) if self.shortcut is not None else x
        return F.relu(self.conv3(self.conv2(self.conv1(x))) + sc)


class ResNet(nn.Module):
    def __init__(self, blocks=(3, 4, 6, 3), stride_in_1x1: bool = True):
        super().__init__()
        self.stem = ConvBNAct(3, 64, 7, 2, 3, act="relu")
        self.stages = nn.ModuleList()
        c_in, c_b = 64, 64
        for i, n in enumerate(blocks):
            c_out = c_b * 4
            layers = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                layers.append(Bottleneck(c_in, c_b, c_out, stride, stride_in_1x1))
                c_in = c_out
            self.stages.append(nn.Sequential(*layers))
            c_b *= 2
        self.out_channels = [256, 512, 1024, 2048]

    def forward(self, x) -> List[torch.Tensor]:
        x = F.max_pool2d(self.stem(x), 3, 2, 1)
        outs = []
        for st in self.stages:
            x = st(x)
            outs.append(x)
        return outs  # res2..res5


class FPN(nn.Module):
    def __init__(self, in_channels=(512, 1024, 2048), out: int = 256, p6p7_from_c5: bool = True):
        super().__init__()
        self.lateral = nn.ModuleList(ConvBNAct(c, out, 1, 1, 0, act="none", bn=False, bias=True) for c in in_channels)
        self.output = nn.ModuleList(ConvBNAct(out, out, 3, 1, 1, act="none", bn=False, bias=True) for _ in in_channels)
        self.p6p7_from_c5 = p6p7_from_c5
        self.p6 = ConvBNAct(in_channels[-1] if p6p7_from_c5 else out, out, 3, 2, 1, act="none", bn=False, bias=True)
        self.p7 = ConvBNAct(out, out, 3, 2, 1, act="none", bn=False, bias=True)

    def forward(self, c3, c4, c5) -> List[torch.Tensor]:
        cs = [c3, c4, c5]
        prev = self.lateral[2](c5)
        outs = [self.output[2](prev)]
        for i in (1, 0):
            prev = self.lateral[i](cs[i]) + F.interpolate(prev, scale_factor=2.0, mode="nearest")
            outs.insert(0, self.output[i](prev))
        p6 = self.p6(c5 if self.p6p7_from_c5 else outs[-1])
        p7 = self.p7(F.relu(p6))
        return outs + [p6, p7]


class RetinaNetHead(nn.Module):
    def __init__(self, c: int, num_anchors: int, num_classes: int, n_convs: int = 4):
        super().__init__()
        self.cls_subnet = nn.ModuleList(ConvBNAct(c, c, 3, 1, 1, act="relu", bn=False, bias=True)
                                        for _ in range(n_convs))
        self.bbox_subnet = nn.ModuleList(ConvBNAct(c, c, 3, 1, 1, act="relu", bn=False, bias=True)
                                         for _ in range(n_convs))
        self.cls_score = nn.Conv2d(c, num_anchors * num_classes, 3, 1, 1)
        self.bbox_pred = nn.Conv2d(c, num_anchors * 4, 3, 1, 1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, std=0.01)
                nn.init.zeros_(m.bias)
        nn.init.constant_(self.cls_score.bias, -math.log((1 - 0.01) / 0.01))

    def forward(self, feats) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        out = []
        for f in feats:
            c, b = f, f
            for m in self.cls_subnet:
                c = m(c)
            for m in self.bbox_subnet:
                b = m(b)
            out.append((self.cls_score(c), self.bbox_pred(b)))
        return out


class FCOSHead(nn.Module):
    def __init__(self, c: int, num_classes: int, n_convs: int = 4, groups: int = 32):
        super().__init__()
        def tower():
            mods = []
            for _ in range(n_convs):
                mods += [nn.Conv2d(c, c, 3, 1, 1), nn.GroupNorm(groups, c), nn.ReLU()]
            return nn.Sequential(*mods)
        self.cls_subnet, self.bbox_subnet = tower(), tower()
        self.cls_score = nn.Conv2d(c, num_classes, 3, 1, 1)
        self.bbox_pred = nn.Conv2d(c, 4, 3, 1, 1)
        self.ctrness = nn.Conv2d(c, 1, 3, 1, 1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, std=0.01)
                nn.init.zeros_(m.bias)
        nn.init.constant_(self.cls_score.bias, -math.log((1 - 0.01) / 0.01))

    def forward(self, feats):
        out = []
        for f in feats:
            c, b = self.cls_subnet(f), self.bbox_subnet(f)
            out.append((self.cls_score(c), self.bbox_pred(b), self.ctrness(b)))
        return out


class DetectronDetector(nn.Module):
    """forward(x: [B, 3, H, W] RGB 0..255) → per-level raw head outputs."""

    def __init__(self, cfg: DetectronConfig | None = None):
        super().__init__()
        cfg = cfg or DetectronConfig()
        self.cfg = cfg
        self.backbone = ResNet(cfg.depth_blocks, cfg.stride_in_1x1)
        self.fpn = FPN((512, 1024, 2048), cfg.fpn_channels, p6p7_from_c5=cfg.arch == "retinanet")
        if cfg.arch == "retinanet":
            self.head = RetinaNetHead(cfg.fpn_channels, cfg.num_anchors, cfg.num_classes, cfg.head_convs)
        else:
            self.head = FCOSHead(cfg.fpn_channels, cfg.num_classes, cfg.head_convs)
        kaiming_init(self.backbone)
        kaiming_init(self.fpn)
        self.register_buffer("mean", torch.tensor(cfg.pixel_mean).view(1, 3, 1, 1))
        self.register_buffer("std", torch.tensor(cfg.pixel_std).view(1, 3, 1, 1))

    def features(self, x):
        x = (x - self.mean.to(x.dtype)) / self.std.to(x.dtype)
        _, c3, c4, c5 = self.backbone(x)
        return self.fpn(c3, c4, c5)

    def forward(self, x):
        return self.head(self.features(x))


def build_detectron(cfg: DetectronConfig | None = None, seed: int = 0) -> DetectronDetector:
    torch.manual_seed(seed)
    return DetectronDetector(cfg)


# ----------------------------------------------------------------------------- reference decode
def _nms_np(boxes, scores, thr):
    order = np.argsort(-scores, kind="stable")
    keep = []
    x1, y1, x2, y2 = boxes.T
    area = (x2 - x1) * (y2 - y1)
    while order.size:
        i = order[0]
        keep.append(i)
        r = order[1:]
        w = np.clip(np.minimum(x2[i], x2[r]) - np.maximum(x1[i], x1[r]), 0, None)
        h = np.clip(np.minimum(y2[i], y2[r]) - np.maximum(y1[i], y1[r]), 0, None)
        inter = w * h
        union = area[i] + area[r] - inter
        iou = np.divide(inter, union, out=np.zeros_like(inter), where=union > 0)
        order = r[iou <= thr]
    return np.asarray(keep, np.int64)


def decode_reference(outs, cfg: DetectronConfig, image_hw=None):
    """CPU reference of the Detectron2 inference path → per image
    (boxes [n, 4] xyxy in model-input pixels, scores [n], classes [n])."""
    B = outs[0][0].shape[0]
    H_in, W_in = image_hw or cfg.input_hw
    res = []
    for b in range(B):
        boxes_l, scores_l, cls_l, keys_l = [], [], [], []
        for lvl, o in enumerate(outs):
            s = cfg.strides[lvl]
            if cfg.arch == "retinanet":
                cls, box = o[0][b].float(), o[1][b].float()
                A, C = cfg.num_anchors, cfg.num_classes
                _, H, W = cls.shape
                prob = torch.sigmoid(cls.view(A, C, H, W).permute(2, 3, 0, 1).reshape(-1))  # (y, x, a, c)
            else:
                cls, box, ctr = o[0][b].float(), o[1][b].float(), o[2][b].float()
                C = cfg.num_classes
                _, H, W = cls.shape
                prob = torch.sqrt(torch.sigmoid(cls).permute(1, 2, 0) * torch.sigmoid(ctr).permute(1, 2, 0)).reshape(-1)
                A = 1
            keep = torch.nonzero(prob > cfg.score_thresh).flatten()
            if cfg.arch == "fcos":
                # the FCOS threshold applies to sqrt(cls * ctr) in Detectron2 (pred_scores > thresh)
                pass
            p = prob[keep]
            # per-level top-k with index tie-break (smaller flat index first)
            k = min(cfg.topk_per_level, len(keep))
            order = np.lexsort((keep.numpy(), -p.numpy().astype(np.float64)))[:k]
            keep, p = keep[order], p[order]
            c = keep % C
            anc = keep // C  # (y, x, a) flattened
            a = anc % A
            yx = anc // A
            y, x = yx // W, yx % W
            if cfg.arch == "retinanet":
                tab = torch.tensor(cfg.anchor_table(lvl), dtype=torch.float32)
                aw, ah = tab[a, 0], tab[a, 1]
                cx, cy = x.float() * s, y.float() * s
                d = box.view(A, 4, H, W)[a, :, y, x]  # [k, 4]
                dw = d[:, 2].clamp(max=cfg.scale_clamp)
                dh = d[:, 3].clamp(max=cfg.scale_clamp)
                px, py = d[:, 0] * aw + cx, d[:, 1] * ah + cy
                pw, ph = torch.exp(dw) * aw, torch.exp(dh) * ah
                bx = torch.stack([px - pw / 2, py - ph / 2, px + pw / 2, py + ph / 2], 1)
            else:
                cx, cy = (x.float() + 0.5) * s, (y.float() + 0.5) * s
                d = F.relu(box[:, y, x].t()) * s  # l, t, r, b
                bx = torch.stack([cx - d[:, 0], cy - d[:, 1], cx + d[:, 2], cy + d[:, 3]], 1)
            bx[:, 0::2] = bx[:, 0::2].clamp(0, W_in)
            bx[:, 1::2] = bx[:, 1::2].clamp(0, H_in)
            boxes_l.append(bx.numpy())
            scores_l.append(p.numpy())
            cls_l.append(c.numpy())
            keys_l.append(keep.numpy() + lvl * (1 << 26))
        if boxes_l:
            bx, sc, cl = np.concatenate(boxes_l), np.concatenate(scores_l), np.concatenate(cls_l)
            kept = []
            for c in np.unique(cl):
                idx = np.nonzero(cl == c)[0]
                kept.extend(idx[_nms_np(bx[idx].astype(np.float64), sc[idx], cfg.nms_thresh)])
            kept = np.asarray(kept, np.int64)
            kept = kept[np.argsort(-sc[kept], kind="stable")][: cfg.max_detections]
            res.append((bx[kept].astype(np.float32), sc[kept].astype(np.float32), cl[kept].astype(np.int64)))
        else:
            res.append((np.zeros((0, 4), np.float32), np.zeros((0,), np.float32), np.zeros((0,), np.int64)))
    return res
