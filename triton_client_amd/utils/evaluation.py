"""Detection accuracy metrics (reference ``communicator/evaluate_inference.py:131-218,400-446``).

Same definitions as the reference evaluator:

* ``match_predictions`` — for one image, mark each prediction correct at each
  of the 10 IoU thresholds 0.5:0.05:0.95 when it overlaps a same-class GT box;
  every GT and every prediction is matched at most once, highest IoU first
  (``evaluate_inference.py:411-425``).
* ``compute_ap`` — precision envelope + 101-point interpolated area (COCO).
* ``ap_per_class`` — per-class PR curves over confidence, AP per IoU
  threshold, precision / recall / F1 at the confidence maximising mean F1.

Differences: predictions and ground truth are joined by
``header.seq`` (the reference zips two lists filled by independent
subscriber threads after a fixed 20 s sleep), and the statistics are
aggregated over the whole run before AP is computed (the reference computed
AP per message on one image's matches).  Everything is vectorised NumPy; the
IoU matrix for large images goes through :func:`..ops.golden.box_iou_np`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

IOU_THRESHOLDS = np.linspace(0.5, 0.95, 10)


def box_iou(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """IoU matrix [len(a), len(b)] of xyxy boxes."""
    a = np.asarray(a, np.float64).reshape(-1, 4)
    b = np.asarray(b, np.float64).reshape(-1, 4)
    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    area_b = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
    inter = np.clip(rb - lt, 0, None).prod(2)
    return inter / np.maximum(area_a[:, None] + area_b[None, :] - inter, 1e-12)


def match_predictions(gt: np.ndarray, pred: np.ndarray, iouv: np.ndarray = IOU_THRESHOLDS) -> np.ndarray:
    """gt [M, >=6] (x1,y1,x2,y2,_,cls), pred [N, 6] (x1,y1,x2,y2,conf,cls) →
    bool correct [N, len(iouv)]."""
    pred = np.asarray(pred, np.float64).reshape(-1, 6)
    gt = np.asarray(gt, np.float64).reshape(-1, gt.shape[-1] if np.ndim(gt) == 2 and len(gt) else 6)
    correct = np.zeros((len(pred), len(iouv)), bool)
    if len(pred) == 0 or len(gt) == 0:
        return correct
    iou = box_iou(gt[:, :4], pred[:, :4])
    li, di = np.nonzero((iou >= iouv[0]) & (gt[:, 5:6] == pred[None, :, 5]))
    if len(li):
        m = np.stack([li, di, iou[li, di]], 1)
        if len(li) > 1:
            m = m[np.argsort(-m[:, 2], kind="stable")]
            m = m[np.unique(m[:, 1], return_index=True)[1]]
            m = m[np.unique(m[:, 0], return_index=True)[1]]
        correct[m[:, 1].astype(np.int64)] = m[:, 2:3] >= iouv[None, :]
    return correct


def compute_ap(recall: np.ndarray, precision: np.ndarray) -> Tuple[float, np.ndarray, np.ndarray]:
    """101-point interpolated AP (COCO).  Returns (ap, envelope, recall axis)."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([1.0], precision, [0.0]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    ap = float(np.trapezoid(np.interp(x, mrec, mpre), x))
    return ap, mpre, mrec


def ap_per_class(tp: np.ndarray, conf: np.ndarray, pred_cls: np.ndarray, target_cls: np.ndarray):
    """Returns (p, r, ap [nc, n_iou], f1, classes) like the reference :158-218."""
    tp = np.asarray(tp).reshape(len(conf), -1)
    i = np.argsort(-np.asarray(conf), kind="stable")
    tp, conf, pred_cls = tp[i], np.asarray(conf)[i], np.asarray(pred_cls)[i]
    classes = np.unique(target_cls)
    nc = classes.shape[0]
    px = np.linspace(0, 1, 1000)
    ap = np.zeros((nc, tp.shape[1]))
    p, r = np.zeros((nc, 1000)), np.zeros((nc, 1000))
    for ci, c in enumerate(classes):
        sel = pred_cls == c
        n_l = int((target_cls == c).sum())
        n_p = int(sel.sum())
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[sel]).cumsum(0)
        tpc = tp[sel].cumsum(0)
        recall = tpc / (n_l + 1e-16)
        r[ci] = np.interp(-px, -conf[sel], recall[:, 0], left=0)
        precision = tpc / (tpc + fpc)
        p[ci] = np.interp(-px, -conf[sel], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j] = compute_ap(recall[:, j], precision[:, j])[0]
    f1 = 2 * p * r / (p + r + 1e-16)
    k = int(f1.mean(0).argmax()) if nc else 0
    return p[:, k], r[:, k], ap, f1[:, k], classes.astype(np.int32)


@dataclass
class EvalSummary:
    precision: np.ndarray
    recall: np.ndarray
    ap: np.ndarray          # [nc, 10]
    f1: np.ndarray
    classes: np.ndarray
    images: int
    matched_images: int

    @property
    def map50(self) -> float:
        return float(self.ap[:, 0].mean()) if len(self.ap) else 0.0

    @property
    def map(self) -> float:
        return float(self.ap.mean()) if self.ap.size else 0.0

    def as_dict(self, names: Optional[Sequence[str]] = None) -> dict:
        per = {}
        for i, c in enumerate(self.classes):
            key = names[c] if names is not None and c < len(names) else str(int(c))
            per[key] = {"p": float(self.precision[i]), "r": float(self.recall[i]), "ap50": float(self.ap[i, 0]),
                        "ap": float(self.ap[i].mean()), "f1": float(self.f1[i])}
        return {"images": self.images, "matched_images": self.matched_images, "map50": self.map50,
                "map50_95": self.map, "per_class": per}


@dataclass
class DetectionEvaluator:
    """Accumulates predictions and ground truth keyed by frame id (seq) —
    either may arrive first, from different threads — and computes AP over
    every frame that has both."""

    iouv: np.ndarray = field(default_factory=lambda: IOU_THRESHOLDS.copy())
    preds: Dict[int, np.ndarray] = field(default_factory=dict)
    gts: Dict[int, np.ndarray] = field(default_factory=dict)

    def add_prediction(self, seq: int, dets: np.ndarray) -> None:
        self.preds[int(seq)] = np.asarray(dets, np.float64).reshape(-1, 6)

    def add_ground_truth(self, seq: int, gt: np.ndarray) -> None:
        self.gts[int(seq)] = np.asarray(gt, np.float64).reshape(-1, 6)

    def matched(self) -> List[int]:
        return sorted(set(self.preds) & set(self.gts))

    def stats(self):
        tp, conf, pc, tc = [], [], [], []
        for s in self.matched():
            p, g = self.preds[s], self.gts[s]
            tp.append(match_predictions(g, p, self.iouv))
            conf.append(p[:, 4])
            pc.append(p[:, 5])
            tc.append(g[:, 5])
        if not tp:
            z = np.zeros((0,))
            return np.zeros((0, len(self.iouv)), bool), z, z, z
        return np.concatenate(tp), np.concatenate(conf), np.concatenate(pc), np.concatenate(tc)

    def summary(self) -> EvalSummary:
        tp, conf, pc, tc = self.stats()
        p, r, ap, f1, cls = ap_per_class(tp, conf, pc, tc)
        return EvalSummary(p, r, ap, f1, cls, len(set(self.preds) | set(self.gts)), len(self.matched()))
