"""Detection accuracy metrics (reference ``communicator/evaluate_inference.py:131-218,400-446``).

Same definitions as the reference evaluator:

* ``match_predictions`` — for one image, mark each prediction correct at each
  of the 10 IoU thresholds 0.5:0.05:0.95 when it overlaps a same-class GT box;
  every GT and every prediction is matched at most once, highest IoU first
  (``evaluate_inference.py:411-425``).
* ``compute_ap`` / ``ap_per_class`` — COCO 101-point AP of each class's PR
  curve at each IoU threshold, and precision / recall / F1 at the confidence
  maximising mean F1; all classes and thresholds in one vectorised pass
  (segmented cumsum / envelope / interpolation, no per-class loop).

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


def _segmented_reverse_cummax(v: np.ndarray, seg: np.ndarray) -> np.ndarray:
    """Running max from the right within each segment of ``v`` (values in
    [0, 1], ``seg`` non-decreasing ints).  One ``maximum.accumulate`` over the
    reversed array: lowering segment s by 2*s puts every segment above all
    segments after it, so the max carried out of a later segment never wins
    in an earlier one."""
    lift = -2.0 * seg
    return np.maximum.accumulate((v + lift)[::-1])[::-1] - lift


def _segmented_interp(x: np.ndarray, xseg: np.ndarray, xp: np.ndarray, fp: np.ndarray, pseg: np.ndarray,
                      span: float) -> np.ndarray:
    """``np.interp`` of every query against its own segment's (xp, fp) in a
    single call: segments are laid side by side on the x axis (offset
    ``span`` * segment id, span > the width of any segment), so the sorted
    concatenation stays sorted and a query never reaches a neighbour's
    points as long as it lies inside its own segment's x range."""
    return np.interp(x + span * xseg, xp + span * pseg, fp)


def compute_ap(recall: np.ndarray, precision: np.ndarray) -> Tuple[float, np.ndarray, np.ndarray]:
    """COCO 101-point AP of one PR curve.  Returns (ap, envelope, recall axis)
    with the (0, 1) / (1, 0) end points included."""
    ap, env, rec = _ap_segments(np.asarray(recall, np.float64)[None], np.asarray(precision, np.float64)[None])
    return float(ap[0]), env[0], rec[0]


_AP_GRID = np.linspace(0.0, 1.0, 101)


def _ap_segments(recall: np.ndarray, precision: np.ndarray):
    """AP of S PR curves at once: recall/precision [S, n] (each row one curve
    over the confidence-sorted predictions).  Every curve gets the end points
    recall 0 -> precision 1 and recall 1 -> precision 0, its precision is
    replaced by the best precision at any higher recall (the envelope), and
    the envelope is sampled on 101 recall points and integrated (trapezoid)."""
    S, n = recall.shape
    rec = np.concatenate([np.zeros((S, 1)), recall, np.ones((S, 1))], 1)
    pre = np.concatenate([np.ones((S, 1)), precision, np.zeros((S, 1))], 1)
    seg = np.repeat(np.arange(S), n + 2)
    env = _segmented_reverse_cummax(pre.ravel(), seg).reshape(S, n + 2)
    g = len(_AP_GRID)
    span = 1.0 + max(1.0, float(rec.max()))  # recall <= 1 when each GT is matched at most once
    samples = _segmented_interp(np.tile(_AP_GRID, S), np.repeat(np.arange(S), g), rec.ravel(), env.ravel(), seg,
                                span=span).reshape(S, g)
    ap = np.trapezoid(samples, _AP_GRID, axis=1)
    return ap, env, rec


def ap_per_class(tp: np.ndarray, conf: np.ndarray, pred_cls: np.ndarray, target_cls: np.ndarray):
    """Per-class PR statistics over a whole run: returns (p, r, ap [nc, n_iou],
    f1, classes) — the metric of the reference's evaluator
    (``communicator/evaluate_inference.py:131-218``, itself YOLOv5's), computed
    for all classes and IoU thresholds at once.

    * Predictions are ordered by class, then by descending confidence; running
      TP / FP counts restart at each class (segmented cumsum).
    * recall = TP / #GT of the class, precision = TP / (TP + FP); AP per
      (class, IoU threshold) from :func:`_ap_segments`.
    * p / r / f1 are read at one confidence threshold shared by all classes:
      each class's precision and recall (IoU 0.5) are interpolated linearly
      over confidence on a 1000-point grid (above the class's top confidence:
      recall 0, precision 1; below its lowest: its last value), and the grid
      point with the best class-mean F1 is taken.
    Classes are those present in the ground truth; a class without
    predictions scores 0."""
    conf = np.asarray(conf, np.float64).reshape(-1)
    tp = np.asarray(tp, np.float64)
    tp = tp.reshape(len(conf), tp.shape[-1] if tp.ndim == 2 else -1) if len(conf) else tp.reshape(0, max(tp.shape[-1:] or [1]))
    pred_cls = np.asarray(pred_cls).reshape(-1)
    target_cls = np.asarray(target_cls).reshape(-1)
    classes = np.unique(target_cls)
    nc, nt = len(classes), tp.shape[1]
    grid = np.linspace(0.0, 1.0, 1000)
    ap = np.zeros((nc, nt))
    p_curve = np.zeros((nc, len(grid)))
    r_curve = np.zeros((nc, len(grid)))
    # class index of each prediction; predictions of classes absent from the GT drop out
    ci = np.searchsorted(classes, pred_cls)
    keep = (ci < nc) & (classes[np.minimum(ci, max(nc - 1, 0))] == pred_cls) if nc else np.zeros(len(conf), bool)
    ci, cf, hits = ci[keep], conf[keep], tp[keep]
    if len(ci):
        order = np.lexsort((-cf, ci))  # by class, then confidence high -> low
        ci, cf, hits = ci[order], cf[order], hits[order]
        n_gt = np.bincount(np.searchsorted(classes, target_cls), minlength=nc).astype(np.float64)
        first = np.r_[0, np.flatnonzero(np.diff(ci)) + 1]  # start of each class run
        count = np.diff(np.r_[first, len(ci)])
        cum_tp = np.cumsum(hits, 0)
        base = np.repeat(np.r_[np.zeros((1, nt)), cum_tp[first[1:] - 1]], count, 0)
        tps = cum_tp - base  # TP among this class's predictions so far
        rank = np.arange(len(ci)) - np.repeat(first, count) + 1.0  # predictions so far
        recall = tps / n_gt[ci][:, None]
        precision = tps / rank[:, None]
        present = ci[first]
        # AP: one curve per (class run, IoU threshold), padded to the longest run
        # by repeating each run's last point (adds no area: same recall, same precision).
        L = int(count.max())
        pos = first[:, None] + np.minimum(np.arange(L)[None], count[:, None] - 1)  # [runs, L]
        R = recall[pos].transpose(0, 2, 1).reshape(-1, L)
        P = precision[pos].transpose(0, 2, 1).reshape(-1, L)
        ap[present] = _ap_segments(R, P)[0].reshape(len(present), nt)
        # p / r at each grid confidence, per class run, linear in confidence
        runs = len(present)
        q = np.tile(-grid, runs)
        qseg = np.repeat(np.arange(runs), len(grid))
        pseg = np.repeat(np.arange(runs), count)
        r_all = _segmented_interp(q, qseg, -cf, recall[:, 0], pseg, span=4.0).reshape(runs, -1)
        p_all = _segmented_interp(q, qseg, -cf, precision[:, 0], pseg, span=4.0).reshape(runs, -1)
        top = cf[first][:, None]
        low = cf[first + count - 1][:, None]
        above, below = grid[None] > top, grid[None] < low
        r_all = np.where(above, 0.0, np.where(below, recall[first + count - 1, 0][:, None], r_all))
        p_all = np.where(above, 1.0, np.where(below, precision[first + count - 1, 0][:, None], p_all))
        r_curve[present], p_curve[present] = r_all, p_all
    f1 = 2 * p_curve * r_curve / (p_curve + r_curve + 1e-16)
    k = int(np.argmax(f1.mean(0))) if nc else 0
    return p_curve[:, k], r_curve[:, k], ap, f1[:, k], classes.astype(np.int32)


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
