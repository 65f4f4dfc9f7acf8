"""Detection metrics (utils/evaluation.py) against hand-computed values."""
import numpy as np

from triton_client_amd.utils.evaluation import (DetectionEvaluator, ap_per_class, box_iou, compute_ap,
                                                match_predictions)


def test_box_iou_basic():
    a = np.array([[0, 0, 10, 10]], float)
    b = np.array([[0, 0, 10, 10], [5, 5, 15, 15], [20, 20, 30, 30]], float)
    np.testing.assert_allclose(box_iou(a, b)[0], [1.0, 25 / 175, 0.0])


# The reference's AP (YOLOv5 definition, evaluate_inference.py:131-156) appends a
# (recall 1, precision 0) sentinel that the 101st interpolation sample hits, so a
# perfect detector scores 0.995 — kept for parity.
PERFECT = 0.995


def test_compute_ap_perfect_and_half():
    assert abs(compute_ap(np.array([1.0]), np.array([1.0]))[0] - PERFECT) < 1e-9
    # precision 1 up to recall 0.5, then linear to the (1, 0) sentinel: 0.5 + 0.25
    ap = compute_ap(np.array([0.5]), np.array([1.0]))[0]
    assert abs(ap - 0.75) < 1e-9


def test_match_predictions_unique_and_thresholds():
    gt = np.array([[0, 0, 10, 10, 1, 0], [20, 20, 30, 30, 1, 1]], float)
    pred = np.array([[0, 0, 10, 10, 0.9, 0],       # exact → correct at all thresholds
                     [0, 0, 10, 9, 0.8, 0],        # duplicate on the same GT → not matched
                     [20, 20, 30, 31, 0.7, 1],     # IoU 10/11 → correct up to 0.9
                     [20, 20, 30, 30, 0.6, 0]],    # wrong class
                    float)
    c = match_predictions(gt, pred)
    assert c[0].all()
    assert not c[1].any()
    assert c[2, :9].all() and not c[2, 9]
    assert not c[3].any()


def test_ap_per_class_perfect():
    tp = np.ones((4, 10), bool)
    p, r, ap, f1, cls = ap_per_class(tp, np.array([0.9, 0.8, 0.7, 0.6]), np.array([0, 0, 1, 1]), np.array([0, 0, 1, 1]))
    np.testing.assert_allclose(ap, PERFECT, atol=1e-6)
    np.testing.assert_allclose(p, 1.0, atol=1e-6)
    np.testing.assert_allclose(r, 1.0, atol=1e-6)
    assert list(cls) == [0, 1]


def test_evaluator_joins_by_seq_not_order():
    ev = DetectionEvaluator()
    gts = {s: np.array([[10 * s, 0, 10 * s + 8, 8, 1, s % 2]], float) for s in range(5)}
    for s in (4, 2, 0, 3, 1):  # predictions arrive in a different order than GT
        g = gts[s].copy()
        g[0, 4] = 0.9
        ev.add_prediction(s, g)
    for s in range(5):
        ev.add_ground_truth(s, gts[s])
    ev.add_ground_truth(99, gts[0])  # GT without a prediction is not matched
    sm = ev.summary()
    assert sm.matched_images == 5
    assert abs(sm.map - PERFECT) < 1e-6


def test_ap_hand_computed_pr_curves():
    """One class, 3 GT boxes, four predictions by falling confidence; two IoU
    thresholds with different hits.  Envelopes and the 101-point trapezoid
    worked out by hand:

    * hits T F T T: recall 1/3 1/3 2/3 1, precision 1 .5 .667 .75 -> envelope 1
      up to recall 1/3, .75 after, 0 at the recall-1 sentinel.  Samples
      x = 0..0.33 -> 1, 0.34..0.99 -> .75, 1.0 -> 0:
      AP = 0.33 + (1 + .75)/2*0.01 + .75*0.65 + .75/2*0.01 = 0.83.
    * hits T T F F: recall 1/3 2/3 2/3 2/3, precision 1 1 .667 .5 -> envelope 1
      below recall 2/3, from (2/3, .5) straight down to (1, 0), i.e. 1.5(1-x):
      AP = 0.66 + (1 + 1.5*0.33)/2*0.01 + 1.5*0.33**2/2 = 0.74915.
    A second class without predictions scores 0; a predicted class absent
    from the ground truth is ignored."""
    tp = np.array([[1, 1], [0, 1], [1, 0], [1, 0], [1, 1]], bool)
    conf = np.array([0.9, 0.8, 0.7, 0.6, 0.95])
    pred_cls = np.array([3, 3, 3, 3, 7])  # class 7 is not in the ground truth
    p, r, ap, f1, cls = ap_per_class(tp, conf, pred_cls, np.array([3, 3, 3, 5]))
    assert list(cls) == [3, 5]
    np.testing.assert_allclose(ap[0], [0.83, 0.66 + 0.007475 + 1.5 * 0.33 ** 2 / 2], atol=1e-9)
    np.testing.assert_allclose(ap[1], 0.0)
    # the same curves through compute_ap directly
    assert abs(compute_ap(np.array([1, 1, 2, 3]) / 3, np.array([1, 0.5, 2 / 3, 0.75]))[0] - 0.83) < 1e-9


def test_ap_per_class_operating_point():
    """p / r / f1 at the confidence that maximises mean F1.  One GT; a false
    positive at 0.9, the true positive at 0.5.  Between those confidences
    recall rises linearly 0 -> 1 and precision 0 -> .5, so F1 = (2/3)u < 2/3
    there; at or below 0.5: p = .5, r = 1, F1 = 2/3 (the maximum)."""
    p, r, ap, f1, cls = ap_per_class(np.array([[0], [1]], bool), np.array([0.9, 0.5]), np.array([0, 0]),
                                     np.array([0]))
    np.testing.assert_allclose([p[0], r[0], f1[0]], [0.5, 1.0, 2 / 3], atol=1e-9)
    # recall 1 at precision .5 from the FP first: envelope .5 over (0, 1), 0 at x = 1
    np.testing.assert_allclose(ap[0, 0], 0.5 * 0.99 + 0.5 * 0.5 * 0.01, atol=1e-9)


def test_ap_per_class_classes_are_independent():
    """Scoring two classes together equals scoring each alone (the vectorised
    segmented pass must not leak running sums or envelopes across classes)."""
    rng = np.random.default_rng(3)
    n = 40
    conf = rng.random(n)
    pc = rng.integers(0, 3, n)
    tc = np.repeat(np.arange(3), 12)
    tp = np.zeros((n, 10), bool)
    for c in range(3):  # at most one TP per GT: at most 12 per class and threshold
        idx = np.flatnonzero(pc == c)
        tp[idx[:12]] = rng.random((min(12, len(idx)), 10)) < 0.7
    ap_all = ap_per_class(tp, conf, pc, tc)[2]
    for c in range(3):
        s = pc == c
        np.testing.assert_allclose(ap_all[c], ap_per_class(tp[s], conf[s], pc[s], tc[tc == c])[2][0], atol=1e-12)


def test_merge_nms_hand_computed():
    """Merge-NMS (reference yolov5_postprocess.py:111-117): A and B overlap
    (IoU 90/110 > 0.45), NMS keeps A; merged A = (0.9 A + 0.6 B) / 1.5.  C has
    no partner: dropped under ``redundant``, unchanged without it."""
    from triton_client_amd.ops.yolo import merge_nms

    box = np.array([[0, 0, 10, 10], [1, 0, 11, 10], [50, 50, 60, 60], [2, 0, 12, 10]], np.float32)
    score = np.array([0.9, 0.6, 0.8, 0.7], np.float32)
    cls = np.array([0, 0, 0, 1])  # the class-1 box overlaps A but is another class
    keep = np.array([0, 2, 3])
    mb, k = merge_nms(box, score, cls, keep, 0.45)
    assert list(k) == [0]
    np.testing.assert_allclose(mb[0], [0.4, 0.0, 10.4, 10.0], rtol=1e-6)
    mb, k = merge_nms(box, score, cls, keep, 0.45, redundant=False)
    assert list(k) == [0, 2, 3]
    np.testing.assert_allclose(mb[1], box[2]) and np.testing.assert_allclose(mb[2], box[3])
    mb, k = merge_nms(box, score, cls, np.array([0, 2]), 0.45, agnostic=True)
    np.testing.assert_allclose(mb[0], (0.9 * box[0] + 0.6 * box[1] + 0.7 * box[3]) / 2.2, rtol=1e-6)
