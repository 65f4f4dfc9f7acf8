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
