"""Headless 3D scene rendering (reference visualize_open3d.draw_scenes /
visualize_mayavi.draw_corners3d), checked geometrically."""
import numpy as np

from triton_client_amd.utils.visualize import (boxes_to_corners_3d, draw_scenes, look_at, project,
                                               project_boxes_to_image)


def test_look_at_projection_centres_target():
    Rt = look_at((-10, 0, 5), (20, 0, 0))
    K = np.array([[500, 0, 640], [0, 500, 360], [0, 0, 1.0]])
    uv, z = project(np.array([[20.0, 0, 0], [20.0, 5.0, 0], [20.0, 0, 3.0]]), Rt, K)
    np.testing.assert_allclose(uv[0], [640, 360], atol=1e-6)
    assert uv[1, 0] < 640  # +y (left in the LiDAR frame) projects to the left
    assert uv[2, 1] < 360  # +z projects up
    assert (z > 0).all()


def test_draw_scenes_draws_points_boxes_axes(tmp_path):
    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.uniform([0, -20, -1.7], [40, 20, 1], (4000, 3)), rng.random((4000, 1))], 1)
    boxes = np.array([[15.0, 2.0, -0.8, 4.0, 1.8, 1.6, 0.3], [25.0, -5.0, -0.8, 4.0, 1.8, 1.6, -1.0]])
    img = draw_scenes(pts, gt_boxes=boxes[:1], ref_boxes=boxes, ref_labels=np.array([1, 2]),
                      ref_scores=np.array([0.9, 0.4]), path=str(tmp_path / "s.png"))
    assert img.shape == (720, 1280, 3) and (tmp_path / "s.png").is_file()
    assert (img.sum(-1) > 0).mean() > 0.005  # points landed
    green = (img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 0)
    cyan = (img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 255)
    assert green.sum() > 50 and cyan.sum() > 50  # label 1 and label 2 wireframes
    # score threshold hides the second prediction
    img2 = draw_scenes(pts, ref_boxes=boxes, ref_labels=np.array([1, 2]), ref_scores=np.array([0.9, 0.4]),
                       score_thresh=0.5, draw_origin=False)
    cyan2 = (img2[..., 0] == 0) & (img2[..., 1] == 255) & (img2[..., 2] == 255)
    assert cyan2.sum() == 0


def test_corners_projected_into_camera_image():
    # camera looking down +x of the LiDAR frame: KITTI-like Tr (x_cam = -y, y_cam = -z, z_cam = x)
    Tr = np.array([[0, -1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0.0]])
    P = np.array([[700, 0, 620, 0], [0, 700, 190, 0], [0, 0, 1, 0.0]])
    img = np.zeros((375, 1242, 3), np.uint8)
    box = np.array([[20.0, 0.0, 0.0, 4.0, 2.0, 1.5, 0.0]])
    project_boxes_to_image(img, box, P, Tr)
    ys, xs = np.nonzero(img.sum(-1))
    cor = boxes_to_corners_3d(box)[0]
    u = 700 * (-cor[:, 1]) / cor[:, 0] + 620
    assert abs(xs.min() - u.min()) <= 2 and abs(xs.max() - u.max()) <= 2
